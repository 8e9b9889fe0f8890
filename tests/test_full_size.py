"""Full-size parity at the headline configurations (BASELINE.json configs 4 and 5).

C4: 2^24-vertex Chung-Lu overlay (gamma 2.5, mean degree 16, seed 4), 4096
messages.  C5: the C4 recipe at 2^26 vertices (seed 5) with 1 %/round crashes,
3-miss liveness detection and seed removal (Peer.py:298-313, Seed.py:358-406).

C4: the oracle (oracle/gossip_oracle.c, OpenMP) runs ALL 4096 messages (W = 64,
the bench's configuration: its message table in spread order) on the overlay
the device built, and the engine's
whole run must equal it output for output: per-round counters, the Message-List
of every vertex, digests, per-message coverage and forwards.  The receive /
forward logic restated is Peer.py:175-216, 395-408 plus forward-once
(DESIGN.md §2).

C5: the oracle runs ALL 4096 messages with churn, and two engine runs must
equal it: the run configured exactly as bench.py times it (bench.engine_config:
no exact frontier rows, so the push gathers whole Message-Lists under
liveness) -- per-round counters, the Message-List of every vertex, digests,
coverage and every round's dead-node reports -- and the same run with
track_msg_forwards = 1, whose per-message forwards are compared too.

Both: the whole 4096-message run is also tied to message shards through the
composition of DESIGN.md §6: shards [0,64) [64,512) [512,1024) [1024,2048)
[2048,4096) -- widths 1, 8, 8, 16 and 32 words, i.e. the flat edge-parallel
kernel and the per-receiver kernel -- must add up to the W = 64 run exactly
(per-round new bits / sends / injections, coverage and forwards concatenate,
digests XOR).  Messages never interact, so this composition is an identity of
the semantics, not of the implementation.

The overlay's degree distribution is also checked.
"""
import os
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

STAT_KEYS = ("injected", "lost", "new_bits", "receivers", "sends", "active", "crashed",
             "reports", "removals", "dup_reports")
SHARDS = [(0, 64), (64, 512), (512, 1024), (1024, 2048), (2048, 4096)]


def _threads():
    return int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)


def _log(msg):
    print(f"[{time.strftime('%H:%M:%S')}] {msg}", flush=True)


def _fmix(x):
    x = x ^ (x >> np.uint64(33))
    x = x * np.uint64(0xff51afd7ed558ccd)
    x = x ^ (x >> np.uint64(33))
    x = x * np.uint64(0xc4ceb9fe1a85ec53)
    return x ^ (x >> np.uint64(33))


def report_fingerprint(rep):
    """Order-free fingerprint of a multiset of (dead, reporter, round) reports:
    count, wrapping sum and xor of a 64-bit mix of each report."""
    rep = np.asarray(rep, dtype=np.int64).reshape(-1, 3)
    with np.errstate(over="ignore"):
        key = (rep[:, 0].astype(np.uint64) << np.uint64(32)) | rep[:, 1].astype(np.uint64)
        key = _fmix(key ^ (rep[:, 2].astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15)))
        s = int(np.sum(key, dtype=np.uint64)) if key.size else 0
    x = int(np.bitwise_xor.reduce(key)) if key.size else 0
    return int(rep.shape[0]), s, x


def _run(eng, with_reports=False, report_cap=1 << 24):
    stats, fps = [], []
    last = int(eng.inject_round.max()) if eng.m else 0
    for r in range(254):
        st = eng.round()
        stats.append(st)
        assert st["overflow"] == 0, st
        if with_reports:
            rep, nrep = eng.reports(report_cap)
            assert nrep == len(rep)
            fps.append(report_fingerprint(rep))
        if st["new_bits"] == 0 and r >= last:
            break
    eng.finalize()
    return stats, fps


def _bench_cfg(churn):
    """The engine configuration bench.py times for this workload (C4 / C5)."""
    import bench
    return bench.engine_config(bench.parse(["--workload", "c5" if churn else "c4"]))


def _read_run(eng, churn, want_fwd=True):
    out = dict(dig=eng.digest().copy(), cov=eng.coverage())
    if want_fwd:
        out["fwd"] = eng.forwards()
    return out


def _check_counters(stats, ref):
    assert len(stats) == ref["rounds"]
    for a, b in zip(stats, ref["stats"]):
        for k in STAT_KEYS:
            assert a[k] == b[k], (k, a["round"], a[k], b[k])


def _check_seen(seen, ref_seen, n):
    assert seen.shape == ref_seen.shape
    for lo in range(0, n, 1 << 20):   # blockwise: no multi-GiB temporaries
        assert np.array_equal(seen[lo:lo + (1 << 20)], ref_seen[lo:lo + (1 << 20)]), lo


def _full_size(pkg, oracle, log2n, seed, churn):
    n, m = 1 << log2n, 4096
    bench_cfg = _bench_cfg(churn)
    okw = {}
    if churn:
        bench_cfg["report_capacity"] = 1 << 24   # the reports buffer only: the kernels are unchanged
        okw = dict(churn=True, p_fail=bench_cfg["p_fail"], churn_seed=bench_cfg["churn_seed"])
        assert bench_cfg.get("track_msg_forwards", 0) == 0
    # tracked: the same run with the per-message forwards of every round kept
    # (exact frontier rows); without churn the bench's run computes them itself
    trk_cfg = dict(bench_cfg, track_msg_forwards=1) if churn else bench_cfg
    t0 = time.time()
    whole = pkg.GossipEngine(0, **bench_cfg)
    whole.build_chung_lu(n, 16.0, 2.5, seed)
    _, nnz, _, _ = whole.info()
    chk = whole.check_degree(2.5)
    _log(f"2^{log2n}: built {nnz} arcs in {time.time() - t0:.1f} s; degree check {chk}")
    assert chk["ok"], chk
    g = whole.graph()
    origin = pkg.overlay.random_origins(n, m, seed=seed)
    origin = origin[whole.spread_order(origin, hops=3)]   # the bench's message order

    # the bench's configuration: all 4096 messages, W = 64
    t0 = time.time()
    whole.set_messages(origin)
    whole.reset()
    w_stats, w_fps = _run(whole, with_reports=churn)
    w = _read_run(whole, churn, want_fwd=not churn)
    w_seen = whole.seen()   # 8 GiB at C4, 32 GiB at C5
    whole.close()
    _log(f"bench-configured run: {len(w_stats)} rounds in {time.time() - t0:.1f} s "
         f"(scan modes {[s['scan'] for s in w_stats]}, push {[s['mode'] for s in w_stats]})")
    assert sum(s["injected"] + s["new_bits"] for s in w_stats) == int(w["cov"].sum())
    if not churn:
        assert sum(s["sends"] for s in w_stats) == int(w["fwd"].sum())

    t_stats, t_fps, t = w_stats, w_fps, w
    if churn:   # the same run with exact frontier rows: per-message forwards
        t0 = time.time()
        with pkg.GossipEngine(0, **trk_cfg) as trk:
            trk.load_graph(g)
            trk.set_messages(origin)
            trk.reset()
            t_stats, t_fps = _run(trk, with_reports=True)
            t = _read_run(trk, churn)
        _log(f"tracked run: {len(t_stats)} rounds in {time.time() - t0:.1f} s")
        assert sum(s["sends"] for s in t_stats) == int(t["fwd"].sum())

    # message shards on a second context
    sh = pkg.GossipEngine(0, **trk_cfg)
    sh.load_graph(g)
    parts = []
    for lo, hi in SHARDS:
        t0 = time.time()
        sh.set_message_shard(origin, None, lo, hi)
        sh.reset()
        stats, fps = _run(sh, with_reports=churn and lo == 0)
        part = dict(stats=stats, fps=fps, digest=sh.digest().copy(), cov=sh.coverage(), fwd=sh.forwards(),
                    words=sh.words)
        if lo == 0:
            part["seen"] = sh.seen()
        parts.append(part)
        _log(f"shard [{lo},{hi}) W={sh.words}: {len(stats)} rounds in {time.time() - t0:.1f} s")
    sh.close()

    # the oracle's run of all 4096 messages (with churn at C5)
    t0 = time.time()
    ref = oracle.run(g, origin, nthreads=_threads(), want_first=False, report_cap=1 << 27, **okw)
    _log(f"oracle, all {m} messages: {ref['rounds']} rounds in {time.time() - t0:.1f} s ({_threads()} threads)")
    # the bench-configured run, output for output
    _check_counters(w_stats, ref)
    _check_seen(w_seen, ref["seen"], n)
    del w_seen
    assert np.array_equal(w["dig"], ref["digest"])
    assert np.array_equal(w["cov"], ref["coverage"])
    assert np.array_equal(t["fwd"], ref["forwards"])
    if churn:
        # every round's dead-node reports (a fingerprinted multiset), both runs
        assert ref["n_reports"] <= 1 << 27
        rep = ref["reports"]
        ref_fps = [report_fingerprint(rep[rep[:, 2] == r]) for r in range(ref["rounds"])]
        assert w_fps == ref_fps
        assert t_fps == ref_fps
        assert sum(s["removals"] for s in w_stats) > 0
        # the tracked run: counters, digests, coverage
        _check_counters(t_stats, ref)
        assert np.array_equal(t["dig"], ref["digest"])
        assert np.array_equal(t["cov"], ref["coverage"])
    p0 = parts[0]   # shard [0, 64): its own columns of the oracle's run
    assert np.array_equal(p0["seen"], ref["seen"][:, :1])
    assert np.array_equal(p0["cov"], ref["coverage"][:64])
    assert np.array_equal(p0["fwd"], ref["forwards"][:64])
    if churn:
        assert p0["fps"] == ref_fps[:len(p0["fps"])]
    del ref

    # the whole run is the composition of the shards
    R = len(t_stats)
    assert max(len(p["stats"]) for p in parts) == R
    for i, s in enumerate(t_stats):
        for k in ("injected", "lost", "new_bits", "sends"):
            assert s[k] == sum(p["stats"][i][k] for p in parts if i < len(p["stats"])), (k, i)
        for k in ("crashed", "reports", "removals", "dup_reports"):
            assert all(p["stats"][i][k] == s[k] for p in parts if i < len(p["stats"])), (k, i)
    dig = np.zeros_like(t["dig"])
    for p in parts:
        dig ^= p["digest"]
    assert np.array_equal(dig, t["dig"])
    assert np.array_equal(np.concatenate([p["cov"] for p in parts]), t["cov"])
    assert np.array_equal(np.concatenate([p["fwd"] for p in parts]), t["fwd"])
    return dict(stats=w_stats, cov=t["cov"], fwd=t["fwd"], dig=t["dig"], g=g, origin=origin, cfg=bench_cfg,
                fps=w_fps)


@pytest.mark.timeout(900)
def test_c4_full_size_parity(pkg, oracle):
    """BASELINE config 4 at its own size: 2^24 vertices x 4096 messages, the
    bench-configured W = 64 run against the oracle's run of all 4096 messages."""
    out = _full_size(pkg, oracle, 24, 4, churn=False)
    assert out["stats"][-1]["new_bits"] == 0
    # the same run with compact Message-Lists (round 2 through the flat record
    # pull, k_expand_rec): identical to the oracle-checked run
    with pkg.GossipEngine(0, compact_rows=1, **{k: v for k, v in out["cfg"].items() if k != "compact_rows"}) as eng:
        eng.load_graph(out["g"])
        eng.set_messages(out["origin"])
        eng.reset()
        stats, _ = _run(eng)
        assert any(s["scan"] & 4 for s in stats)
        for a, b in zip(stats, out["stats"]):
            for k in STAT_KEYS:
                assert a[k] == b[k], (k, a["round"])
        assert np.array_equal(eng.coverage(), out["cov"])
        assert np.array_equal(eng.forwards(), out["fwd"])
        assert np.array_equal(eng.digest(), out["dig"])


@pytest.mark.timeout(1500)
def test_c5_full_size_parity(pkg, oracle):
    """BASELINE config 5 at its own size: 2^26 vertices x 4096 messages, 1 %/round
    crashes, 3-miss detection, seed removal (Peer.py:298-313, 395-408,
    Seed.py:358-406): the bench-configured run and the tracked run against the
    oracle's run of all 4096 messages."""
    out = _full_size(pkg, oracle, 26, 5, churn=True)
    # the last message word, [4032, 4096), as a shard of its own: the whole
    # run's columns and reports
    with pkg.GossipEngine(0, **dict(out["cfg"], track_msg_forwards=1)) as eng:
        eng.load_graph(out["g"])
        eng.set_message_shard(out["origin"], None, 4032, 4096)
        eng.reset()
        stats, fps = _run(eng, with_reports=True)
        assert fps == out["fps"][:len(fps)]
        assert np.array_equal(eng.coverage(), out["cov"][4032:])
        assert np.array_equal(eng.forwards(), out["fwd"][4032:])
