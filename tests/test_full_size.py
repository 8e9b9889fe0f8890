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

C5: the oracle runs message word 0 -- messages [0, 64) -- and the last word --
[4032, 4096) -- each as a one-word run, against the engine's one-word runs of
the same messages (every counter, digests, coverage, forwards and every round's
dead-node reports).

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


def _check_word(part, ref, w_fps=None):
    """A one-word engine run (counters, Message-Lists when read, digest,
    coverage, forwards, per-round report fingerprints) against the oracle's."""
    assert len(part["stats"]) == ref["rounds"]
    for a, b in zip(part["stats"], ref["stats"]):
        for k in STAT_KEYS:
            assert a[k] == b[k], (k, a["round"], a[k], b[k])
    if "seen" in part:
        assert np.array_equal(part["seen"], ref["seen"][:, :1])
    assert np.array_equal(part["digest"], ref["digest"])
    assert np.array_equal(part["cov"], ref["coverage"])
    assert np.array_equal(part["fwd"], ref["forwards"])
    if part["fps"]:
        assert ref["n_reports"] <= 1 << 27
        rep = ref["reports"]
        for r, fp in enumerate(part["fps"]):
            assert fp == report_fingerprint(rep[rep[:, 2] == r]), r
        if w_fps is not None:   # liveness is replicated: the same reports every round
            k = min(len(part["fps"]), len(w_fps))
            assert k >= 4 and part["fps"][:k] == w_fps[:k]


def _full_size(pkg, oracle, log2n, seed, churn):
    n, m = 1 << log2n, 4096
    cfg = dict(track_digest=1)
    okw = {}
    if churn:
        cfg.update(churn=1, p_fail=0.01, churn_seed=seed, miss_threshold=3, track_msg_forwards=1,
                   report_capacity=1 << 24)
        okw = dict(churn=True, p_fail=0.01, churn_seed=seed)
    t0 = time.time()
    whole = pkg.GossipEngine(0, **cfg)
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
    w_dig, w_cov, w_fwd = whole.digest().copy(), whole.coverage(), whole.forwards()
    w_seen = whole.seen() if not churn else None   # 8 GiB at C4
    whole.close()
    _log(f"whole run: {len(w_stats)} rounds in {time.time() - t0:.1f} s")
    assert sum(s["sends"] for s in w_stats) == int(w_fwd.sum())
    assert sum(s["injected"] + s["new_bits"] for s in w_stats) == int(w_cov.sum())

    # message shards on a second context
    sh = pkg.GossipEngine(0, **cfg)
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

    if not churn:
        # the whole W = 64 run against the oracle's run of all 4096 messages
        t0 = time.time()
        ref = oracle.run(g, origin, nthreads=_threads(), want_first=False)
        _log(f"oracle, all {m} messages: {ref['rounds']} rounds in {time.time() - t0:.1f} s ({_threads()} threads)")
        assert len(w_stats) == ref["rounds"]
        for a, b in zip(w_stats, ref["stats"]):
            for k in STAT_KEYS:
                assert a[k] == b[k], (k, a["round"], a[k], b[k])
        assert w_seen.shape == ref["seen"].shape
        for lo in range(0, n, 1 << 20):   # blockwise: no 8 GiB temporaries
            assert np.array_equal(w_seen[lo:lo + (1 << 20)], ref["seen"][lo:lo + (1 << 20)]), lo
        assert np.array_equal(w_dig, ref["digest"])
        assert np.array_equal(w_cov, ref["coverage"])
        assert np.array_equal(w_fwd, ref["forwards"])
        p0 = parts[0]   # shard [0, 64): its own columns of the oracle's run
        assert np.array_equal(p0["seen"], ref["seen"][:, :1])
        assert np.array_equal(p0["cov"], ref["coverage"][:64])
        assert np.array_equal(p0["fwd"], ref["forwards"][:64])
        del ref, w_seen
    else:
        # one-word runs of the first and the last message word against the oracle
        ref = oracle.run(g, origin[:64], nthreads=_threads(), want_first=False, report_cap=1 << 27, **okw)
        _log(f"oracle, word 0: {ref['rounds']} rounds ({_threads()} threads)")
        _check_word(parts[0], ref, w_fps)
        del ref

    # the whole run is the composition of the shards
    R = len(w_stats)
    assert max(len(p["stats"]) for p in parts) == R
    for i, s in enumerate(w_stats):
        for k in ("injected", "lost", "new_bits", "sends"):
            assert s[k] == sum(p["stats"][i][k] for p in parts if i < len(p["stats"])), (k, i)
        for k in ("crashed", "reports", "removals", "dup_reports"):
            assert all(p["stats"][i][k] == s[k] for p in parts if i < len(p["stats"])), (k, i)
    dig = np.zeros_like(w_dig)
    for p in parts:
        dig ^= p["digest"]
    assert np.array_equal(dig, w_dig)
    assert np.array_equal(np.concatenate([p["cov"] for p in parts]), w_cov)
    assert np.array_equal(np.concatenate([p["fwd"] for p in parts]), w_fwd)
    return dict(stats=w_stats, cov=w_cov, fwd=w_fwd, dig=w_dig, g=g, origin=origin, cfg=cfg, fps=w_fps)


@pytest.mark.timeout(900)
def test_c4_full_size_parity(pkg, oracle):
    """BASELINE config 4 at its own size: 2^24 vertices x 4096 messages, the
    whole W = 64 run against the oracle's run of all 4096 messages."""
    out = _full_size(pkg, oracle, 24, 4, churn=False)
    assert out["stats"][-1]["new_bits"] == 0
    # the same run with compact Message-Lists (round 2 through the flat record
    # pull, k_expand_rec): identical to the oracle-checked run
    with pkg.GossipEngine(0, compact_rows=1, **out["cfg"]) as eng:
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


@pytest.mark.timeout(1200)
def test_c5_full_size_parity(pkg, oracle):
    """BASELINE config 5 at its own size: 2^26 vertices x 4096 messages, 1 %/round
    crashes, 3-miss detection, seed removal."""
    out = _full_size(pkg, oracle, 26, 5, churn=True)
    assert sum(s["removals"] for s in out["stats"]) > 0
    # the last message word, [4032, 4096), alone against the oracle and against
    # the whole run's columns
    with pkg.GossipEngine(0, **out["cfg"]) as eng:
        eng.load_graph(out["g"])
        eng.configure(msg_word_base=0)   # local word numbers, as the oracle's digest
        eng.set_messages(out["origin"][4032:])
        eng.reset()
        stats, fps = _run(eng, with_reports=True)
        part = dict(stats=stats, fps=fps, digest=eng.digest().copy(), cov=eng.coverage(), fwd=eng.forwards())
    ref = oracle.run(out["g"], out["origin"][4032:], nthreads=_threads(), want_first=False, report_cap=1 << 27,
                     churn=True, p_fail=0.01, churn_seed=5)
    _log(f"oracle, last word: {ref['rounds']} rounds")
    _check_word(part, ref, out["fps"])
    assert np.array_equal(part["cov"], out["cov"][4032:])
    assert np.array_equal(part["fwd"], out["fwd"][4032:])
