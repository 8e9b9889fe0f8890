"""GPU parity: the HIP engine (through the C-ABI) against the CPU oracle.

Bar: bit-exact for everything -- first-receipt matrices, per-vertex digests,
Message-List bitmaps, per-message coverage/forwards, per-round counters,
dead-node reports (as sets), vertex state.  Oracles: oracle/gossip_oracle.c
(cross-checked against the per-peer sha256 harness in test_oracle.py) and the
reference's own fixtures in tests/golden/.
"""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

STAT_KEYS = ("injected", "lost", "new_bits", "receivers", "sends", "active", "crashed",
             "reports", "removals", "dup_reports")


def _engine(pkg, g, origin, inject=None, **cfg):
    eng = pkg.GossipEngine(0, **cfg)
    eng.load_graph(g)
    eng.set_messages(origin, inject)
    eng.reset()
    return eng


# (push_ratio, unfiltered_pct, flat_max_words, arc_mask_permille): always pull
# with the per-arc activity probe, per-receiver kernel at every width; the same
# with the per-arc activity mask whenever >= 0.1 % of vertices send; always
# pull, unfiltered whenever >= 1 % of vertices send, edge-parallel kernel up to
# W = 32; always push; adaptive direction + unfiltered dense rounds (defaults)
MODES = [(0.0, 0, 0, 0), (0.0, 0, 0, 1), (0.0, 1, 32, 0), (1e-12, 90, 16, 10), (10.0, 90, 16, 10)]
MODE_IDS = ["pull", "pull-masked", "pull-unfiltered", "push", "adaptive"]


def _compare(pkg, oracle, g, origin, inject=None, crashes=(), first=True, hub_threshold=4096,
             push_ratio=10.0, unfiltered_pct=90, flat_max_words=16, arc_mask_permille=10, prefilter_pct=20,
             compact_rows=1, summary_min_n=None, track_fwd=None, split_deg=None, split_max_permille=None, **kw):
    """track_fwd: keep exact frontier rows for per-message forwards (default:
    with liveness).  track_fwd=0 under churn is bench.py's C5 configuration:
    no frontier rows, so the push gathers whole Message-Lists under liveness;
    forwards are then not kept and not compared."""
    churn = kw.get("churn", False)
    live = bool(churn or crashes)
    if track_fwd is None:
        track_fwd = int(live)
    cfg = dict(track_first=int(first), track_digest=1, track_msg_forwards=int(track_fwd),
               churn=int(churn), p_fail=kw.get("p_fail", 0.0), churn_seed=kw.get("churn_seed", 0),
               hub_threshold=hub_threshold, push_ratio=push_ratio,
               unfiltered_pct=unfiltered_pct, flat_max_words=flat_max_words,
               arc_mask_permille=arc_mask_permille, prefilter_pct=prefilter_pct, compact_rows=compact_rows)
    if summary_min_n is not None:
        cfg["summary_min_n"] = summary_min_n
    if split_deg is not None:
        cfg["split_deg"] = split_deg
    if split_max_permille is not None:
        cfg["split_max_permille"] = split_max_permille
    eng = _engine(pkg, g, origin, inject, **cfg)
    by_round = {}
    for v, r in crashes:
        by_round.setdefault(r, []).append(v)
    stats, reports = [], []
    last = int(np.max(inject)) if inject is not None and len(inject) else 0
    for r in range(254):
        if r in by_round:
            eng.crash(by_round[r])
        st = eng.round()
        stats.append(st)
        rep, nrep = eng.reports()
        assert nrep == len(rep)
        reports.extend(map(tuple, rep.tolist()))
        if st["new_bits"] == 0 and r >= last:
            break
    eng.finalize()
    ref = oracle.run(g, origin, inject, crashes=crashes, want_first=first, **kw)
    assert len(stats) == ref["rounds"]
    for a, b in zip(stats, ref["stats"]):
        for k in STAT_KEYS:
            assert a[k] == b[k], (k, a["round"], a[k], b[k])
    W = eng.words
    for s in stats:   # word skip and compact records only ever drop loads (+ a record mask each)
        assert s["row_bytes"] <= (8 * W + (8 if s["scan"] & 4 else 0)) * s["rows_gathered"], s
        if s["mode"] == 1:
            assert s["row_bytes"] == 8 * W * s["rows_gathered"], s
    assert np.array_equal(eng.seen(), ref["seen"][:, :W])
    if first:
        assert np.array_equal(eng.first(), ref["first"])
    assert np.array_equal(eng.digest(), ref["digest"])
    assert np.array_equal(eng.coverage(), ref["coverage"])
    if track_fwd or not live:
        assert np.array_equal(eng.forwards(), ref["forwards"])
    else:
        with pytest.raises(pkg.GossipError):   # not kept: refused, never approximated
            eng.forwards()
    assert sorted(reports) == sorted(map(tuple, ref["reports"].tolist()))
    out = {"stats": stats, "eng": eng, "ref": ref}
    return out


@pytest.mark.parametrize("mode", MODES, ids=MODE_IDS)
def test_c2_ba_10k_64(pkg, oracle, mode):
    """BASELINE config 2: 10^4-node BA(m=2), 64 concurrent messages."""
    push_ratio, unfiltered_pct, flat_max_words, arc_mask = mode
    g = pkg.overlay.barabasi_albert(10_000, 2, seed=2)
    origin = pkg.overlay.random_origins(g.n, 64, seed=2)
    r = _compare(pkg, oracle, g, origin, push_ratio=push_ratio, unfiltered_pct=unfiltered_pct, flat_max_words=flat_max_words, arc_mask_permille=arc_mask)
    if push_ratio == 1e-12:
        assert all(s["mode"] == 1 for s in r["stats"])
    if push_ratio == 0.0:
        assert all(s["mode"] == 0 for s in r["stats"])
        assert any(s["scan"] == 2 for s in r["stats"]) == (unfiltered_pct == 1)
        assert any(s["scan"] == 1 for s in r["stats"]) == (arc_mask == 1)
    total = sum(s["sends"] for s in r["stats"])
    assert total == 64 * g.nnz   # connected BA: every message crosses every arc once
    r["eng"].close()


@pytest.mark.parametrize("mode", MODES, ids=MODE_IDS)
@pytest.mark.parametrize("m", [1, 10, 63, 64, 65, 130, 300, 1000, 2000, 4096])
def test_message_widths(pkg, oracle, m, mode):
    push_ratio, unfiltered_pct, flat_max_words, arc_mask = mode
    g = pkg.overlay.barabasi_albert(1500, 3, seed=m)
    origin = pkg.overlay.random_origins(g.n, m, seed=m)
    inject = (np.arange(m) % 5).astype(np.int32)
    _compare(pkg, oracle, g, origin, inject, push_ratio=push_ratio, unfiltered_pct=unfiltered_pct, flat_max_words=flat_max_words, arc_mask_permille=arc_mask)["eng"].close()


@pytest.mark.parametrize("mode", MODES, ids=MODE_IDS)
def test_hub_split(pkg, oracle, mode):
    """Force the multi-wave hub paths (pull: partials + final; push: grid-wide
    sweep of big senders) on every vertex above 64 arcs."""
    push_ratio, unfiltered_pct, flat_max_words, arc_mask = mode
    rp, col = oracle.chung_lu(20_000, 8, 2.2, 11)
    g = pkg.CSR(20_000, rp, col, False)
    assert np.diff(rp).max() > 1000
    origin = pkg.overlay.random_origins(g.n, 256, seed=11)
    _compare(pkg, oracle, g, origin, hub_threshold=64, push_ratio=push_ratio, unfiltered_pct=unfiltered_pct, flat_max_words=flat_max_words, arc_mask_permille=arc_mask)["eng"].close()


def test_c1_directed_schedule_and_direct_deliveries(pkg, oracle):
    """C1: 10 peers, first-3 overlay, 10 msgs/peer every 5 rounds.  Round 1 after
    each injection reproduces the reference's direct delivery matrix."""
    golden = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "c1_wire.json")))
    g = pkg.overlay.first3_overlay(10)
    origin, inject, count = pkg.peer.c1_schedule(10)
    origin, inject = np.array(origin, np.int32), np.array(inject, np.int32)
    r = _compare(pkg, oracle, g, origin, inject)
    first = r["eng"].first()
    direct = sorted([int(origin[k]), int(count[k]), int(v)] for k in range(len(origin))
                    for v in np.nonzero(first[:, k] == inject[k] + 1)[0])
    assert direct == sorted(golden["deliveries"])
    r["eng"].close()


@pytest.mark.parametrize("mode", MODES, ids=MODE_IDS)
@pytest.mark.parametrize("track_fwd", [1, 0], ids=["frontier-rows", "bench-c5"])
def test_churn_random(pkg, oracle, mode, track_fwd):
    """Random churn, with exact frontier rows (per-message forwards) and
    without them (bench.py's C5 configuration: the push gathers whole
    Message-Lists under liveness, the pull keeps no frontier stores)."""
    push_ratio, unfiltered_pct, flat_max_words, arc_mask = mode
    g = pkg.overlay.barabasi_albert(5000, 2, seed=5)
    origin = pkg.overlay.random_origins(g.n, 128, seed=5)
    inject = (np.arange(128) % 9).astype(np.int32)
    r = _compare(pkg, oracle, g, origin, inject, churn=True, p_fail=0.03, churn_seed=77, track_fwd=track_fwd,
                 push_ratio=push_ratio, unfiltered_pct=unfiltered_pct, flat_max_words=flat_max_words, arc_mask_permille=arc_mask)
    assert sum(s["removals"] for s in r["stats"]) > 0
    if push_ratio == 1e-12:
        assert all(s["mode"] == 1 for s in r["stats"])
    r["eng"].close()


@pytest.mark.parametrize("mode", MODES, ids=MODE_IDS)
@pytest.mark.parametrize("m", [4096, 1000])
def test_churn_wide_rows_bench_c5(pkg, oracle, mode, m):
    """bench.py's C5 configuration (no frontier rows) at W = 64 and W = 16 on
    a Chung-Lu overlay with hubs: pushes of whole Message-Lists under
    liveness, parked rows, alive sets, sated vertices."""
    push_ratio, unfiltered_pct, flat_max_words, arc_mask = mode
    rp, col = oracle.chung_lu(60_000, 10, 2.4, 27)
    g = pkg.CSR(60_000, rp, col, False)
    origin = pkg.overlay.random_origins(g.n, m, seed=27)
    r = _compare(pkg, oracle, g, origin, first=False, hub_threshold=512, push_ratio=push_ratio,
                 unfiltered_pct=unfiltered_pct, flat_max_words=flat_max_words, arc_mask_permille=arc_mask,
                 churn=True, p_fail=0.01, churn_seed=8, track_fwd=0, compact_rows=0)
    assert sum(s["removals"] for s in r["stats"]) > 0
    r["eng"].close()


@pytest.mark.parametrize("n,m,p_fail", [(5000, 128, 0.03), (3000, 1000, 0.02), (1500, 4096, 0.05)])
@pytest.mark.parametrize("flat_max_words", [0, 16])
def test_unfiltered_pull_parks_crashed_rows(pkg, oracle, n, m, p_fail, flat_max_words):
    """Unfiltered pull under churn: before each unfiltered round the rows of the
    down vertices move to the parked slot (k_park), so no receiver ORs in bits a
    crashed vertex never sent; seen rows, coverage (finalize reads parked rows)
    and reports match the oracle."""
    g = pkg.overlay.barabasi_albert(n, 3, seed=n)
    origin = pkg.overlay.random_origins(g.n, m, seed=m)
    inject = (np.arange(m) % 4).astype(np.int32)
    r = _compare(pkg, oracle, g, origin, inject, crashes=[(int(origin[0]), 2), (int(origin[1]), 3)],
                 churn=True, p_fail=p_fail, churn_seed=31, push_ratio=0.0, unfiltered_pct=1,
                 flat_max_words=flat_max_words, arc_mask_permille=0)
    assert sum(1 for s in r["stats"] if s["scan"] & 3 == 2) >= 3, [s["scan"] for s in r["stats"]]
    assert sum(s["crashed"] for s in r["stats"]) > 0
    r["eng"].close()


@pytest.mark.parametrize("mode", MODES, ids=MODE_IDS)
def test_detection_of_crashed_hubs(pkg, oracle, mode):
    """Crashed vertices with more than 2048 heartbeat links are detected by the
    grid-wide k_det_big_* kernels, the rest inside k_detect's waves: the top
    hubs crash explicitly (and at random), reports and removals match."""
    push_ratio, unfiltered_pct, flat_max_words, arc_mask = mode
    rp, col = oracle.chung_lu(60_000, 12, 2.1, 17)
    g = pkg.CSR(60_000, rp, col, False)
    deg = np.diff(rp)
    hubs = np.argsort(-deg)[:6]
    assert deg[hubs[3]] > 2048, deg[hubs]
    origin = pkg.overlay.random_origins(g.n, 256, seed=17)
    inject = (np.arange(256) % 3).astype(np.int32)
    crashes = [(int(h), 1 + i % 3) for i, h in enumerate(hubs)]
    r = _compare(pkg, oracle, g, origin, inject, crashes=crashes, churn=True, p_fail=0.02, churn_seed=23,
                 push_ratio=push_ratio, unfiltered_pct=unfiltered_pct, flat_max_words=flat_max_words,
                 arc_mask_permille=arc_mask)
    assert sum(s["removals"] for s in r["stats"]) >= 6
    assert sum(s["reports"] for s in r["stats"]) > 6 * 2048
    r["eng"].close()


@pytest.mark.parametrize("mode", MODES, ids=MODE_IDS)
def test_explicit_crashes_directed(pkg, oracle, mode):
    push_ratio, unfiltered_pct, flat_max_words, arc_mask = mode
    g = pkg.overlay.first3_overlay(10)
    origin, inject, _ = pkg.peer.c1_schedule(10)
    r = _compare(pkg, oracle, g, np.array(origin, np.int32), np.array(inject, np.int32),
                 crashes=[(4, 1), (0, 6), (9, 3)], push_ratio=push_ratio, unfiltered_pct=unfiltered_pct, flat_max_words=flat_max_words, arc_mask_permille=arc_mask)
    assert sum(s["removals"] for s in r["stats"]) >= 2
    r["eng"].close()


def test_chung_lu_device_builder_matches_oracle(pkg, oracle):
    for n, dbar, seed in [(1000, 4, 1), (100_000, 8, 3)]:
        with pkg.GossipEngine(0) as eng:
            eng.build_chung_lu(n, dbar, 2.5, seed)
            dg = eng.graph()
        rp, col = oracle.chung_lu(n, dbar, 2.5, seed)
        assert np.array_equal(dg.row_ptr, rp)
        assert np.array_equal(dg.col, col)


@pytest.mark.parametrize("n,dbar,seed", [(1_000_000, 8, 3), (1_000_000, 16, 3), (1 << 24, 16, 4)])
def test_degree_check_on_device_overlays(pkg, n, dbar, seed):
    """SURVEY.md §8a A9 on the engine's own overlays (C3's recipe, C4's 2^24
    overlay): the discrete power-law MLE recovers gamma = 2.5 within 0.15
    (degree-weighted selection is the reference's intent,
    demonstrate_powerlaw.py:19-27)."""
    with pkg.GossipEngine(0) as eng:
        eng.build_chung_lu(n, dbar, 2.5, seed)
        chk = eng.check_degree(2.5)
    assert chk["ok"] and abs(chk["gamma_hat"] - 2.5) <= 0.15, chk
    assert chk["n_tail"] >= 1000 and chk["max_degree"] > 100 * dbar, chk


@pytest.mark.parametrize("mode", MODES, ids=MODE_IDS)
def test_c3_chung_lu_1e6_1024(pkg, oracle, mode):
    """BASELINE config 3: 10^6-node Chung-Lu (gamma 2.5), 1024 messages."""
    push_ratio, unfiltered_pct, flat_max_words, arc_mask = mode
    n = 1_000_000
    with pkg.GossipEngine(0, track_digest=1, push_ratio=push_ratio, unfiltered_pct=unfiltered_pct, flat_max_words=flat_max_words, arc_mask_permille=arc_mask) as eng:
        eng.build_chung_lu(n, 8, 2.5, 3)
        g = eng.graph()
        origin = pkg.overlay.random_origins(n, 1024, seed=3)
        eng.set_messages(origin)
        eng.reset()
        stats = eng.run()
        eng.finalize()
        digest, cov, fwd = eng.digest(), eng.coverage(), eng.forwards()
    ref = oracle.run(g, origin, nthreads=8, want_first=False)
    assert len(stats) == ref["rounds"]
    for a, b in zip(stats, ref["stats"]):
        for k in STAT_KEYS:
            assert a[k] == b[k], (k, a["round"])
    assert np.array_equal(digest, ref["digest"])
    assert np.array_equal(cov, ref["coverage"])
    assert np.array_equal(fwd, ref["forwards"])


def _group_run(pkg, g, origin, inject, P, crashes=(), **cfg):
    """Vertex partition over P contexts on one GPU (gp_round_group: the
    boundary exchange through device-to-device copies)."""
    engs = []
    for k in range(P):
        e = pkg.GossipEngine(0, **cfg)
        e.load_graph(g)
        e.set_partition(k, P)
        e.set_messages(origin, inject)
        e.reset()
        engs.append(e)
    by_round = {}
    for v, r in crashes:
        by_round.setdefault(r, []).append(v)
    stats, reports = [], []
    last = int(np.max(inject)) if inject is not None and len(inject) else 0
    for r in range(254):
        if r in by_round:
            for e in engs:   # the host hands every rank the same (global) crash list
                e.crash(by_round[r])
        st = pkg.GossipEngine.round_group(engs)
        stats.append(st)
        for e in engs:
            rep, nrep = e.reports()
            assert nrep == len(rep)
            reports.extend(map(tuple, rep.tolist()))
        if st["new_bits"] == 0 and r >= last:
            break
    return engs, stats, reports


@pytest.mark.parametrize("mode", MODES, ids=MODE_IDS)
@pytest.mark.parametrize("churn", [False, True])
@pytest.mark.parametrize("by_arcs", [0, 1], ids=["vertex-slices", "arc-slices"])
def test_group_partition_invariance(pkg, oracle, mode, churn, by_arcs):
    """Vertex partition over P = 2, 3, 4 contexts: owned
    slices (equal vertex counts, or equal arc counts) + ghost
    rows, the sparse boundary exchange of this round's new bits (and removal
    flags) through the same pack / unpack buffers and the same exchange plan
    (csrc/xplan.h) as the RCCL path.  Every output equals the oracle's (one
    context)."""
    push_ratio, unfiltered_pct, flat_max_words, arc_mask = mode
    g = pkg.overlay.barabasi_albert(3001, 2, seed=8)
    origin = pkg.overlay.random_origins(g.n, 200, seed=8)
    inject = (np.arange(200) % 4).astype(np.int32)
    kw = dict(churn=True, p_fail=0.02, churn_seed=3) if churn else {}
    crashes = [(int(origin[5]), 1), (17, 2)] if churn else []
    ref = oracle.run(g, origin, inject, crashes=crashes, want_first=True, **kw)
    cfg = dict(track_first=1, track_msg_forwards=int(churn), push_ratio=push_ratio, unfiltered_pct=unfiltered_pct,
               flat_max_words=flat_max_words, arc_mask_permille=arc_mask, partition_by_arcs=by_arcs)
    if churn:
        cfg.update(churn=1, p_fail=0.02, churn_seed=3)
    for P in (2, 3, 4):
        engs, stats, reports = _group_run(pkg, g, origin, inject, P, crashes, **cfg)
        bounds = pkg.dist.partition_bounds(g.n, P, g.row_ptr if by_arcs else None)
        assert [e.partition() for e in engs] == bounds
        assert len(stats) == ref["rounds"], P
        for a, b in zip(stats, ref["stats"]):
            for k in STAT_KEYS:
                assert a[k] == b[k], (P, k, a["round"], a[k], b[k])
        assert sum(s["xchg_rows"] for s in stats) > 0
        assert sorted(reports) == sorted(map(tuple, ref["reports"].tolist()))
        first = np.concatenate([e.first() for e in engs])
        digest = np.concatenate([e.digest() for e in engs])
        seen = np.concatenate([e.seen() for e in engs])
        assert np.array_equal(first, ref["first"])
        assert np.array_equal(digest, ref["digest"])
        assert np.array_equal(seen, ref["seen"][:, :engs[0].words])
        cov = fwd = 0
        for e in engs:
            e.finalize()
            cov = cov + e.coverage()
            if churn:
                fwd = fwd + e.forwards()
            else:
                fwd = fwd + e.forwards()
        assert np.array_equal(cov, ref["coverage"])
        assert np.array_equal(fwd, ref["forwards"])
        if churn:   # owned slices of the vertex state agree with one context's
            with pkg.GossipEngine(0, **cfg) as one:
                one.load_graph(g)
                one.set_messages(origin, inject)
                one.reset()
                by_round = {}
                for v, r in crashes:
                    by_round.setdefault(r, []).append(v)
                for r in range(len(stats)):
                    if r in by_round:
                        one.crash(by_round[r])
                    one.round()
                assert np.array_equal(np.concatenate([e.state() for e in engs]), one.state())
                assert np.array_equal(np.concatenate([e.deg_live() for e in engs]), one.deg_live())
                assert np.array_equal(np.concatenate([e.miss() for e in engs]), one.miss())
        for e in engs:
            e.close()


@pytest.mark.parametrize("churn", [False, True])
def test_group_partition_at_scale(pkg, oracle, churn):
    """Vertex partition at 2^20 vertices (Chung-Lu, 16.7 M arcs) x 512
    messages over P = 4 arc-balanced slices: per-round counters, digests,
    Message-Lists, coverage and forwards equal the one-context run's, which
    the oracle pins (run here too at this size)."""
    n = 1 << 20
    rp, col = oracle.chung_lu(n, 16, 2.5, 12)
    g = pkg.CSR(n, rp, col, False)
    origin = pkg.overlay.random_origins(n, 512, seed=12)
    cfg = dict(track_msg_forwards=int(churn), partition_by_arcs=1)
    kw = {}
    if churn:
        cfg.update(churn=1, p_fail=0.01, churn_seed=4)
        kw = dict(churn=True, p_fail=0.01, churn_seed=4)
    engs, stats, _ = _group_run(pkg, g, origin, None, 4, **cfg)
    ref = oracle.run(g, origin, nthreads=int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1),
                     report_cap=1 << 24, **kw)
    assert len(stats) == ref["rounds"]
    for a, b in zip(stats, ref["stats"]):
        for k in STAT_KEYS:
            assert a[k] == b[k], (k, a["round"], a[k], b[k])
    assert sum(s["xchg_rows"] for s in stats) > 0
    assert np.array_equal(np.concatenate([e.digest() for e in engs]), ref["digest"])
    assert np.array_equal(np.concatenate([e.seen() for e in engs]), ref["seen"])
    cov = fwd = 0
    for e in engs:
        e.finalize()
        cov = cov + e.coverage()
        fwd = fwd + e.forwards()
        e.close()
    assert np.array_equal(cov, ref["coverage"])
    assert np.array_equal(fwd, ref["forwards"])


@pytest.mark.parametrize("by_arcs", [0, 1], ids=["vertex-slices", "arc-slices"])
def test_partition_local_graph(pkg, by_arcs):
    """The local CSR of a partition: owned rows are the global in-lists
    (gather order, local ids), ghost rows list their owned neighbours, and
    every rank's ghosts of owner p are exactly the vertices p sends to it."""
    g = pkg.overlay.barabasi_albert(2000, 3, seed=1)
    P = 3
    origin = np.array([0, 1999, 1000], np.int32)
    locs = []
    bounds = pkg.dist.partition_bounds(g.n, P, g.row_ptr if by_arcs else None)
    for k in range(P):
        with pkg.GossipEngine(0, partition_by_arcs=by_arcs) as e:
            e.load_graph(g)
            e.set_partition(k, P)
            e.set_messages(origin)
            vb, ve = e.partition()
            rp, col, l2g = e.local_graph()
            locs.append((vb, ve, rp, col, l2g, e.local_info()))
    if by_arcs:   # BA's early vertices are its hubs: arc slices hold fewer of them
        arcs = [int(g.row_ptr[e] - g.row_ptr[b]) for b, e in bounds]
        assert max(arcs) - min(arcs) <= int(np.diff(g.row_ptr).max())
        assert bounds[0][1] - bounds[0][0] < bounds[-1][1] - bounds[-1][0]
    for k, (vb, ve, rp, col, l2g, (nloc, ng, nx, nnz_l, nb)) in enumerate(locs):
        assert (vb, ve) == bounds[k] and nloc == ve - vb
        assert np.array_equal(l2g[:nloc], np.arange(vb, ve))
        ghosts = l2g[nloc:nloc + ng]
        assert np.all(np.diff(ghosts) > 0) and not np.any((ghosts >= vb) & (ghosts < ve))
        extras = l2g[nloc + ng:]
        assert set(extras.tolist()) == {int(o) for o in origin if not (vb <= o < ve) and o not in set(ghosts.tolist())}
        for i in range(nloc):   # owned rows: the whole in-list
            v = vb + i
            assert sorted(l2g[col[rp[i]:rp[i + 1]]].tolist()) == g.col[g.row_ptr[v]:g.row_ptr[v + 1]].tolist()
        for x in range(nloc, nloc + ng):   # ghost rows: owned neighbours
            u = int(l2g[x])
            nb_own = [w for w in g.col[g.row_ptr[u]:g.row_ptr[u + 1]].tolist() if vb <= w < ve]
            assert sorted(l2g[col[rp[x]:rp[x + 1]]].tolist()) == nb_own
        assert rp[-1] == nnz_l and np.all(np.diff(rp[nloc + ng:]) == 0)
        # boundary entries = sum over peers of the ghosts they hold from this rank
        held = sum(int(np.sum((o[4][o[5][0]:o[5][0] + o[5][1]] >= vb) & (o[4][o[5][0]:o[5][0] + o[5][1]] < ve)))
                   for j, o in enumerate(locs) if j != k)
        assert nb == held


def test_rccl_one_rank(pkg, oracle):
    """The RCCL path on a one-GPU box: a real one-rank communicator
    (gp_comm_unique_id + gp_comm_init), rounds through round_exchange_rccl
    (the counters' all-reduce), results equal to the oracle's."""
    g = pkg.overlay.barabasi_albert(5000, 2, seed=9)
    origin = pkg.overlay.random_origins(g.n, 128, seed=9)
    inject = (np.arange(128) % 3).astype(np.int32)
    ref = oracle.run(g, origin, inject, churn=True, p_fail=0.01, churn_seed=2, want_first=True)
    with pkg.GossipEngine(0, track_first=1, track_msg_forwards=1, churn=1, p_fail=0.01, churn_seed=2) as e:
        e.load_graph(g)
        e.comm_init(pkg.GossipEngine.comm_unique_id(), 1, 0)
        e.set_messages(origin, inject)
        e.reset()
        stats = e.run()
        e.finalize()
        assert len(stats) == ref["rounds"]
        for a, b in zip(stats, ref["stats"]):
            for k in STAT_KEYS:
                assert a[k] == b[k], (k, a["round"])
        assert np.array_equal(e.first(), ref["first"])
        assert np.array_equal(e.digest(), ref["digest"])
        assert np.array_equal(e.coverage(), ref["coverage"])
        assert np.array_equal(e.forwards(), ref["forwards"])


def test_asymmetric_overlay_rejected_by_partition(pkg):
    """A vertex partition relies on the overlay being symmetric (Seed.py:131-149):
    rank q's ghosts of owner p are then exactly p's send list B_pq.  An
    asymmetric in-CSR loaded as undirected must be rejected before the first
    exchange (xplan_check_lists), not unpacked into another owner's ghosts."""
    arcs = [(0, 1), (1, 0), (5, 6), (6, 5), (2, 7)]   # 2 -> 7 without 7 -> 2
    src = np.array([a for a, _ in arcs]); dst = np.array([b for _, b in arcs])
    g = pkg.CSR.from_arcs(10, src, dst, directed=True)
    g = pkg.CSR(g.n, g.row_ptr, g.col, False)
    engs = []
    try:
        for k in range(2):
            e = pkg.GossipEngine(0)
            e.load_graph(g)
            e.set_partition(k, 2)
            e.set_messages(np.array([2, 0], np.int32))
            e.reset()
            engs.append(e)
        with pytest.raises(pkg.GossipError, match="not symmetric"):
            pkg.GossipEngine.round_group(engs)
    finally:
        for e in engs:
            e.close()


def test_partitioned_round_needs_an_exchange(pkg):
    g = pkg.overlay.barabasi_albert(500, 2, seed=1)
    with pkg.GossipEngine(0) as e:
        e.load_graph(g)
        e.set_partition(0, 2)
        e.set_messages(np.array([3], np.int32))
        e.reset()
        with pytest.raises(pkg.GossipError):
            e.round()
        with pytest.raises(pkg.GossipError):   # the partition is fixed once per overlay
            e.set_partition(1, 2)


@pytest.mark.parametrize("mode", MODES, ids=MODE_IDS)
def test_edge_cases(pkg, oracle, mode):
    push_ratio, unfiltered_pct, flat_max_words, arc_mask = mode
    # isolated vertices, a single message, origin that crashes before injection
    g = pkg.CSR.from_edges(50, [(0, 1), (1, 2), (2, 3), (10, 11)])
    kw = dict(push_ratio=push_ratio, unfiltered_pct=unfiltered_pct, flat_max_words=flat_max_words, arc_mask_permille=arc_mask)
    _compare(pkg, oracle, g, np.array([0], np.int32), **kw)["eng"].close()
    _compare(pkg, oracle, g, np.array([7, 7, 7], np.int32), **kw)["eng"].close()
    _compare(pkg, oracle, g, np.array([0, 10, 2], np.int32), np.array([0, 2, 4], np.int32),
             crashes=[(10, 1)], **kw)["eng"].close()
    # all messages at one origin of a star (hub receives nothing new after round 1)
    star = pkg.CSR.from_edges(200, [(0, i) for i in range(1, 200)])
    _compare(pkg, oracle, star, np.full(100, 5, np.int32), hub_threshold=64, **kw)["eng"].close()


@pytest.mark.parametrize("mode", MODES, ids=MODE_IDS)
def test_raw_csr_self_loops_and_repeated_arcs(pkg, oracle, mode):
    """An in-CSR loaded as given (gp_load_graph): self-loops and repeated arcs
    count as links in the sends (deg) but can never bring a vertex anything
    it does not hold; unsorted in-lists; W = 2 rows, hubs split at 64."""
    push_ratio, unfiltered_pct, flat_max_words, arc_mask = mode
    g0 = pkg.overlay.barabasi_albert(3000, 3, seed=41)
    rng = np.random.default_rng(41)
    src, dst = g0.arcs()
    loops = rng.choice(g0.n, 300, replace=False)
    again = rng.choice(src.size, 2000, replace=False)   # repeated arcs, both directions
    s = np.concatenate([src, loops, src[again], dst[again]])
    d = np.concatenate([dst, loops, dst[again], src[again]])
    order = rng.permutation(s.size)   # in-lists in no particular order
    s, d = s[order], d[order]
    rp = np.zeros(g0.n + 1, np.int64)
    np.add.at(rp, d + 1, 1)
    rp = np.cumsum(rp)
    col = np.empty(s.size, np.int32)
    cur = rp[:-1].copy()
    for u, v in zip(s.tolist(), d.tolist()):
        col[cur[v]] = u
        cur[v] += 1
    g = pkg.CSR(g0.n, rp, col, False)
    origin = pkg.overlay.random_origins(g.n, 100, seed=41)
    inject = (np.arange(100) % 3).astype(np.int32)
    kw = dict(push_ratio=push_ratio, unfiltered_pct=unfiltered_pct, flat_max_words=flat_max_words,
              arc_mask_permille=arc_mask, hub_threshold=64)
    _compare(pkg, oracle, g, origin, inject, **kw)["eng"].close()
    _compare(pkg, oracle, g, origin, inject, churn=True, p_fail=0.05, churn_seed=41, **kw)["eng"].close()


@pytest.mark.parametrize("p_fail", [0.3, 1.0])
@pytest.mark.parametrize("mode", MODES, ids=MODE_IDS)
def test_extreme_churn(pkg, oracle, mode, p_fail):
    """A third of the live vertices crash every round, or all of them at once:
    detection, removals and lost messages at their limits, W = 64 rows."""
    push_ratio, unfiltered_pct, flat_max_words, arc_mask = mode
    g = pkg.overlay.barabasi_albert(4000, 3, seed=43)
    origin = pkg.overlay.random_origins(g.n, 4096, seed=43)
    inject = (np.arange(4096) % 4).astype(np.int32)
    for track_fwd in (1, 0):
        _compare(pkg, oracle, g, origin, inject, first=False, track_fwd=track_fwd, churn=True, p_fail=p_fail,
                 churn_seed=43, push_ratio=push_ratio, unfiltered_pct=unfiltered_pct,
                 flat_max_words=flat_max_words, arc_mask_permille=arc_mask, hub_threshold=256)["eng"].close()


def test_full_size_invariants_c3(pkg):
    """Size-independent properties at a large size: conservation of sends and
    receipts, idempotence of a repeated run."""
    n, m = 1 << 20, 4096
    with pkg.GossipEngine(0, track_digest=1) as eng:
        eng.build_chung_lu(n, 16, 2.5, 4)
        origin = pkg.overlay.random_origins(n, m, seed=4)
        eng.set_messages(origin)
        eng.reset()
        s1 = eng.run()
        d1 = eng.digest().copy()
        eng.finalize()
        cov, fwd = eng.coverage(), eng.forwards()
        eng.reset()
        s2 = eng.run()
        d2 = eng.digest()
    assert np.array_equal(d1, d2)
    assert [x["new_bits"] for x in s1] == [x["new_bits"] for x in s2]
    assert sum(x["sends"] for x in s1) == int(fwd.sum())
    assert sum(x["new_bits"] + x["injected"] for x in s1) == int(cov.sum())


@pytest.mark.parametrize("mode", MODES, ids=MODE_IDS)
def test_wide_rows_churn(pkg, oracle, mode):
    """W = 64 (4096 messages), injections spread over rounds, churn: exercises
    the Message-List slots through pull, push, injection into a sender's row,
    the exact frontier rows kept for per-message forwards, and hub splits."""
    push_ratio, unfiltered_pct, flat_max_words, arc_mask = mode
    rp, col = oracle.chung_lu(60_000, 10, 2.4, 21)
    g = pkg.CSR(60_000, rp, col, False)
    m = 4096
    origin = pkg.overlay.random_origins(g.n, m, seed=21)
    inject = (np.arange(m) % 6).astype(np.int32)
    cfg_first = push_ratio != 10.0   # first matrix on three of the four modes (1 GB host copy otherwise)
    churn = dict(churn=True, p_fail=0.01, churn_seed=5)
    r = _compare(pkg, oracle, g, origin, inject, first=cfg_first, hub_threshold=512, push_ratio=push_ratio,
                 unfiltered_pct=unfiltered_pct, flat_max_words=flat_max_words, arc_mask_permille=arc_mask, **churn)
    if push_ratio == 0.0:   # unfiltered under liveness: crashed rows parked first
        assert any(s["scan"] == 2 for s in r["stats"]) == (unfiltered_pct == 1)
    r["eng"].close()


@pytest.mark.parametrize("schedule", ["round0", "spread"])
@pytest.mark.parametrize("m", [4096, 2048])
@pytest.mark.parametrize("mode", [MODES[0], MODES[2], MODES[4]], ids=["pull", "pull-unfiltered", "adaptive"])
def test_sated_vertices(pkg, oracle, schedule, m, mode):
    """Sated vertices: under churn, once no injection is
    left, a receiver that ends an early-exit round holding every alive message
    of its component is skipped by every later pull (the alive sets only
    shrink).  All injections at round 0 (sated from the first early-exit
    round on) or spread over rounds 0-2; outputs equal the oracle's
    (Peer.py:298-313 liveness, Seed.py:358-406 removal, forward-once)."""
    push_ratio, unfiltered_pct, flat_max_words, arc_mask = mode
    rp, col = oracle.chung_lu(40_000, 12, 2.4, 31)
    g = pkg.CSR(40_000, rp, col, False)
    origin = pkg.overlay.random_origins(g.n, m, seed=31)
    inject = np.zeros(m, np.int32) if schedule == "round0" else (np.arange(m) % 3).astype(np.int32)
    r = _compare(pkg, oracle, g, origin, inject, first=False, hub_threshold=256, push_ratio=push_ratio,
                 unfiltered_pct=unfiltered_pct, flat_max_words=flat_max_words, arc_mask_permille=arc_mask,
                 churn=True, p_fail=0.02, churn_seed=7)
    r["eng"].close()


@pytest.mark.parametrize("mode", MODES, ids=MODE_IDS)
@pytest.mark.parametrize("m", [4096, 2048])
def test_lost_messages_drop_from_targets(pkg, oracle, mode, m):
    """Messages whose origin is down at the inject round are dropped from the
    early-exit targets of their component for that run (k_lost_clear,
    k_done_fix), and late rounds narrow the targets to the alive messages
    (SCAN_ALIVE variants at W = 64 and 32): the run stays bit-exact, and
    gp_reset restores the targets, so repeated runs on one context are
    identical."""
    push_ratio, unfiltered_pct, flat_max_words, arc_mask = mode
    rp, col = oracle.chung_lu(40_000, 10, 2.4, 23)
    g = pkg.CSR(40_000, rp, col, False)
    origin = pkg.overlay.random_origins(g.n, m, seed=23)
    inject = (np.arange(m) % 5).astype(np.int32)
    crashes = [(int(v), int(r)) for v, r in zip(origin[:300], inject[:300])]   # down when injected
    r = _compare(pkg, oracle, g, origin, inject, crashes=crashes, first=False, push_ratio=push_ratio,
                 unfiltered_pct=unfiltered_pct, flat_max_words=flat_max_words, arc_mask_permille=arc_mask,
                 churn=True, p_fail=0.02, churn_seed=9)
    assert sum(s["lost"] for s in r["stats"]) >= 300
    eng, ref = r["eng"], r["ref"]
    by_round = {}
    for v, rr in crashes:
        by_round.setdefault(rr, []).append(v)
    for _ in range(2):
        eng.reset()
        stats = []
        for rr in range(len(ref["stats"])):
            if rr in by_round:
                eng.crash(by_round[rr])
            stats.append(eng.round())
        assert [s["new_bits"] for s in stats] == [s["new_bits"] for s in ref["stats"]]
        assert [s["lost"] for s in stats] == [s["lost"] for s in ref["stats"]]
        assert np.array_equal(eng.digest(), ref["digest"])
    eng.close()


@pytest.mark.parametrize("mode", MODES, ids=MODE_IDS)
@pytest.mark.parametrize("stop,p_fail", [(1, 0.01), (3, 0.01), (2, 0.0), (4, 0.0)])
def test_checkpoint_restore_continues_exactly(pkg, oracle, mode, stop, p_fail, tmp_path):
    """gp_checkpoint_save after `stop` rounds, then (a) the same context runs
    on, (b) a fresh context loads the .npz and runs on, (c) the first context
    loads it again after finishing and re-runs the tail: all three match the
    oracle's uninterrupted run bit for bit (counters, Message-Lists, first
    receipts, digests, per-message coverage/forwards, dead-node reports)."""
    push_ratio, unfiltered_pct, flat_max_words, arc_mask = mode
    rp, col = oracle.chung_lu(30_000, 10, 2.4, 31)
    g = pkg.CSR(30_000, rp, col, False)
    m = 4096
    origin = pkg.overlay.random_origins(g.n, m, seed=31)
    inject = (np.arange(m) % 5).astype(np.int32)
    kw = dict(churn=p_fail > 0, p_fail=p_fail, churn_seed=13)
    cfg = dict(track_first=1, track_digest=1, track_msg_forwards=1, churn=int(p_fail > 0), p_fail=p_fail,
               churn_seed=13, push_ratio=push_ratio, unfiltered_pct=unfiltered_pct,
               flat_max_words=flat_max_words, arc_mask_permille=arc_mask, compact_rows=1)
    ref = oracle.run(g, origin, inject, want_first=True, **kw)

    def tail(eng):
        stats, reports = [], []
        while True:
            st = eng.round()
            stats.append(st)
            rep, _ = eng.reports()
            reports.extend(map(tuple, rep.tolist()))
            if st["new_bits"] == 0 and st["round"] >= 4:
                return stats, reports

    def check(eng, stats, reports):
        assert len(stats) == ref["rounds"] - stop
        for a, b in zip(stats, ref["stats"][stop:]):
            for k in STAT_KEYS:
                assert a[k] == b[k], (k, a["round"], a[k], b[k])
        eng.finalize()
        assert np.array_equal(eng.seen(), ref["seen"][:, :eng.words])
        assert np.array_equal(eng.first(), ref["first"])
        assert np.array_equal(eng.digest(), ref["digest"])
        assert np.array_equal(eng.coverage(), ref["coverage"])
        assert np.array_equal(eng.forwards(), ref["forwards"])
        ref_tail = [tuple(x) for x in ref["reports"].tolist() if x[2] >= stop]
        assert sorted(reports) == sorted(ref_tail)

    a = _engine(pkg, g, origin, inject, **cfg)
    for _ in range(stop):
        a.round()
    saved_reports = sorted(map(tuple, a.reports()[0].tolist()))
    path = tmp_path / "ck.npy"
    a.save_checkpoint(path)
    check(a, *tail(a))
    b = _engine(pkg, g, origin, inject, **cfg)
    b.load_checkpoint(path)
    # the reports of the round the checkpoint was taken after come back too
    assert sorted(map(tuple, b.reports()[0].tolist())) == saved_reports
    check(b, *tail(b))
    b.close()
    a.load_checkpoint(path)
    check(a, *tail(a))
    a.close()


@pytest.mark.parametrize("mode", MODES, ids=MODE_IDS)
def test_wide_rows_no_churn(pkg, oracle, mode):
    """W = 64 without liveness: unfiltered dense rounds read whole Message-List
    rows of every in-neighbour (stale slots zeroed by k_fixup_rows); repeated
    runs on one context reuse the unclear slot buffers."""
    push_ratio, unfiltered_pct, flat_max_words, arc_mask = mode
    rp, col = oracle.chung_lu(60_000, 10, 2.4, 22)
    g = pkg.CSR(60_000, rp, col, False)
    m = 4096
    origin = pkg.overlay.random_origins(g.n, m, seed=22)
    inject = (np.arange(m) % 4).astype(np.int32)
    r = _compare(pkg, oracle, g, origin, inject, first=False, push_ratio=push_ratio,
                 unfiltered_pct=unfiltered_pct, flat_max_words=flat_max_words, arc_mask_permille=arc_mask)
    if unfiltered_pct == 1:
        assert any(s["scan"] == 2 for s in r["stats"])
    eng, ref = r["eng"], r["ref"]
    for _ in range(2):   # stale rows of the previous run must not leak in
        eng.reset()
        stats = eng.run()
        assert [s["new_bits"] for s in stats] == [s["new_bits"] for s in ref["stats"]]
        assert np.array_equal(eng.digest(), ref["digest"])
    eng.close()


@pytest.mark.parametrize("split_deg", [1, 8, 128, 1 << 20])
@pytest.mark.parametrize("m,flat_max_words", [(4096, 16), (2048, 16), (512, 0), (512, 16), (64, 16)])
@pytest.mark.parametrize("churn", [False, True])
def test_degree_split(pkg, oracle, split_deg, m, flat_max_words, churn):
    """Degree-split sparse rounds: in a prefiltered pull
    without early exit, senders of in-degree < split_deg push their rows into
    the accumulator (k_active_list filter, k_push / k_push_big) and receivers
    probe only the prefix of their gather-ordered in-list whose senders have
    in-degree >= split_deg; a touched receiver's accumulator row is one more
    staged row (hubs: k_hub_final), and k_acc_clear re-zeroes it.  From
    nothing pushed (1) to everything pushed (2^20), per-receiver kernel at
    W = 64 / 32 / 8 and the edge-parallel kernel at W = 8 / 1 (whose receiver
    side ORs the accumulator rows), hubs split over waves, with and without
    churn: the run equals the oracle's (scan bit 32 marks the split rounds)."""
    rp, col = oracle.chung_lu(200_000, 10, 2.4, 61)
    g = pkg.CSR(200_000, rp, col, False)
    origin = pkg.overlay.random_origins(g.n, m, seed=61)
    inject = (np.arange(m) % 2).astype(np.int32)
    kw = dict(churn=True, p_fail=0.01, churn_seed=9) if churn else {}
    r = _compare(pkg, oracle, g, origin, inject, first=False, hub_threshold=512, push_ratio=1000.0,
                 unfiltered_pct=90, flat_max_words=flat_max_words, arc_mask_permille=0, prefilter_pct=20,
                 compact_rows=0, split_deg=split_deg, split_max_permille=1000, **kw)
    scans = [s["scan"] for s in r["stats"]]
    assert any(x & 32 for x in scans), scans
    assert all((x & 3) == 3 for x in scans if x & 32), scans
    r["eng"].close()


@pytest.mark.parametrize("push_ratio", [0.0, 100.0], ids=["pull", "adaptive"])
@pytest.mark.parametrize("schedule", ["round0", "staggered"])
def test_line_masks(pkg, oracle, push_ratio, schedule):
    """64-word line masks: filtered pulls without early exit
    gather only the 128-B lines a sender's nibble names.  The masks come from
    k_mklm or, in one context without liveness, from the previous round's
    commits (finish_row / pair_finish ballots, hub receivers OR-ed in after
    the pull, k_inject's nibbles of the next round's origins): round stats'
    scan bit 8 = masks read, 16 = masks from the commits.  Both paths must
    run here, with hubs split over waves and staggered injections, and the
    run must equal the oracle's."""
    rp, col = oracle.chung_lu(120_000, 12, 2.4, 52)
    g = pkg.CSR(120_000, rp, col, False)
    m = 4096
    origin = pkg.overlay.random_origins(g.n, m, seed=52)
    inject = None if schedule == "round0" else (np.arange(m) % 3).astype(np.int32)
    r = _compare(pkg, oracle, g, origin, inject, first=False, hub_threshold=256, push_ratio=push_ratio,
                 unfiltered_pct=90, flat_max_words=16, arc_mask_permille=0, prefilter_pct=0, compact_rows=0)
    scans = [s["scan"] for s in r["stats"]]
    assert any(x & 8 for x in scans), scans
    assert any(x & 16 for x in scans), scans
    assert all(x & 8 for x in scans if x & 16), scans
    r["eng"].close()


@pytest.mark.parametrize("m,flat_max_words", [(4096, 16), (2048, 16), (512, 0), (64, 0)])
def test_done_in_neighbours(pkg, oracle, m, flat_max_words):
    """Late early-exit rounds without liveness: a receiver whose first in-arcs
    (gather order, hubs first) come from a vertex that held its whole component
    at the end of the last round takes cmask & ~seen without gathering a row
    (done_nb counts them; W = 64 two or four per wave step, W = 32 four per
    step, one per 16-lane group (dnb_groups), narrower rows in the
    per-receiver kernel's serial loop).  Bit-exact against the oracle,
    first-receipt matrix included."""
    rp, col = oracle.chung_lu(150_000, 12, 2.5, 41)
    g = pkg.CSR(150_000, rp, col, False)
    origin = pkg.overlay.random_origins(g.n, m, seed=41)
    r = _compare(pkg, oracle, g, origin, flat_max_words=flat_max_words)
    dnb = [s["done_nb"] for s in r["stats"]]
    assert sum(dnb) > 0, dnb
    for s in r["stats"]:   # only pulls of rounds once most messages are held
        assert s["done_nb"] == 0 or (s["mode"] == 0 and s["done_nb"] <= s["vertices_visited"])
    r["eng"].close()


@pytest.mark.parametrize("m", [1024, 512])
@pytest.mark.parametrize("mode", [MODES[0], MODES[2]], ids=["pull", "pull-unfiltered"])
def test_narrow_late_rounds_per_receiver(pkg, oracle, m, mode):
    """W = 16 / 8 rows (the message shards of 4- and 8-GPU jobs) run on the
    flat kernel, except the thin late rounds (under n*m/16 bits missing),
    which take the per-receiver kernel with receivers in groups of 8 / 16
    per wave step (dnb_groups, gather_groups): done-neighbour receivers can
    only show up there.  Bit-exact against the oracle, first-receipt matrix
    included."""
    push_ratio, unfiltered_pct, _, arc_mask = mode
    rp, col = oracle.chung_lu(150_000, 12, 2.5, 43)
    g = pkg.CSR(150_000, rp, col, False)
    origin = pkg.overlay.random_origins(g.n, m, seed=43)
    r = _compare(pkg, oracle, g, origin, push_ratio=push_ratio, unfiltered_pct=unfiltered_pct,
                 flat_max_words=16, arc_mask_permille=arc_mask)
    dnb = [s["done_nb"] for s in r["stats"]]
    assert sum(dnb) > 0, dnb
    r["eng"].close()


@pytest.mark.parametrize("hops", [1, 2, 3])
def test_spread_keys_match_host(pkg, oracle, hops):
    """gp_spread_keys (device) equals overlay.spread_keys (host), u64-exact, on
    a Chung-Lu overlay with hubs, repeated origins and isolated vertices."""
    rp, col = oracle.chung_lu(80_000, 10, 2.3, 44)
    g = pkg.CSR(80_000, rp, col, False)
    origin = pkg.overlay.random_origins(g.n, 3000, seed=44)
    origin[:5] = np.argsort(-np.diff(rp))[:5]                # the top hubs
    iso = np.nonzero(np.diff(rp) == 0)[0]
    if iso.size:
        origin[5] = iso[0]
    origin[6] = origin[7]
    with pkg.GossipEngine(0) as eng:
        eng.load_graph(g)
        assert np.array_equal(eng.spread_keys(origin, hops), pkg.overlay.spread_keys(rp, col, origin, hops))
        with pytest.raises(pkg.GossipError):
            eng.spread_keys(origin, 4)


@pytest.mark.parametrize("mode", [MODES[0], MODES[2], MODES[4]], ids=["pull", "pull-unfiltered", "adaptive"])
@pytest.mark.parametrize("churn", [False, True])
def test_spread_order_is_a_relabelling(pkg, oracle, mode, churn):
    """The spread order only relabels messages: the engine's
    run of the ordered table equals the oracle's run of that table (first
    matrix, digests, counters), and its per-message outputs are those of the
    given order, permuted -- coverage, forwards and first-matrix columns; sends
    and receipts per round are unchanged.  Late rounds load fewer row bytes."""
    push_ratio, unfiltered_pct, flat_max_words, arc_mask = mode
    rp, col = oracle.chung_lu(120_000, 12, 2.5, 45)
    g = pkg.CSR(120_000, rp, col, False)
    origin = pkg.overlay.random_origins(g.n, 4096, seed=45)
    kw = dict(churn=True, p_fail=0.01, churn_seed=5) if churn else {}
    base = _compare(pkg, oracle, g, origin, first=True, push_ratio=push_ratio, unfiltered_pct=unfiltered_pct,
                    flat_max_words=flat_max_words, arc_mask_permille=arc_mask, **kw)
    perm = base["eng"].spread_order(origin)
    assert sorted(perm.tolist()) == list(range(origin.size)) and not np.array_equal(perm, np.arange(origin.size))
    ordered = _compare(pkg, oracle, g, origin[perm], first=True, push_ratio=push_ratio,
                       unfiltered_pct=unfiltered_pct, flat_max_words=flat_max_words, arc_mask_permille=arc_mask,
                       **kw)
    a, b = base["eng"], ordered["eng"]
    assert [s["new_bits"] for s in base["stats"]] == [s["new_bits"] for s in ordered["stats"]]
    assert [s["sends"] for s in base["stats"]] == [s["sends"] for s in ordered["stats"]]
    assert np.array_equal(b.coverage(), a.coverage()[perm])
    assert np.array_equal(b.forwards(), a.forwards()[perm])
    assert np.array_equal(b.first(), a.first()[:, perm])
    if not churn and unfiltered_pct == 90:
        assert sum(s["row_bytes"] for s in ordered["stats"]) < sum(s["row_bytes"] for s in base["stats"])
    a.close()
    b.close()


@pytest.mark.parametrize("prefilter", [0, 20])
@pytest.mark.parametrize("churn", [False, True])
def test_compact_message_lists(pkg, oracle, prefilter, churn):
    """W = 64, every message injected at round 0 on a sparse overlay: the early
    rounds gather senders from compact Message-Lists (scan bit 4): without the
    prefilter through the flat record pull (k_expand_rec, 8 receivers per wave,
    4 record instructions in flight), with it through the per-receiver loop;
    with churn (exact frontier rows, alive sets); results are those of the
    oracle (first-receipt matrix included) and of a run with compact rows off."""
    rp, col = oracle.chung_lu(200_000, 8, 2.5, 31)
    g = pkg.CSR(200_000, rp, col, False)
    origin = pkg.overlay.random_origins(g.n, 4096, seed=31)
    kw = dict(churn=True, p_fail=0.01, churn_seed=3) if churn else {}
    # no hub splits: in early-exit rounds a split hub's chunks stop once one
    # of them covers the target (hub_done), so how much the chunks scan -- the
    # work counters compared below, not the rows -- depends on wave timing
    hub = max(4096, int(np.diff(rp).max()) + 1)
    r = _compare(pkg, oracle, g, origin, first=True, push_ratio=0.0, prefilter_pct=prefilter, arc_mask_permille=0,
                 compact_rows=1, hub_threshold=hub, **kw)
    assert any(s["scan"] & 4 for s in r["stats"])
    assert any((s["scan"] & 3) == (3 if prefilter else 0) and s["scan"] & 4 for s in r["stats"])
    r["eng"].close()
    if churn:
        return
    # (the same work without records: degree-split rounds off, as record rounds never split)
    with pkg.GossipEngine(0, track_digest=1, push_ratio=0.0, prefilter_pct=prefilter, compact_rows=0,
                          arc_mask_permille=0, unfiltered_pct=90, flat_max_words=16, hub_threshold=hub,
                          split_deg=0) as eng:
        eng.load_graph(g)
        eng.set_messages(origin)
        eng.reset()
        stats = eng.run()
        assert not any(s["scan"] & 4 for s in stats)
        # (without records the late rounds alias complete receivers instead of
        # writing their rows, and once aliases exist every scanned arc probes
        # the done bitmap, which can stop a scan before the early exit would)
        for a, b in zip(stats, r["stats"]):
            for k in STAT_KEYS:
                assert a[k] == b[k], k
            assert a["rows_written"] + a["aliased"] == b["rows_written"] and b["aliased"] == 0
            if not a["scan"] & 64:
                for k in ("rows_gathered", "arcs_scanned"):
                    assert a[k] == b[k], k
        assert np.array_equal(eng.digest(), r["ref"]["digest"])


@pytest.mark.parametrize("shards", [2, 4])
@pytest.mark.parametrize("churn", [False, True])
def test_message_shards_match_whole_run(pkg, shards, churn):
    """Message shards on one GPU, one context each: the per-round
    sends and new bits add up to the whole run's, coverage / forwards / first
    columns concatenate, and the shard digests XOR to the whole run's digest.
    With churn every shard draws the same crashes and reports (liveness is
    replicated) and runs its own alive sets."""
    rp, col = pkg_oracle_chung_lu(20_000, 8, 2.4, 13)
    g = pkg.CSR(20_000, rp, col, False)
    m = 1024
    origin = pkg.overlay.random_origins(g.n, m, seed=13)
    inject = (np.arange(m) % 3).astype(np.int32)

    def run(lo, hi):
        cfg = dict(churn=1, p_fail=0.02, churn_seed=7, track_msg_forwards=1) if churn else {}
        eng = pkg.GossipEngine(0, track_first=1, track_digest=1, **cfg)
        eng.load_graph(g)
        eng.set_message_shard(origin, inject, lo, hi)
        eng.reset()
        stats = eng.run()
        eng.finalize()
        out = (stats, eng.first(), eng.digest(), eng.coverage(), eng.forwards())
        eng.close()
        return out

    whole = run(0, m)
    parts = [run(*pkg.dist.message_shard(m, shards, r)) for r in range(shards)]
    for i, s in enumerate(whole[0]):
        for k in ("new_bits", "sends", "injected"):
            assert s[k] == sum(p[0][i][k] if i < len(p[0]) else 0 for p in parts), (k, i)
        for p in parts:
            if i < len(p[0]):
                for k in ("crashed", "reports", "removals"):
                    assert p[0][i][k] == s[k], (k, i)
    if churn:
        assert sum(s["removals"] for s in whole[0]) > 0
    assert np.array_equal(np.concatenate([p[1] for p in parts], axis=1), whole[1])
    dig = np.zeros_like(whole[2])
    for p in parts:
        dig ^= p[2]
    assert np.array_equal(dig, whole[2])
    assert np.array_equal(np.concatenate([p[3] for p in parts]), whole[3])
    assert np.array_equal(np.concatenate([p[4] for p in parts]), whole[4])


def pkg_oracle_chung_lu(n, dbar, gamma, seed):
    from oracle import lib as oracle
    return oracle.chung_lu(n, dbar, gamma, seed)


@pytest.mark.parametrize("prefilter", [0, 20])
@pytest.mark.parametrize("churn", [False, "frontier-rows", "bench-c5"])
def test_summary_probes(pkg, oracle, prefilter, churn):
    """Summary-level activity probes (one bit per 64 vertices read before the
    bitmap word) forced on at any size: sparse filtered pull rounds, with and
    without the lane-parallel prefilter, per-receiver kernel, with churn (with
    and without exact frontier rows: bench.py's C5 runs without)."""
    rp, col = oracle.chung_lu(200_000, 8, 2.5, 21)
    g = pkg.CSR(200_000, rp, col, False)
    origin = pkg.overlay.random_origins(g.n, 256, seed=21)
    inject = (np.arange(256) % 6).astype(np.int32)
    kw = dict(churn=True, p_fail=0.01, churn_seed=5) if churn else {}
    if churn:
        kw["track_fwd"] = int(churn == "frontier-rows")
    r = _compare(pkg, oracle, g, origin, inject, push_ratio=0.0, flat_max_words=0, arc_mask_permille=0,
                 prefilter_pct=prefilter, compact_rows=0, summary_min_n=1, **kw)
    # the summary path runs in filtered pull rounds with <= n/256 senders
    assert any(s["mode"] == 0 and s["scan"] != 2 and s["active"] * 256 <= g.n for s in r["stats"])
    r["eng"].close()


def test_checkpoint_rejected_blob_leaves_run_intact(pkg, oracle, tmp_path):
    """A blob of another configuration (tracked outputs, partition, message
    set) is rejected before anything is reset: the run in progress continues
    exactly as if the load had never been tried."""
    rp, col = oracle.chung_lu(20_000, 8, 2.4, 41)
    g = pkg.CSR(20_000, rp, col, False)
    origin = pkg.overlay.random_origins(g.n, 512, seed=41)
    inject = (np.arange(512) % 3).astype(np.int32)
    kw = dict(churn=True, p_fail=0.02, churn_seed=4)
    cfg = dict(track_first=1, track_digest=1, track_msg_forwards=1, churn=1, p_fail=0.02, churn_seed=4)
    ref = oracle.run(g, origin, inject, want_first=True, **kw)
    other = []
    e = _engine(pkg, g, origin, inject, **dict(cfg, track_first=0))   # other tracked outputs
    e.round()
    other.append(e.checkpoint())
    e.close()
    e = _engine(pkg, g, origin[:300], inject[:300], **cfg)             # other message set
    e.round()
    other.append(e.checkpoint())
    e.close()
    e = pkg.GossipEngine(0, **cfg)                                      # other partition
    e.load_graph(g)
    e.set_partition(1, 2)
    e.set_messages(origin, inject)
    e.reset()
    other.append(e.checkpoint())
    e.close()
    a = _engine(pkg, g, origin, inject, **cfg)
    stats = [a.round(), a.round()]
    for blob in other + [np.zeros(64, np.uint8)]:
        with pytest.raises(pkg.GossipError):
            a.restore(blob)
    while True:
        st = a.round()
        stats.append(st)
        if st["new_bits"] == 0 and st["round"] >= 2:
            break
    assert len(stats) == ref["rounds"]
    for x, y in zip(stats, ref["stats"]):
        for k in STAT_KEYS:
            assert x[k] == y[k], (k, x["round"])
    a.finalize()
    assert np.array_equal(a.first(), ref["first"])
    assert np.array_equal(a.digest(), ref["digest"])
    assert np.array_equal(a.forwards(), ref["forwards"])
    a.close()


@pytest.mark.parametrize("m,churn", [(64, None), (1000, None), (4096, None), (300, "random"), (4096, "random"),
                                     (200, "few"), (4096, "few")])
def test_finalize_paths_agree(pkg, oracle, m, churn, monkeypatch):
    """gp_finalize_messages through the component targets (complete vertices
    add their component's mask row; a few incomplete rows -- explicit crashes --
    bit by bit from a list; many -- random churn -- the bit-sliced pass over
    every row) against the bit-sliced pass forced (GP_FINALIZE_ROWS=1) and the
    oracle, at widths 1..64."""
    g = pkg.overlay.barabasi_albert(3000, 2, seed=11)
    origin = pkg.overlay.random_origins(g.n, m, seed=11)
    cfg = dict(track_digest=1)
    okw = {}
    crashes = []
    if churn == "random":
        cfg.update(churn=1, p_fail=0.02, churn_seed=7, track_msg_forwards=1)
        okw = dict(churn=True, p_fail=0.02, churn_seed=7)
    elif churn == "few":
        cfg.update(track_msg_forwards=1)
        crashes = [(int(v), 2) for v in range(100, 3000, 300)]
        okw = dict(crashes=crashes)
    with pkg.GossipEngine(0, **cfg) as eng:
        eng.load_graph(g)
        eng.set_messages(origin)
        eng.reset()
        for r in range(254):
            if crashes and r == 2:
                eng.crash([v for v, _ in crashes])
            st = eng.round()
            if st["new_bits"] == 0 and r >= 0:
                break
        monkeypatch.delenv("GP_FINALIZE_ROWS", raising=False)
        eng.finalize()
        cov_c, fwd_c = eng.coverage(), eng.forwards()
        monkeypatch.setenv("GP_FINALIZE_ROWS", "1")
        eng.finalize()
        cov_r, fwd_r = eng.coverage(), eng.forwards()
        monkeypatch.delenv("GP_FINALIZE_ROWS")
    ref = oracle.run(g, origin, **okw)
    assert np.array_equal(cov_c, ref["coverage"]) and np.array_equal(cov_r, ref["coverage"])
    assert np.array_equal(fwd_c, ref["forwards"]) and np.array_equal(fwd_r, ref["forwards"])


# (push_ratio, unfiltered_pct, hub_threshold): pull with the activity probe;
# unfiltered dense rounds; adaptive direction (the last rounds push: their
# aliased senders are materialized first); hubs split over waves (their chunks
# probe the done bitmap too)
ALIAS_MODES = {"pull": (0.0, 0, 1 << 30), "unfiltered": (0.0, 50, 1 << 30), "adaptive": (10.0, 90, 4096),
               "hubs": (0.0, 90, 256)}


@pytest.mark.parametrize("mode", list(ALIAS_MODES))
def test_aliased_message_lists(pkg, oracle, mode):
    """W = 64 early-exit rounds with the done bitmap, no liveness, one context
    (DESIGN.md §3.2): every arc the pull scans probes the done bitmap, and a
    receiver that completes its component commits SLOT_CMASK instead of a
    512-B row.  The run equals the oracle's: counters, first receipts,
    digests, coverage / forwards and every Message-List (gp_read writes the
    aliased rows it returns).  Reference: each peer's Message-List,
    Peer.py:175-216."""
    push_ratio, unfiltered_pct, hub = ALIAS_MODES[mode]
    rp, col = oracle.chung_lu(120_000, 12, 2.4, 41)
    g = pkg.CSR(120_000, rp, col, False)
    origin = pkg.overlay.random_origins(g.n, 4096, seed=41)
    r = _compare(pkg, oracle, g, origin, first=True, push_ratio=push_ratio, unfiltered_pct=unfiltered_pct,
                 hub_threshold=hub, arc_mask_permille=0, compact_rows=0)
    st = r["stats"]
    assert sum(s["aliased"] for s in st) > 0
    assert any(s["scan"] & 64 for s in st)
    for s in st:   # aliased receivers write no row
        if s["scan"] & 64:
            assert s["rows_written"] + s["aliased"] <= s["receivers"]
    if mode == "adaptive":
        k = max(i for i, s in enumerate(st) if s["aliased"])
        assert any(s["mode"] == 1 for s in st[k + 1:]), "no push round after aliasing"
    if mode == "pull":   # the last pulls take their receivers from the list the one before left
        assert any(s["scan"] & 128 for s in st)
    r["eng"].close()


@pytest.mark.parametrize("push_ratio", [0.0, 10.0])
@pytest.mark.parametrize("track_fwd", [0, 1])
def test_receiver_lists_under_churn(pkg, oracle, push_ratio, track_fwd):
    """Late W = 64 early-exit pulls under liveness: each
    appends its receivers that are neither sated nor complete, and a pull
    whose list is short launches waves for the listed vertices alone
    (SCAN_LIST, scan bit 128) while k_mkbits counts every sender's sends.
    Counters, first receipts, digests, coverage and the dead-node reports
    equal the oracle's (Peer.py:298-313, Seed.py:387-391: crashes, 3-miss
    detection and removal every round)."""
    rp, col = oracle.chung_lu(150_000, 12, 2.4, 47)
    g = pkg.CSR(150_000, rp, col, False)
    origin = pkg.overlay.random_origins(g.n, 4096, seed=47)
    r = _compare(pkg, oracle, g, origin, first=True, push_ratio=push_ratio, compact_rows=0, arc_mask_permille=0,
                 track_fwd=track_fwd, churn=True, p_fail=0.01, churn_seed=9)
    assert any(s["scan"] & 128 for s in r["stats"])
    r["eng"].close()


def test_aliased_rows_materialize_for_every_reader(pkg, oracle, monkeypatch, tmp_path):
    """Readers of Message-List rows outside the probing pulls see the rows the
    aliases stand for: the bit-sliced finalize over every row
    (GP_FINALIZE_ROWS=1), a checkpoint taken right after the first aliasing
    round and continued in a fresh context, and a crash injected after it
    (liveness turns on, the rest of the run keeps no alias)."""
    rp, col = oracle.chung_lu(60_000, 12, 2.4, 43)
    g = pkg.CSR(60_000, rp, col, False)
    origin = pkg.overlay.random_origins(g.n, 4096, seed=43)
    cfg = dict(track_first=1, track_digest=1, push_ratio=0.0, compact_rows=0, arc_mask_permille=0)
    ref = oracle.run(g, origin, None, want_first=True)

    def finish(eng, stats, ref):
        while True:
            s = eng.round()
            stats.append(s)
            if s["new_bits"] == 0:
                break
        eng.finalize()
        assert len(stats) == ref["rounds"]
        for a, b in zip(stats, ref["stats"]):
            for k in STAT_KEYS:
                assert a[k] == b[k], (k, a["round"])
        assert np.array_equal(eng.first(), ref["first"])
        assert np.array_equal(eng.digest(), ref["digest"])
        assert np.array_equal(eng.coverage(), ref["coverage"])
        assert np.array_equal(eng.forwards(), ref["forwards"])
        assert np.array_equal(eng.seen(), ref["seen"][:, :eng.words])

    # the row-by-row finalize
    monkeypatch.setenv("GP_FINALIZE_ROWS", "1")
    with _engine(pkg, g, origin, **cfg) as e:
        finish(e, [], ref)
    monkeypatch.delenv("GP_FINALIZE_ROWS")
    # checkpoint after the first aliasing round, continued elsewhere
    with _engine(pkg, g, origin, **cfg) as e:
        stats = []
        while not stats or not stats[-1]["aliased"]:
            stats.append(e.round())
        path = tmp_path / "alias.npy"
        e.save_checkpoint(path)
        with _engine(pkg, g, origin, **cfg) as f:
            f.load_checkpoint(path)
            finish(f, list(stats), ref)
        finish(e, stats, ref)
    # a crash after aliasing: the oracle's run with the same crash
    with _engine(pkg, g, origin, track_msg_forwards=1, **cfg) as e:
        stats = []
        while not stats or not stats[-1]["aliased"]:
            stats.append(e.round())
        r0 = len(stats)
        e.crash([int(origin[0]), 7])
        ref2 = oracle.run(g, origin, None, crashes=[(int(origin[0]), r0), (7, r0)], want_first=True)
        finish(e, stats, ref2)
