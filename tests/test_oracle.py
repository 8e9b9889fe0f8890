"""The two CPU restatements (C oracle, per-peer sha256 harness) agree with each
other on every output, the overlay generators match their published
definitions, and the digest is a function of the first-receipt matrix."""
import numpy as np
import pytest

KEYS = ("injected", "lost", "new_bits", "receivers", "sends", "active", "crashed", "reports",
        "removals", "dup_reports")


def _both(pkg, oracle, harness, g, origin, inject, **kw):
    ref = oracle.run(g, origin, inject, want_first=True, **kw)
    in_lists = [g.in_neighbors(v).tolist() for v in range(g.n)]
    h = harness.run(g.n, in_lists, g.directed, list(map(int, origin)), list(map(int, inject)), **kw)
    assert h["rounds"] == ref["rounds"]
    for a, b in zip(h["stats"], ref["stats"]):
        assert a == b
    assert np.array_equal(h["first"], ref["first"])
    assert np.array_equal(h["coverage"], ref["coverage"])
    assert np.array_equal(h["forwards"], ref["forwards"])
    assert sorted(h["reports"]) == sorted(map(tuple, ref["reports"].tolist()))
    return ref


CASES = [
    ("ba", dict()),
    ("ba", dict(churn=True, p_fail=0.04, churn_seed=5)),
    ("ba", dict(crashes=[(3, 0), (11, 2), (0, 4)])),
    ("c1", dict()),
    ("c1", dict(crashes=[(4, 1), (0, 6), (9, 3)])),
    ("join", dict(churn=True, p_fail=0.02, churn_seed=1)),
    ("chunglu", dict(churn=True, p_fail=0.01, churn_seed=2)),
]


@pytest.mark.parametrize("kind,kw", CASES)
def test_oracle_equals_harness(pkg, oracle, harness, kind, kw):
    if kind == "ba":
        g = pkg.overlay.barabasi_albert(600, 2, seed=3)
        m = 100
        origin = pkg.overlay.random_origins(g.n, m, 3)
        inject = (np.arange(m) % 7).astype(np.int32)
    elif kind == "c1":
        g = pkg.first3_overlay(10)
        o, i, _ = pkg.peer.c1_schedule(10)
        origin, inject = np.array(o, np.int32), np.array(i, np.int32)
    elif kind == "join":
        g = pkg.overlay.powerlaw_join(400, 7)
        origin = pkg.overlay.random_origins(g.n, 64, 7)
        inject = np.zeros(64, np.int32)
    else:
        rp, col = oracle.chung_lu(3000, 6, 2.5, 9)
        g = pkg.CSR(3000, rp, col, False)
        origin = pkg.overlay.random_origins(g.n, 130, 9)
        inject = (np.arange(130) % 3).astype(np.int32)
    _both(pkg, oracle, harness, g, origin, inject, **kw)


def test_digest_is_function_of_first_matrix(pkg, oracle):
    g = pkg.overlay.barabasi_albert(500, 2, seed=4)
    m = 150
    origin = pkg.overlay.random_origins(g.n, m, 4)
    inject = (np.arange(m) % 4).astype(np.int32)
    ref = oracle.run(g, origin, inject, want_first=True)
    assert np.array_equal(oracle.digest_from_first(ref["first"], origin), ref["digest"])


def test_no_churn_totals(pkg, oracle):
    """Connected overlay, no churn: every message crosses every arc exactly once."""
    g = pkg.overlay.barabasi_albert(2000, 3, seed=1)
    origin = pkg.overlay.random_origins(g.n, 64, 1)
    ref = oracle.run(g, origin)
    assert sum(s["sends"] for s in ref["stats"]) == 64 * g.nnz
    assert np.all(ref["coverage"] == g.n)
    assert np.all(ref["forwards"] == g.nnz)


def test_chung_lu_oracle_matches_numpy_restatement(pkg, oracle):
    from oracle import graph_ref
    for n, dbar, gamma, seed in [(1000, 4, 2.5, 1), (5000, 8, 2.2, 7)]:
        rp, col = oracle.chung_lu(n, dbar, gamma, seed)
        rp2, col2 = graph_ref.chung_lu(n, dbar, gamma, seed)
        assert np.array_equal(rp, rp2)
        assert np.array_equal(col, col2)


def test_chung_lu_properties_and_degree_check(pkg, oracle):
    n = 200_000
    rp, col = oracle.chung_lu(n, 8, 2.5, 3)
    g = pkg.CSR(n, rp, col, False)
    src, dst = g.arcs()
    assert np.all(src != dst)
    fwd = set(zip(src[:20000].tolist(), dst[:20000].tolist()))
    rev = pkg.CSR.from_arcs(n, dst, src, directed=True)
    assert np.array_equal(rev.row_ptr, g.row_ptr) and np.array_equal(rev.col, g.col)   # symmetric
    assert len(fwd) == 20000   # de-duplicated
    for v in range(0, n, 9973):
        row = g.in_neighbors(v)
        assert np.all(np.diff(row) > 0)   # sorted, unique
    chk = pkg.degree.check_powerlaw(g.in_degree(), 2.5)
    assert chk["ok"], chk
    assert 7.0 < chk["mean_degree"] < 8.1


def test_ba_matches_networkx_and_degree_check(pkg):
    nx = pytest.importorskip("networkx")
    for n, m, s in [(100, 2, 0), (2000, 2, 2), (800, 3, 5)]:
        G = nx.barabasi_albert_graph(n, m, seed=s)
        ref = np.array(sorted((min(a, b), max(a, b)) for a, b in G.edges()))
        assert np.array_equal(pkg.overlay.barabasi_albert(n, m, s).edges_undirected(), ref)
    g = pkg.overlay.barabasi_albert(20_000, 2, 2)
    chk = pkg.degree.check_powerlaw(g.in_degree(), 3.0, tol=0.3)
    assert chk["ok"], chk


def test_csr_from_arcs(pkg):
    g = pkg.CSR.from_edges(5, [(0, 1), (1, 0), (1, 2), (2, 2), (3, 4), (3, 4)])
    assert g.nnz == 6
    assert g.in_neighbors(1).tolist() == [0, 2]
    assert g.in_neighbors(2).tolist() == [1]
    d = pkg.CSR.from_arcs(3, [0, 0, 1], [1, 2, 2], directed=True)
    assert d.in_neighbors(2).tolist() == [0, 1]
    assert d.out_degree().tolist() == [2, 1, 0]
    with pytest.raises(ValueError):
        pkg.CSR.from_edges(2, [(0, 5)])
