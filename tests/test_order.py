"""Message order: the host restatement of gp_spread_keys and
the ordering rule, on the CPU.  The device keys are checked against these in
tests/test_gpu_parity.py::test_spread_keys_match_host."""
import numpy as np
import pytest


def _brute(g, origin, hops):
    deg = np.diff(g.row_ptr)
    nb = lambda v, val: sum(int(val[u]) for u in g.col[g.row_ptr[v]:g.row_ptr[v + 1]])   # noqa: E731
    if hops == 1:
        return [int(deg[v]) for v in origin]
    if hops == 2:
        return [nb(v, deg) for v in origin]
    s2 = [nb(v, deg) for v in range(g.n)]
    return [nb(v, s2) for v in origin]


@pytest.mark.parametrize("hops", [1, 2, 3])
def test_spread_keys_host(pkg, hops):
    g = pkg.overlay.barabasi_albert(1500, 2, seed=7)
    # an isolated vertex at the end (empty trailing rows)
    g = pkg.CSR(g.n + 3, np.concatenate([g.row_ptr, [g.nnz] * 3]).astype(np.int64), g.col, False)
    origin = np.concatenate([pkg.overlay.random_origins(g.n, 200, seed=7), [g.n - 1, 0, 0]]).astype(np.int32)
    k = pkg.overlay.spread_keys(g.row_ptr, g.col, origin, hops)
    assert k.dtype == np.uint64
    assert k.tolist() == _brute(g, origin, hops)
    with pytest.raises(ValueError):
        pkg.overlay.spread_keys(g.row_ptr, g.col, origin, 0)


def test_spread_order_rule(pkg):
    keys = np.array([5, 9, 9, 1, 7, 9], np.uint64)
    assert pkg.overlay.spread_order(keys).tolist() == [1, 2, 5, 4, 0, 3]   # key desc, ties by index
    inject = np.array([1, 1, 0, 0, 0, 2])
    assert pkg.overlay.spread_order(keys, inject).tolist() == [2, 4, 3, 1, 0, 5]   # inject round first
    assert pkg.overlay.spread_order(np.zeros(0, np.uint64)).tolist() == []
