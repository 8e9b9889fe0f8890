"""Multi-process host orchestration on CPU (dist.py's TCP control plane, world
size 2 and 3): RCCL-id hand-off, partition bounds, ordered gather of owned
slices, counter sums.
The per-rank compute is the CPU oracle on the full overlay, sliced as the
engine slices it; the device exchange itself is covered on the GPU by
test_gpu_parity.py::test_group_partition_invariance."""
import os
import socket

import multiprocessing as mp

import numpy as np
import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import _gossip_pkg
    from oracle import lib as oracle
    pkg = _gossip_pkg.load()
    d = pkg.dist
    pg = d.init(timeout=120)
    try:
        uid = d.share_comm_id(pg, lambda: bytes(range(128)))
        g = pkg.overlay.barabasi_albert(1001, 2, seed=3)
        origin = pkg.overlay.random_origins(g.n, 100, 3)
        ref = oracle.run(g, origin, want_first=True)
        vb, ve = d.partition_bounds(g.n, world)[rank]
        first = d.gather_slices(pg, ref["first"][vb:ve])
        digest = d.gather_slices(pg, ref["digest"][vb:ve])
        cov_local = (ref["first"][vb:ve] != 255).sum(axis=0)
        cov = d.allsum(pg, cov_local)
        tmax = d.allmax(pg, float(rank))
        q.put((rank, uid == bytes(range(128)), np.array_equal(first, ref["first"]),
               np.array_equal(digest, ref["digest"]), np.array_equal(cov, ref["coverage"]), tmax))
    finally:
        pg.close()


def test_two_rank_gloo_orchestration():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, uid_ok, first_ok, dig_ok, cov_ok, tmax in res:
        assert uid_ok and first_ok and dig_ok and cov_ok and tmax == 1.0


def test_partition_bounds(pkg):
    d = pkg.dist
    for n, p in [(10, 3), (1 << 24, 8), (7, 8), (1000, 1)]:
        b = d.partition_bounds(n, p)
        assert b[0][0] == 0 and b[-1][1] == n
        assert all(b[i][1] == b[i + 1][0] for i in range(p - 1))
        s = (n + p - 1) // p
        assert all(e - s0 <= s for s0, e in b)
    # arc-balanced slices: each holds about nnz / p in-arcs
    g = pkg.overlay.barabasi_albert(5000, 3, seed=2)
    deg = np.diff(g.row_ptr)
    for p in (2, 3, 8):
        b = d.partition_bounds(g.n, p, g.row_ptr)
        assert b[0][0] == 0 and b[-1][1] == g.n
        assert all(b[i][1] == b[i + 1][0] for i in range(p - 1))
        arcs = [int(g.row_ptr[e] - g.row_ptr[s0]) for s0, e in b]
        assert max(arcs) <= g.nnz / p + deg.max()


def _shard_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import _gossip_pkg
    from oracle import lib as oracle
    pkg = _gossip_pkg.load()
    d = pkg.dist
    pg = d.init(timeout=120)
    try:
        g = pkg.overlay.barabasi_albert(700, 2, seed=6)
        m = 200
        origin = pkg.overlay.random_origins(g.n, m, 6)
        inject = (np.arange(m) % 3).astype(np.int32)
        full = oracle.run(g, origin, inject, want_first=True)
        lo, hi = d.message_shard(m, world, rank)
        part = oracle.run(g, origin[lo:hi], inject[lo:hi], want_first=True)
        # per-round counters add up (pad the shorter shard runs with quiet rounds)
        R = 64
        loc = np.zeros((R, 2))
        for i, s in enumerate(part["stats"]):
            loc[i] = (s["new_bits"], s["sends"])
        tot = d.allsum(pg, loc)
        ok_rounds = all(tot[i, 0] == s["new_bits"] and tot[i, 1] == s["sends"]
                        for i, s in enumerate(full["stats"]))
        # columns concatenate, digests (global word numbering) XOR
        first = np.concatenate([x for x in _gather(pg, part["first"].T)]).T
        dig = 0
        for x in _gather(pg, oracle.digest_from_first(part["first"], origin[lo:hi], lo // 64)):
            dig = np.bitwise_xor(dig, x)
        cov = np.concatenate(_gather(pg, part["coverage"]))
        q.put((rank, ok_rounds, np.array_equal(first, full["first"]), np.array_equal(dig, full["digest"]),
               np.array_equal(cov, full["coverage"])))
    finally:
        pg.close()


def _gather(pg, x):
    return pg.all_gather_array(np.asarray(x))


def test_two_rank_message_shards_compose():
    """Message shards (the default multi-GPU decomposition): two
    ranks each run the oracle on their word-aligned message block; per-round
    counters sum, first-receipt columns and coverage concatenate and the
    shard digests (global word numbering) XOR to the whole run's."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_shard_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, *oks in res:
        assert all(oks), (rank, oks)


def test_message_shard_bounds(pkg):
    d = pkg.dist
    for m, p in [(4096, 1), (4096, 2), (4096, 8), (200, 2), (130, 3), (64, 1)]:
        b = [d.message_shard(m, p, r) for r in range(p)]
        assert b[0][0] == 0 and b[-1][1] == m
        assert all(b[i][1] == b[i + 1][0] for i in range(p - 1))
        assert all(lo % 64 == 0 for lo, _ in b)
    assert d.message_shard(4096, 8, 3) == (1536, 2048)
    with pytest.raises(ValueError):
        d.message_shard(100, 3, 0)


def _plane_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import _gossip_pkg
    d = _gossip_pkg.load().dist
    pg = d.init(timeout=120)
    try:
        out = []
        for it in range(50):   # many small collectives back to back keep their order
            out.append(d.allsum(pg, [rank + it, 1.0])[0])
        big = d.gather_slices(pg, np.full(100000 + rank, rank, dtype=np.uint64))
        pg.barrier()
        mx = d.allmax(pg, 10.0 * rank)
        q.put((rank, out, big.size, int(big[-1]), mx, "torch" in sys.modules))
    finally:
        pg.close()


def test_control_plane_three_ranks():
    """The TCP star with 3 ranks: ordered collectives, a 2.4 MB gather, and no
    PyTorch in a rank process."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 3
    procs = [ctx.Process(target=_plane_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, out, size, last, mx, torch_loaded in res:
        assert out == [3 * it + 3 for it in range(50)]
        assert size == 3 * 100000 + 3 and last == 2 and mx == 20.0
        assert not torch_loaded


def test_bench_imports_no_torch():
    """The product process (bench.py, the package, the control plane) never
    imports PyTorch."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys; sys.path.insert(0, %r); import bench, _gossip_pkg; pkg = _gossip_pkg.load(); "
            "import importlib; importlib.import_module(pkg.__name__ + '.dist'); "
            "print('torch' in sys.modules)" % root)
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip() == "False"
