"""bench.py's message table for N message shards, on the CPU:
every assignment is a permutation of the drawn table, `blocked` cuts the
whole table in spread order (rank p's block is the p-th slice of the speed
order), `interleaved` orders inside each rank's block of the drawn table,
`wordsnake` deals the ordered words in snake order; and --emulate-shard is
parsed and checked."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import _gossip_pkg  # noqa: E402

dist = _gossip_pkg.load().dist


def _speed_order(o):
    # a stand-in for spread_order: fastest = largest id (any fixed rule works)
    return np.argsort(-o, kind="stable")


@pytest.mark.parametrize("nranks", [1, 2, 3, 4, 5, 6, 8])
@pytest.mark.parametrize("assign", ["blocked", "interleaved", "wordsnake"])
def test_message_table_is_a_permutation(nranks, assign):
    rng = np.random.default_rng(nranks)
    origin = rng.permutation(100000)[:4096].astype(np.int32)
    if assign == "wordsnake" and 64 % nranks:   # snake counts would not match the shard blocks
        with pytest.raises(ValueError):
            bench.message_table(origin, nranks, assign, _speed_order, dist.message_shard)
        return
    t = bench.message_table(origin, nranks, assign, _speed_order, dist.message_shard)
    assert sorted(t.tolist()) == sorted(origin.tolist())
    blocks = [dist.message_shard(4096, nranks, p) for p in range(nranks)]
    if nranks == 1 or assign == "blocked":
        assert np.array_equal(t, origin[_speed_order(origin)])
    if assign == "blocked" and nranks > 1:   # rank p: the p-th slice of the speed order
        for p in range(nranks - 1):
            assert t[blocks[p][0]:blocks[p][1]].min() > t[blocks[p + 1][0]:blocks[p + 1][1]].max()
    if assign == "interleaved" and nranks > 1:   # rank p: its own block of the drawn table
        for lo, hi in blocks:
            assert sorted(t[lo:hi].tolist()) == sorted(origin[lo:hi].tolist())
    if assign == "wordsnake" and nranks > 1:   # rank 0 gets word 0 and word 2N-1 of the ordered table
        ordered = origin[_speed_order(origin)]
        lo, hi = blocks[0]
        assert np.array_equal(t[lo:lo + 64], ordered[:64])
        assert np.array_equal(t[lo + 64:lo + 128], ordered[64 * (2 * nranks - 1):64 * 2 * nranks])


def test_emulate_shard_parsing():
    a = bench.parse(["--emulate-shard", "3/8", "--shard-assign", "blocked"])
    assert a.emulate_shard == "3/8" and a.shard_assign == "blocked"
    assert bench.parse([]).shard_assign == "blocked" and bench.parse([]).emulate_shard is None
