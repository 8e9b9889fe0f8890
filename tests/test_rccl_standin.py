"""The vertex partition's RCCL path with P > 1 ranks on one GPU.

RCCL refuses two ranks on one device, so `exchange_rccl` (csrc/partition.hip:
count all-gather, grouped ncclSend / ncclRecv of the boundary entries, unpack,
counters' all-reduce) would otherwise first run on an 8-GPU node.  A test
build of the engine links the in-process stand-in of
tests/native/rccl_standin.cpp in place of librccl
(build_lib.build_standin -> _build/libgossip_hip_rccl_standin.so); a child
process loads it (GOSSIP_HIP_LIB) and drives P = 2, 3, 4 (and 8 on the hub overlay) ranks as threads,
both slice rules, with and without churn, against the oracle
(tests/rccl_standin_driver.py).  The product library keeps real RCCL.
Reference: gossip crosses real links only (Peer.py:402-404).
"""
import ctypes
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NCCL_SYMBOLS = ("ncclGetUniqueId", "ncclCommInitRank", "ncclCommDestroy", "ncclGetErrorString", "ncclGroupStart",
                "ncclGroupEnd", "ncclAllReduce", "ncclAllGather", "ncclSend", "ncclRecv", "ncclCommCount",
                "ncclCommUserRank")


def _standin_lib(pkg):
    import importlib
    sys.path.insert(0, os.path.dirname(pkg._lib.__file__))
    build_lib = importlib.import_module("build_lib")
    return build_lib.STANDIN_LIB


def test_standin_library_defines_the_rccl_calls(pkg):
    """CPU: the test build exists, defines every RCCL entry point the engine
    calls itself and does not pull librccl in; the product library does."""
    path = _standin_lib(pkg)
    assert os.path.exists(path), "run __graft_entry__.build()"
    nm = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True, check=True).stdout
    defined = {ln.split()[-1] for ln in nm.splitlines() if ln.strip()}
    assert set(NCCL_SYMBOLS) <= defined
    und = subprocess.run(["nm", "-D", "--undefined-only", pkg._lib.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    assert set(NCCL_SYMBOLS) <= {ln.split()[-1] for ln in und.splitlines() if ln.strip()}
    needed = subprocess.run(["readelf", "-d", path], capture_output=True, text=True, check=True).stdout
    assert "librccl" not in needed
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
    assert lib.gp_abi_version() == pkg._lib.ABI_VERSION


def _driver(pkg, mode, *args, extra_env=None, timeout=840):
    path = _standin_lib(pkg)
    assert os.path.exists(path)
    env = dict(os.environ, GOSSIP_HIP_LIB=path, GP_STANDIN_ASYNC="1" if mode == "async" else "0")
    env.pop("GP_STANDIN_CORRUPT", None)
    env.update(extra_env or {})
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tests", "rccl_standin_driver.py"), *args], env=env,
                       capture_output=True, text=True, timeout=timeout)
    print(r.stdout[-6000:])
    assert r.returncode == 0, r.stderr[-6000:]
    return r.stdout


@pytest.mark.gpu
@pytest.mark.timeout(900)
@pytest.mark.parametrize("mode", ["sync", "async"])
def test_exchange_rccl_multi_rank(pkg, mode):
    """27 partitioned runs through exchange_rccl against the oracle, with the
    stand-in synchronous or enqueue-only (async: RCCL's stream semantics, so a
    missing stream dependency in the engine would show up as a mismatch)."""
    out = _driver(pkg, mode)
    assert f"stand-in mode: {mode}" in out
    assert "cases ok: 27" in out


@pytest.mark.gpu
@pytest.mark.timeout(300)
@pytest.mark.parametrize("mode", ["sync", "async"])
def test_exchange_rccl_corrupt_entry_fails_every_rank(pkg, mode):
    """A boundary entry corrupted in flight (the stand-in overwrites rank 1's
    third non-empty receive) fails the round on both ranks with GP_ERCCL: the
    unpack checks every entry against the exchange plan before writing, and
    the counters' all-reduce carries the count to every rank."""
    out = _driver(pkg, mode, "--corrupt", extra_env={"GP_STANDIN_CORRUPT": "1:2"}, timeout=280)
    assert "corrupt ok: ranks=2 status=-5" in out


@pytest.mark.gpu
@pytest.mark.timeout(600)
@pytest.mark.parametrize("mode", ["sync", "async"])
def test_shard_job_combine_multi_rank(pkg, mode):
    """Message-shard jobs of P = 1-4 and 8 ranks through gp_shard_combine
    (csrc/shard.hip: the XOR reduce-scatter of the digests by ncclSend /
    ncclRecv + the all-gather of the reduced slices, the OR reduce-scatter of
    the per-round receiver / sender bitmaps, the all-gather of coverage /
    forwards and counters), over the stand-in RCCL and over the host
    all-gather: every rank's job record equals the oracle's whole run,
    with and without churn (Peer.py:175-216, each peer's whole receive record)."""
    out = _driver(pkg, mode, "--shards", timeout=580)
    assert "shard cases ok: 24" in out
