"""Build libgossip_hip.so for gfx950 in-tree (csrc/ -> _build/).

hipcc cross-compiles without a GPU, so this runs in the CPU container; the
built .so travels to the GPU box with the repo snapshot.
"""
import os
import subprocess
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG_DIR, "csrc")
OUT_DIR = os.path.join(PKG_DIR, "_build")
LIB = os.path.join(OUT_DIR, "libgossip_hip.so")
INCLUDE = os.path.join(os.path.dirname(PKG_DIR), "include", "gossip_capi.h")
SOURCES = ["driver.hip", "setup.hip", "pull.hip", "hub.hip", "push.hip", "liveness.hip", "graph_build.hip",
           "checkpoint.hip", "partition.hip", "bitcount.hip", "shard.hip"]
HEADERS = ["gp_common.h", "gp_internal.h", "gp_device.h", "xplan.h"]
ARCH = os.environ.get("GOSSIP_OFFLOAD_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-result", f"--offload-arch={ARCH}"]


def _hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.sep not in c or os.path.exists(c)):
            return c
    return "hipcc"


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


STANDIN_SRC = os.path.join(os.path.dirname(PKG_DIR), "tests", "native", "rccl_standin.cpp")
STANDIN_LIB = os.path.join(OUT_DIR, "libgossip_hip_rccl_standin.so")


def build_standin(force=False, verbose=True):
    """TEST build: the engine's own objects linked against the in-process RCCL
    stand-in of tests/native/rccl_standin.cpp instead of librccl, so the vertex
    partition's RCCL path (exchange_rccl) runs with P > 1 ranks as threads of
    one process on one GPU (tests/test_rccl_standin.py).  The product library
    (libgossip_hip.so) is not touched."""
    build(force=force, verbose=verbose)
    objs = [os.path.join(OUT_DIR, os.path.splitext(s)[0] + ".o") for s in SOURCES]
    if not force and not _stale(STANDIN_LIB, objs + [STANDIN_SRC, __file__]):
        return STANDIN_LIB
    sobj = os.path.join(OUT_DIR, "rccl_standin.o")
    cmd = [_hipcc(), "-O2", "-std=c++17", "-fPIC", "-Wall", f"--offload-arch={ARCH}", "-c", STANDIN_SRC, "-o", sobj]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    tmp = STANDIN_LIB + ".tmp"
    cmd = [_hipcc(), *FLAGS, "-shared", *objs, sobj, "-o", tmp, "-pthread"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    os.replace(tmp, STANDIN_LIB)
    return STANDIN_LIB


def build(force=False, verbose=True):
    os.makedirs(OUT_DIR, exist_ok=True)
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS] + [INCLUDE, __file__]
    if not force and not _stale(LIB, deps):
        return LIB
    objs, procs = [], []
    for s in SOURCES:
        obj = os.path.join(OUT_DIR, os.path.splitext(s)[0] + ".o")
        objs.append(obj)
        cmd = [_hipcc(), *FLAGS, "-c", os.path.join(CSRC, s), "-o", obj]
        if verbose:
            print(" ".join(cmd), flush=True)
        procs.append(subprocess.Popen(cmd))
    for p in procs:
        if p.wait() != 0:
            raise RuntimeError("hipcc failed")
    tmp = LIB + ".tmp"
    cmd = [_hipcc(), *FLAGS, "-shared", *objs, "-o", tmp, "-lrccl", "-pthread"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
    build_standin(force="--force" in sys.argv)
