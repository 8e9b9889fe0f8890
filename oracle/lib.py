"""ctypes binding of oracle/_build/liboracle_gossip.so (test infrastructure)."""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "liboracle_gossip.so")


class RoundStats(ctypes.Structure):
    _fields_ = [(k, ctypes.c_int64) for k in
                ("injected", "lost", "new_bits", "receivers", "sends", "active", "crashed",
                 "reports", "removals", "dup_reports")]


_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])
    return LIB


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        lib = ctypes.CDLL(LIB)
        P = ctypes.c_void_p
        lib.or_chung_lu.restype = ctypes.c_int64
        lib.or_chung_lu.argtypes = [ctypes.c_int64, ctypes.c_double, ctypes.c_double, ctypes.c_uint64,
                                    ctypes.POINTER(P), ctypes.POINTER(P)]
        lib.or_free.argtypes = [P]
        lib.or_digest_term.restype = ctypes.c_uint64
        lib.or_digest_term.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64]
        lib.or_draw_export.restype = ctypes.c_uint64
        lib.or_draw_export.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64]
        lib.or_run.restype = ctypes.c_int32
        lib.or_run.argtypes = [ctypes.c_int64, P, P, ctypes.c_int32, P, P, ctypes.c_int32, P, P,
                               ctypes.c_int32, ctypes.c_double, ctypes.c_uint64, ctypes.c_int32,
                               ctypes.c_int32, P, P, ctypes.c_int32, ctypes.c_int32, P, P, P, P, P,
                               ctypes.POINTER(RoundStats), P, ctypes.c_int64,
                               ctypes.POINTER(ctypes.c_int64)]
        _lib = lib
    return _lib


def _p(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


def chung_lu(n, dbar, gamma, seed):
    """(row_ptr int64[n+1], col int32[nnz]) of the Chung-Lu overlay."""
    lib = load()
    rp, cl = ctypes.c_void_p(), ctypes.c_void_p()
    nnz = lib.or_chung_lu(int(n), float(dbar), float(gamma), int(seed), ctypes.byref(rp), ctypes.byref(cl))
    row_ptr = np.ctypeslib.as_array((ctypes.c_int64 * (n + 1)).from_address(rp.value)).copy()
    col = np.ctypeslib.as_array((ctypes.c_int32 * max(nnz, 1)).from_address(cl.value))[:nnz].copy()
    lib.or_free(rp)
    lib.or_free(cl)
    return row_ptr, col


def transpose(n, row_ptr, col):
    """In-CSR -> out-CSR (rows sorted)."""
    dst = np.repeat(np.arange(n, dtype=np.int64), np.diff(row_ptr))
    src = col.astype(np.int64)
    order = np.lexsort((dst, src))
    orp = np.zeros(n + 1, np.int64)
    np.cumsum(np.bincount(src, minlength=n), out=orp[1:])
    return orp, np.ascontiguousarray(dst[order].astype(np.int32))


def digest_term(rr, w, bits):
    return int(load().or_digest_term(rr, w, bits))


def digest_from_first(first, origin, word_base=0):
    """Per-vertex digest recomputed from a first-receipt matrix
    [n][m] whose column k is global message 64*word_base + k -- the digest of a
    message shard in global word numbering (shard digests XOR together)."""
    n, m = first.shape
    own = {}
    for k in range(m):
        own.setdefault(int(origin[k]), set()).add(k)
    out = np.zeros(n, np.uint64)
    for v in range(n):
        groups = {}
        for k in np.nonzero(first[v] != 255)[0]:
            key = (int(first[v, k]), int(k) >> 6, int(k) in own.get(v, ()))
            groups[key] = groups.get(key, 0) | (1 << (int(k) & 63))
        d = 0
        for (rr, w, inj), bits in groups.items():
            d ^= digest_term(rr, (word_base + w) | (0x80000000 if inj else 0), bits)
        out[v] = d
    return out


def run(csr, origin, inject_round=None, churn=False, p_fail=0.0, churn_seed=0, miss_threshold=3,
        crashes=(), max_rounds=254, nthreads=1, want_first=False, want_forwards=True,
        report_cap=1 << 20, want_seen=True):
    """Full propagation on the CPU.  crashes: iterable of (vertex, round).
    want_seen=False skips the Message-List copy-out (8 GiB at C4)."""
    lib = load()
    n = int(csr.n)
    origin = np.ascontiguousarray(origin, dtype=np.int32)
    m = int(origin.size)
    inj = np.zeros(m, np.int32) if inject_round is None else np.ascontiguousarray(inject_round, np.int32)
    W = 1
    while W * 64 < m:
        W <<= 1
    rp = np.ascontiguousarray(csr.row_ptr, np.int64)
    col = np.ascontiguousarray(csr.col, np.int32)
    orp = ocol = None
    if csr.directed:
        orp, ocol = transpose(n, rp, col)
    cr = np.array(list(crashes), dtype=np.int32).reshape(-1, 2)
    cv = np.ascontiguousarray(cr[:, 0])
    crd = np.ascontiguousarray(cr[:, 1])
    seen = np.zeros((n, W), np.uint64) if want_seen else None
    first = np.zeros((n, m), np.uint8) if want_first else None
    digest = np.zeros(n, np.uint64)
    cov = np.zeros(m, np.uint64)
    fwd = np.zeros(m, np.uint64) if want_forwards else None
    stats = (RoundStats * max_rounds)()
    reports = np.zeros((report_cap, 3), np.int32)
    nrep = ctypes.c_int64()
    rounds = lib.or_run(n, _p(rp), _p(col), 1 if csr.directed else 0, _p(orp), _p(ocol), m, _p(origin),
                        _p(inj), 1 if churn else 0, float(p_fail), int(churn_seed), int(miss_threshold),
                        int(cv.size), _p(cv), _p(crd), int(max_rounds), int(nthreads), _p(seen),
                        _p(first), _p(digest), _p(cov), _p(fwd), stats, _p(reports), int(report_cap),
                        ctypes.byref(nrep))
    if rounds < 0:
        raise ValueError("or_run rejected its input")
    st = [{k: getattr(stats[i], k) for k, _ in RoundStats._fields_} for i in range(rounds)]
    return {"rounds": rounds, "stats": st, "seen": seen, "first": first, "digest": digest,
            "coverage": cov, "forwards": fwd, "reports": reports[:min(nrep.value, report_cap)],
            "n_reports": nrep.value}
