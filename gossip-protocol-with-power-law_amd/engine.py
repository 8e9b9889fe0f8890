"""GossipEngine: host driver of the MI355X gossip hot path over the C-ABI.

Replaces, for all peers at once, the reference's per-peer threads:
gossip_sender (Peer.py:395-408), the receive handlers (Peer.py:175-216,
258-296), the heartbeat monitor (Peer.py:298-393) and the seed's dead-node
removal (Seed.py:358-406).  One `round()` = liveness + injection + pull
expansion (+ RCCL exchange on multi-GPU), all on the device.
"""
import ctypes
import os

import numpy as np

from . import _lib
from ._lib import check


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


class GossipEngine:
    def __init__(self, device=0, **config):
        self._lib = _lib.load()
        self._ctx = ctypes.c_void_p()
        check(self._lib.gp_create(int(device), ctypes.byref(self._ctx)))
        self.device = device
        self.cfg = _lib.Config()
        self._lib.gp_default_config(ctypes.byref(self.cfg))
        self.n = 0
        self.m = 0
        self.words = 0
        self.origin = None
        self.inject_round = None
        self.nranks = 1
        if config:
            self.configure(**config)

    # -- lifecycle ---------------------------------------------------------
    def close(self):
        if self._ctx:
            self._lib.gp_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def configure(self, **kw):
        for k, v in kw.items():
            if not hasattr(self.cfg, k):
                raise KeyError(f"unknown config field {k}")
            setattr(self.cfg, k, v)
        check(self._lib.gp_configure(self._ctx, ctypes.byref(self.cfg)))

    # -- overlay -----------------------------------------------------------
    def load_graph(self, csr):
        rp = np.ascontiguousarray(csr.row_ptr, dtype=np.int64)
        col = np.ascontiguousarray(csr.col, dtype=np.int32)
        check(self._lib.gp_load_graph(self._ctx, int(csr.n), int(col.size), _ptr(rp), _ptr(col),
                                      1 if csr.directed else 0, None, None))
        self.n = int(csr.n)

    def build_chung_lu(self, n, dbar, gamma, seed):
        check(self._lib.gp_build_chung_lu(self._ctx, int(n), float(dbar), float(gamma), int(seed)))
        self.n = int(n)

    def graph(self):
        """The overlay as loaded / built (global CSR).  A partitioned context
        keeps only its local CSR: see local_graph()."""
        from .overlay import CSR
        if self.nranks > 1:
            raise RuntimeError("a partitioned context holds its local CSR only (local_graph())")
        n, nnz = self.info()[:2]
        rp = np.empty(n + 1, dtype=np.int64)
        col = np.empty(nnz, dtype=np.int32)
        check(self._lib.gp_read(self._ctx, _lib.ROW_PTR, _ptr(rp), rp.nbytes))
        check(self._lib.gp_read(self._ctx, _lib.COL, _ptr(col), col.nbytes))
        return CSR(n, rp, col, False)

    def local_info(self):
        """(nloc, nghost, nextra, nnz_local, n_boundary) of this context."""
        v = [ctypes.c_int64() for _ in range(5)]
        check(self._lib.gp_local_info(self._ctx, *[ctypes.byref(x) for x in v]))
        return tuple(x.value for x in v)

    def local_graph(self):
        """(row_ptr, col, l2g) of the context's local CSR: owned vertices
        [0, nloc) with their full in-lists, ghosts with their owned neighbours,
        origin extras with none; l2g maps local ids to global ids."""
        nloc, ng, nx, nnz_l, _ = self.local_info()
        nv = nloc + ng + nx if self.nranks > 1 else self.n
        rp = self._read(_lib.ROW_PTR, np.empty(nv + 1, dtype=np.int64))
        col = self._read(_lib.COL, np.empty(nnz_l, dtype=np.int32))
        l2g = self._read(_lib.L2G, np.empty(nv, dtype=np.int32))
        return rp, col, l2g

    def degrees(self):
        """Degree of every vertex of the loaded overlay (in-degree of the
        in-CSR; = degree for undirected overlays), from row_ptr alone."""
        if self.nranks > 1:
            raise RuntimeError("degrees() needs the global overlay (check it before partitioning)")
        n = self.info()[0]
        rp = np.empty(n + 1, dtype=np.int64)
        check(self._lib.gp_read(self._ctx, _lib.ROW_PTR, _ptr(rp), rp.nbytes))
        return np.diff(rp)

    def check_degree(self, gamma, tol=0.15):
        """SURVEY.md §8a A9 on the overlay this context holds: discrete MLE
        gamma_hat with KS-chosen kmin against the generator's gamma (the
        reference's intent, degree-weighted selection, demonstrate_powerlaw.py:19-27)."""
        from . import degree
        return degree.check_powerlaw(self.degrees(), gamma, tol)

    def info(self):
        n, nnz = ctypes.c_int64(), ctypes.c_int64()
        m, w = ctypes.c_int32(), ctypes.c_int32()
        check(self._lib.gp_info(self._ctx, ctypes.byref(n), ctypes.byref(nnz), ctypes.byref(m), ctypes.byref(w)))
        return n.value, nnz.value, m.value, w.value

    # -- partition / RCCL --------------------------------------------------
    def set_partition(self, rank, nranks):
        """Vertex partition: keep the owned slice of rank `rank`
        of `nranks` plus ghost rows; nranks > 1 drops the global CSR and the
        message table (set_messages again, in global ids)."""
        check(self._lib.gp_set_partition(self._ctx, int(rank), int(nranks)))
        self.nranks = int(nranks)
        if nranks > 1:
            self.m = self.words = 0

    def partition(self):
        b, e = ctypes.c_int64(), ctypes.c_int64()
        check(self._lib.gp_get_partition(self._ctx, ctypes.byref(b), ctypes.byref(e)))
        return b.value, e.value

    @staticmethod
    def comm_unique_id():
        buf = ctypes.create_string_buffer(128)
        check(_lib.load().gp_comm_unique_id(buf))
        return buf.raw

    def comm_init(self, unique_id, nranks, rank):
        buf = ctypes.create_string_buffer(bytes(unique_id), 128)
        check(self._lib.gp_comm_init(self._ctx, buf, int(nranks), int(rank)))

    # -- message-shard jobs (csrc/shard.hip) -----------------
    def shard_comm_init(self, unique_id, nranks, rank):
        """Join an nranks-rank message-shard job over RCCL (one GPU per rank;
        rank 0 makes the id with comm_unique_id())."""
        buf = ctypes.create_string_buffer(bytes(unique_id), 128)
        check(self._lib.gp_shard_comm_init(self._ctx, buf, int(nranks), int(rank)))

    def shard_host_init(self, all_gather_bytes, nranks, rank):
        """Join a message-shard job whose combine moves its chunks through the
        host: all_gather_bytes(bytes) -> [bytes of rank 0, ..., rank nranks-1]
        (ranks sharing a GPU, which RCCL refuses)."""
        def fn(_user, send, nbytes, recv):
            try:
                parts = all_gather_bytes(ctypes.string_at(send, nbytes))
                if len(parts) != nranks or any(len(p) != nbytes for p in parts):
                    return -1
                ctypes.memmove(recv, b"".join(parts), nranks * nbytes)
                return 0
            except Exception:   # (a C caller cannot take a Python exception)
                return -1
        self._shard_cb = _lib.AllGatherFn(fn)   # kept alive as long as the context
        check(self._lib.gp_shard_host_init(self._ctx, self._shard_cb, None, int(nranks), int(rank)))

    def shard_info(self):
        """(nranks, rank, transport) as the job's transport reports them:
        ncclCommCount / ncclCommUserRank for RCCL (transport 1), the host
        all-gather's (2), or (0, 0, 0) outside a shard job."""
        v = [ctypes.c_int32() for _ in range(3)]
        check(self._lib.gp_shard_info(self._ctx, *[ctypes.byref(x) for x in v]))
        return tuple(x.value for x in v)

    def combine(self, max_rounds=254):
        """gp_shard_combine after run(): the job's per-round counters (list of
        dicts, every rank the same) and the combine's device time in ms.  The
        job's digest / coverage / forwards are then job_digest() etc."""
        buf = (_lib.RoundStats * max_rounds)()
        k = ctypes.c_int32()
        ms = ctypes.c_double()
        check(self._lib.gp_shard_combine(self._ctx, buf, int(max_rounds), ctypes.byref(k), ctypes.byref(ms)))
        return [buf[i].as_dict() for i in range(k.value)], ms.value

    def job_digest(self):
        return self._read(_lib.JOB_DIGEST, np.empty(self.n, dtype=np.uint64))

    def job_coverage(self, m_total):
        return self._read(_lib.JOB_COVERAGE, np.empty(int(m_total), dtype=np.uint64))

    def job_forwards(self, m_total):
        return self._read(_lib.JOB_FORWARDS, np.empty(int(m_total), dtype=np.uint64))

    # -- messages / run ----------------------------------------------------
    def set_messages(self, origin, inject_round=None):
        o = np.ascontiguousarray(origin, dtype=np.int32)
        r = None if inject_round is None else np.ascontiguousarray(inject_round, dtype=np.int32)
        if r is not None and r.shape != o.shape:
            raise ValueError("origin and inject_round differ in length")
        check(self._lib.gp_set_messages(self._ctx, int(o.size), _ptr(o), _ptr(r)))
        self.origin = o
        self.inject_round = r if r is not None else np.zeros_like(o)
        _, _, self.m, self.words = self.info()

    def spread_keys(self, origin, hops=2):
        """gp_spread_keys: arc endpoints within `hops` of each origin (the
        global overlay; call before a vertex partition)."""
        o = np.ascontiguousarray(origin, dtype=np.int32)
        keys = np.zeros(o.size, np.uint64)
        check(self._lib.gp_spread_keys(self._ctx, int(hops), int(o.size), _ptr(o), _ptr(keys)))
        return keys

    def spread_order(self, origin, inject_round=None, hops=2):
        """Permutation p that orders a message table by spread speed
        (overlay.spread_order): run origin[p] (and inject_round[p]); per-message
        outputs of that run are those of message p[k] at index k."""
        from .overlay import spread_order
        return spread_order(self.spread_keys(origin, hops), inject_round)

    def set_message_shard(self, origin, inject_round, lo, hi):
        """Take messages [lo, hi) of a larger message table as this context's
        shard: local message k is global message lo + k.  lo must
        be word aligned so that digests of the shards XOR into the digest of
        the whole table, and first/coverage/forwards concatenate."""
        if lo % 64:
            raise ValueError("message shards start on a 64-message word boundary")
        self.configure(msg_word_base=lo // 64)
        r = None if inject_round is None else np.asarray(inject_round)[lo:hi]
        self.set_messages(np.asarray(origin)[lo:hi], r)

    def reset(self):
        check(self._lib.gp_reset(self._ctx))

    def crash(self, verts):
        v = np.ascontiguousarray(verts, dtype=np.int32)
        check(self._lib.gp_crash(self._ctx, int(v.size), _ptr(v)))

    def round(self):
        st = _lib.RoundStats()
        check(self._lib.gp_round(self._ctx, ctypes.byref(st)))
        return st.as_dict()

    @staticmethod
    def round_group(engines):
        """One round over single-process contexts engines[k] owning partition k
        (device-to-device exchange, no RCCL); returns the summed counters."""
        arr = (ctypes.c_void_p * len(engines))(*[e._ctx.value for e in engines])
        st = _lib.RoundStats()
        check(_lib.load().gp_round_group(arr, len(engines), ctypes.byref(st)))
        return st.as_dict()

    @staticmethod
    def run_group(engines, max_rounds=254):
        out = []
        last = max(int(engines[0].inject_round.max()), 0) if engines[0].m else -1
        for _ in range(max_rounds):
            st = GossipEngine.round_group(engines)
            out.append(st)
            if st["new_bits"] == 0 and st["round"] >= last:
                break
        return out

    def run(self, max_rounds=254):
        buf = (_lib.RoundStats * max_rounds)()
        k = ctypes.c_int32()
        check(self._lib.gp_run(self._ctx, int(max_rounds), buf, ctypes.byref(k)))
        return [buf[i].as_dict() for i in range(k.value)]

    def synchronize(self):
        check(self._lib.gp_synchronize(self._ctx))

    # -- checkpoints ----------------------------------
    def checkpoint(self):
        """The context's whole per-run state between rounds, as an opaque
        uint8 blob (gp_checkpoint_save)."""
        nb = ctypes.c_int64()
        check(self._lib.gp_checkpoint_size(self._ctx, ctypes.byref(nb)))
        blob = np.empty(nb.value, dtype=np.uint8)
        check(self._lib.gp_checkpoint_save(self._ctx, _ptr(blob), blob.nbytes))
        return blob

    def restore(self, blob):
        """Continue the run a checkpoint() blob captured: same overlay,
        messages, partition and tracked outputs (gp_checkpoint_load)."""
        b = np.ascontiguousarray(blob, dtype=np.uint8)
        check(self._lib.gp_checkpoint_load(self._ctx, _ptr(b), b.nbytes))

    def save_checkpoint(self, path):
        """Write the checkpoint() blob to `path` as a .npy file, straight into a
        memory map of the file: host memory stays bounded by the page cache
        even for the 32 GiB of Message-List rows of a 2^26 x 4096 run.  The
        blob goes to `path`.tmp first and replaces `path` only once it is
        complete, so a failed save leaves the previous checkpoint intact."""
        nb = ctypes.c_int64()
        check(self._lib.gp_checkpoint_size(self._ctx, ctypes.byref(nb)))
        path = os.fspath(path)
        tmp = path + ".tmp"
        out = np.lib.format.open_memmap(tmp, mode="w+", dtype=np.uint8, shape=(nb.value,))
        ok = False
        try:
            check(self._lib.gp_checkpoint_save(self._ctx, _ptr(out), out.nbytes))
            out.flush()
            ok = True
        finally:
            del out
            if not ok:
                try:
                    os.unlink(tmp)
                except OSError:
                    pass
        os.replace(tmp, path)

    def load_checkpoint(self, path):
        """Restore a save_checkpoint() file (memory-mapped, read-only).  The
        blob's header names its overlay, messages, partition and tracked
        outputs; a mismatch raises and leaves the current run untouched."""
        blob = np.load(path, mmap_mode="r", allow_pickle=False)
        try:
            if blob.dtype != np.uint8 or blob.ndim != 1:
                raise ValueError(f"{path}: not a gossip checkpoint")
            check(self._lib.gp_checkpoint_load(self._ctx, ctypes.c_void_p(blob.ctypes.data), blob.nbytes))
        finally:
            del blob

    # -- outputs -----------------------------------------------------------
    def _read(self, what, arr):
        check(self._lib.gp_read(self._ctx, what, _ptr(arr), arr.nbytes))
        return arr

    def nloc(self):
        b, e = self.partition()
        return e - b

    def seen(self):
        return self._read(_lib.SEEN, np.empty((self.nloc(), self.words), dtype=np.uint64))

    def first(self):
        return self._read(_lib.FIRST, np.empty((self.nloc(), self.m), dtype=np.uint8))

    def digest(self):
        return self._read(_lib.DIGEST, np.empty(self.nloc(), dtype=np.uint64))

    def finalize(self):
        check(self._lib.gp_finalize_messages(self._ctx))

    def coverage(self):
        return self._read(_lib.COVERAGE, np.empty(self.m, dtype=np.uint64))

    def forwards(self):
        return self._read(_lib.FORWARDS, np.empty(self.m, dtype=np.uint64))

    def _nv(self):   # per-vertex reads: the owned slice of a partitioned context
        return self.nloc() if self.nranks > 1 else self.n

    def state(self):
        return self._read(_lib.STATE, np.empty(self._nv(), dtype=np.uint8))

    def miss(self):
        return self._read(_lib.MISS, np.empty(self._nv(), dtype=np.uint8))

    def deg_live(self):
        return self._read(_lib.DEG_LIVE, np.empty(self._nv(), dtype=np.int32))

    def frontier(self):
        return self._read(_lib.FRONTIER, np.empty((self._nv(), self.words), dtype=np.uint64))

    def reports(self, cap=1 << 20):
        """Reports of the last round as int32 [k, 3] (dead, reporter, round),
        unordered, plus the exact total (k < total if the buffer overflowed).
        gp_reports copies at most min(total, cap, report_capacity) rows: only
        those are returned."""
        buf = np.empty((cap, 3), dtype=np.int32)
        n = ctypes.c_int64()
        check(self._lib.gp_reports(self._ctx, ctypes.cast(buf.ctypes.data, ctypes.POINTER(_lib.Report)),
                                   int(cap), ctypes.byref(n)))
        k = min(n.value, cap, max(int(self.cfg.report_capacity), 1))
        return buf[:k].copy(), n.value
