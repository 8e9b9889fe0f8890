"""Multi-process (one process per GPU) host orchestration.

Two ways to spread one gossip run over N GPUs:

* message shards (default): messages are independent objects -- a message's
  spread never reads another message's bits -- so rank p runs the whole overlay
  for the word-aligned message block message_shard(m, N, p).  No data-path
  collective: the shards' per-round counters add up, their digests XOR, their
  first / coverage / forwards columns concatenate.
* vertex partition: rank p owns a contiguous vertex slice, by default
  [p*S, min((p+1)*S, n)) with S = ceil(n / nranks), or with
  partition_by_arcs=1 the slice holding in-arcs [p*A/N, (p+1)*A/N) (SURVEY.md
  §8e; partition_bounds below mirrors csrc/xplan.h); every round each rank ships the new frontier words
  of its boundary vertices to the ranks holding them as ghosts (ncclSend /
  ncclRecv inside libgossip_hip.so, csrc/partition.hip).

The control plane is this module's own TCP star (no PyTorch in the product
process): rank 0 listens on MASTER_ADDR:(MASTER_PORT + 1) -- MASTER_PORT itself
belongs to the launcher's store under torch.distributed.run -- and every
collective is an all-gather of byte strings through rank 0.  It carries rank
0's 128-byte RCCL unique id, aligns the timed region and sums / maxes a few
counters per step; the data path never touches it.  Payloads are raw bytes,
JSON or .npy (allow_pickle=False): nothing received is unpickled.
"""
import io
import json
import os
import socket
import struct
import time

import numpy as np


def env():
    """(world_size, rank, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def message_shard(m, nranks, rank):
    """Word-aligned contiguous message block [lo, hi) of rank `rank`: the
    m messages are cut into 64-message words, spread as evenly as possible."""
    words = (m + 63) // 64
    if nranks > words:
        raise ValueError(f"{m} messages give {words} words: at most {words} message shards")
    w0 = rank * words // nranks
    w1 = (rank + 1) * words // nranks
    return min(m, 64 * w0), min(m, 64 * w1)


def partition_bounds(n, nranks, row_ptr=None):
    """Owned slices [(begin, end)] of a vertex partition, as the engine cuts
    them (csrc/xplan.h partition_bounds): equal vertex counts, or, given the
    global in-CSR row_ptr (partition_by_arcs=1), equal in-arc counts --
    rank p starts at the first vertex whose arcs start at or after
    ceil(p * nnz / nranks)."""
    b = [0] * (nranks + 1)
    b[nranks] = n
    nnz = int(row_ptr[n]) if row_ptr is not None else 0
    s = (n + nranks - 1) // nranks
    for p in range(1, nranks):
        if row_ptr is not None and nnz > 0:
            b[p] = int(np.searchsorted(row_ptr, (p * nnz + nranks - 1) // nranks, side="left"))
        else:
            b[p] = min(n, p * s)
        b[p] = max(b[p], b[p - 1])
    return [(b[p], b[p + 1]) for p in range(nranks)]


# ---------------------------------------------------------------------------
# control plane

_HDR = struct.Struct("<Q")


def _send(sock, data):
    sock.sendall(_HDR.pack(len(data)) + data)


def _recv_exact(sock, k):
    buf = bytearray(k)
    view = memoryview(buf)
    got = 0
    while got < k:
        r = sock.recv_into(view[got:], k - got)
        if r == 0:
            raise ConnectionError("control-plane peer closed the connection")
        got += r
    return bytes(buf)


def _recv(sock):
    (k,) = _HDR.unpack(_recv_exact(sock, _HDR.size))
    return _recv_exact(sock, k)


def _np_bytes(a):
    f = io.BytesIO()
    np.save(f, np.asarray(a), allow_pickle=False)
    return f.getvalue()


def _np_load(b):
    return np.load(io.BytesIO(b), allow_pickle=False)


class Group:
    """A star of `world` processes around rank 0 over TCP.  Every collective
    is all_gather_bytes: ranks send their payload to rank 0, which returns the
    rank-ordered list to everybody."""

    def __init__(self, rank, world, addr="127.0.0.1", port=29501, timeout=300.0):
        self.rank, self.world = int(rank), int(world)
        self._peers = {}
        self._sock = None
        self._listener = None
        deadline = time.monotonic() + timeout
        if self.rank == 0:
            ls = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            ls.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            ls.bind((addr, port))
            ls.listen(self.world)
            ls.settimeout(max(deadline - time.monotonic(), 1.0))
            self._listener = ls
            while len(self._peers) < self.world - 1:
                conn, _ = ls.accept()
                conn.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                conn.settimeout(timeout)
                (r,) = struct.unpack("<I", _recv_exact(conn, 4))
                if not 0 < r < self.world or r in self._peers:
                    conn.close()
                    raise ConnectionError(f"control plane: unexpected rank {r}")
                self._peers[r] = conn
        else:
            while True:
                try:
                    s = socket.create_connection((addr, port), timeout=5.0)
                    break
                except OSError:
                    if time.monotonic() > deadline:
                        raise
                    time.sleep(0.05)
            s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            s.settimeout(timeout)
            s.sendall(struct.pack("<I", self.rank))
            self._sock = s

    def get_rank(self):
        return self.rank

    def get_world_size(self):
        return self.world

    def all_gather_bytes(self, data):
        data = bytes(data)
        if self.rank == 0:
            parts = [data] + [b""] * (self.world - 1)
            for r, conn in self._peers.items():
                parts[r] = _recv(conn)
            blob = b"".join(_HDR.pack(len(p)) + p for p in parts)
            for conn in self._peers.values():
                _send(conn, blob)
            return parts
        _send(self._sock, data)
        blob = _recv(self._sock)
        parts, off = [], 0
        for _ in range(self.world):
            (k,) = _HDR.unpack_from(blob, off)
            off += _HDR.size
            parts.append(blob[off:off + k])
            off += k
        return parts

    def barrier(self):
        self.all_gather_bytes(b"")

    def broadcast_bytes(self, data, src=0):
        return self.all_gather_bytes(data if self.rank == src else b"")[src]

    def all_gather_array(self, a):
        return [_np_load(b) for b in self.all_gather_bytes(_np_bytes(a))]

    def close(self):
        for conn in self._peers.values():
            conn.close()
        self._peers = {}
        for s in (self._sock, self._listener):
            if s is not None:
                s.close()
        self._sock = self._listener = None

    destroy_process_group = close


def init(timeout=300.0):
    """Control-plane group for a multi-process launch (None at world size 1)."""
    world, rank, _ = env()
    if world <= 1:
        return None
    addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
    port = int(os.environ.get("GP_CTRL_PORT") or int(os.environ.get("MASTER_PORT", "29500")) + 1)
    return Group(rank, world, addr, port, timeout)


def broadcast_bytes(pg, data, src=0):
    if pg is None:
        return data
    return pg.broadcast_bytes(data, src)


def share_comm_id(pg, make_id):
    """Rank 0 creates the RCCL unique id (128 bytes); every rank receives it."""
    rank = pg.get_rank() if pg is not None else 0
    return broadcast_bytes(pg, make_id() if rank == 0 else b"")


def gather_slices(pg, local):
    """Concatenate the ranks' owned slices in rank order (all ranks get it)."""
    if pg is None:
        return local
    return np.concatenate(pg.all_gather_array(local))


def allsum(pg, x):
    if pg is None:
        return x
    parts = pg.all_gather_array(np.asarray(x, dtype=np.float64))
    return np.sum(parts, axis=0)


def allmax(pg, x):
    if pg is None:
        return x
    vals = pg.all_gather_bytes(json.dumps(float(x)).encode())
    return max(float(json.loads(v)) for v in vals)
