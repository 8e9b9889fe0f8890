"""Multi-process (one process per GPU) host orchestration.

Two ways to spread one gossip run over N GPUs:

* message shards (default): messages are independent objects -- a message's
  spread never reads another message's bits -- so rank p runs the whole overlay
  for the word-aligned message block message_shard(m, N, p).  No data-path
  collective: the shards' per-round counters add up, their digests XOR, their
  first / coverage / forwards columns concatenate.
* vertex partition: rank p owns the contiguous vertex slice [p*S, min((p+1)*S, n))
  with S = ceil(n / nranks) and every round all-gathers the owned next rows over
  RCCL inside libgossip_hip.so (equal-size slices as RCCL's all-gather requires;
  ids are randomly relabelled, DESIGN.md §2.7, so slices carry equal arc counts).

torch.distributed (gloo, CPU) is only the control plane: it hands rank 0's
RCCL unique id to every rank, aligns the timed region and gathers per-rank
results for checking.
"""
import os
import sys

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


def partition_bounds(n, nranks):
    s = (n + nranks - 1) // nranks
    return [(min(n, p * s), min(n, (p + 1) * s)) for p in range(nranks)]


def init(backend="gloo"):
    """Control-plane process group.  Gloo's C++ side prints its peer-connection
    messages to stdout, where rank 0's one JSON line (bench.py) must stand
    alone: stdout is pointed at stderr while the group connects."""
    import torch.distributed as dist
    world, rank, _ = env()
    if world > 1 and not dist.is_initialized():
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group(backend, rank=rank, world_size=world)
            dist.barrier()
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
    return dist if world > 1 else None


def broadcast_bytes(pg, data, src=0):
    if pg is None:
        return data
    box = [data if pg.get_rank() == src else None]
    pg.broadcast_object_list(box, src=src)
    return box[0]


def share_comm_id(pg, make_id):
    """Rank 0 creates the RCCL unique id (128 bytes); every rank receives it."""
    rank = pg.get_rank() if pg is not None else 0
    return broadcast_bytes(pg, make_id() if rank == 0 else None)


def gather_slices(pg, local):
    """Concatenate the ranks' owned slices in rank order (all ranks get it)."""
    if pg is None:
        return local
    parts = [None] * pg.get_world_size()
    pg.all_gather_object(parts, np.asarray(local))
    return np.concatenate(parts)


def allsum(pg, x):
    if pg is None:
        return x
    import torch
    t = torch.as_tensor(np.asarray(x, dtype=np.float64))
    pg.all_reduce(t)
    return t.numpy()


def allmax(pg, x):
    if pg is None:
        return x
    import torch
    t = torch.tensor([float(x)], dtype=torch.float64)
    pg.all_reduce(t, op=pg.ReduceOp.MAX)
    return float(t.item())
