"""The message-shard job's combine at C4 size: P ranks as P
threads on one GPU through the RCCL stand-in (GOSSIP_HIP_LIB =
_build/libgossip_hip_rccl_standin.so; tests/native/rccl_standin.cpp), each
running its blocked shard of the spread-ordered 4096-message table on the
2^24-node overlay, then gp_shard_combine.  Prints, per rank, the combine's
device time and the bytes its chunks move, and checks the job record against
the one-context run of the whole table (digest, coverage, forwards, counters).

The stand-in moves chunks with device-to-device copies on one GPU, so the
time here is the combine's kernels plus HBM-speed copies; the xGMI estimate
adds the per-link bytes at 64 GB/s per direction (scripts/README.md)."""
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _gossip_pkg  # noqa: E402

KEYS = ("injected", "lost", "new_bits", "receivers", "sends", "active", "crashed", "reports", "removals")


def main():
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    log2n = int(sys.argv[2]) if len(sys.argv) > 2 else 24
    pkg = _gossip_pkg.load()
    assert "rccl_standin" in pkg._lib.load()._name
    n = 1 << log2n
    bench = __import__("bench")
    args = bench.parse(["--log2n", str(log2n)])
    t0 = time.time()
    whole = pkg.GossipEngine(0, **bench.engine_config(args))
    whole.build_chung_lu(n, 16.0, 2.5, 4)
    origin = pkg.overlay.random_origins(n, 4096, seed=4)
    table = bench.message_table(origin, P, "blocked", lambda o: whole.spread_order(o, hops=3), pkg.dist.message_shard)
    whole.set_messages(table)
    whole.reset()
    ref = whole.run()
    whole.finalize()
    ref_dig, ref_cov, ref_fwd = whole.digest(), whole.coverage(), whole.forwards()
    whole.close()
    print(f"whole run: {len(ref)} rounds, {time.time() - t0:.1f} s", flush=True)
    uid = pkg.GossipEngine.comm_unique_id()
    engs = []
    for k in range(P):
        e = pkg.GossipEngine(0, **bench.engine_config(args))
        e.build_chung_lu(n, 16.0, 2.5, 4)
        lo, hi = pkg.dist.message_shard(4096, P, k)
        e.set_message_shard(table, None, lo, hi)
        engs.append(e)
    out = [None] * P
    errs = []
    bar = threading.Barrier(P, timeout=300)

    def rank(k):
        try:
            e = engs[k]
            e.shard_comm_init(uid, P, k)
            ms = []
            for _ in range(3):
                e.reset()
                e.run()
                e.finalize()
                e.synchronize()
                bar.wait()   # (the ranks share one GPU: start the combines together, after every run)
                job, t = e.combine()
                ms.append(t)
            out[k] = dict(job=job, ms=ms, dig=e.job_digest(), cov=e.job_coverage(4096), fwd=e.job_forwards(4096))
        except BaseException as x:
            errs.append((k, x))

    ts = [threading.Thread(target=rank, args=(k,)) for k in range(P)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    if errs:
        raise RuntimeError(errs)
    R = len(out[0]["job"])
    nw = (n + 63) // 64
    L = (nw + P - 1) // P
    Ld = (n + P - 1) // P
    # bytes each rank sends to its P - 1 peers: the bitmaps' and digests'
    # reduce-scatter chunks, then the reduced digest slice and the columns
    # (all-gather), and the counters
    per_peer = 8 * (2 * R * L + Ld + Ld + 2 * 64 * 8 + R * 32 + 2 * R + 16)
    for k, o in enumerate(out):
        assert np.array_equal(o["dig"], ref_dig) and np.array_equal(o["cov"], ref_cov)
        assert np.array_equal(o["fwd"], ref_fwd)
        assert len(o["job"]) == len(ref)
        for a, b in zip(o["job"], ref):
            for key in KEYS:
                assert a[key] == b[key], (key, a["round"])
    line = {"P": P, "n": n, "rounds": R, "combine_ms_per_rank": [round(min(o["ms"]), 3) for o in out],
            "bytes_per_peer_link": per_peer, "bytes_per_rank_out": per_peer * (P - 1),
            "xgmi_estimate_ms": round(per_peer / 64e9 * 1e3, 3), "job_record_equals_whole_run": True}
    print(json.dumps(line), flush=True)
    for e in engs:
        e.close()


if __name__ == "__main__":
    main()
