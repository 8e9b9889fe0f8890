#!/usr/bin/env python3
"""Vertex partition of C4 (2^24 x 4096) over P contexts on one
GPU (gp_round_group: the same pack / unpack as the RCCL exchange, device
copies instead of ncclSend/Recv).  Prints per-round boundary entries and bytes
summed over the ranks, per-rank local sizes, and checks the run's per-round
counters against the one-context run.  usage: partition_c4.py P [log2n]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _gossip_pkg  # noqa: E402


def main():
    P = int(sys.argv[1])
    log2n = int(sys.argv[2]) if len(sys.argv) > 2 else 24
    pkg = _gossip_pkg.load()
    n, m, seed = 1 << log2n, 4096, 4
    with pkg.GossipEngine(0, track_digest=1) as one:
        one.build_chung_lu(n, 16.0, 2.5, seed)
        g = one.graph()
        origin = pkg.overlay.random_origins(n, m, seed=seed)
        one.set_messages(origin)
        one.reset()
        ref = one.run()
    print(json.dumps({"P": P, "n": n, "arcs": int(g.nnz), "rounds": len(ref)}), flush=True)
    engs = []
    for k in range(P):
        e = pkg.GossipEngine(0, track_digest=1)
        e.load_graph(g)
        e.set_partition(k, P)
        e.set_messages(origin)
        e.reset()
        nloc, ng, nx, nnz_l, nb = e.local_info()
        print(json.dumps({"rank": k, "nloc": nloc, "nghost": ng, "nextra": nx, "arcs_local": nnz_l,
                          "boundary_entries": nb}), flush=True)
        engs.append(e)
    del g
    tot = 0
    for r in range(254):
        t0 = time.perf_counter()
        st = pkg.GossipEngine.round_group(engs)
        dt = time.perf_counter() - t0
        a = ref[r]
        ok = all(st[k] == a[k] for k in ("new_bits", "sends", "receivers", "injected"))
        tot += st["xchg_bytes"]
        print(json.dumps({"round": r, "new_bits": st["new_bits"], "xchg_entries": st["xchg_rows"],
                          "xchg_bytes": st["xchg_bytes"], "xchg_bytes_per_rank": st["xchg_bytes"] / P,
                          "matches_one_context": ok, "group_round_s": round(dt, 4)}), flush=True)
        assert ok, (st, a)
        if st["new_bits"] == 0 and r >= 0:
            break
    print(json.dumps({"P": P, "total_xchg_bytes": tot, "per_rank_bytes": tot / P}), flush=True)
    for e in engs:
        e.close()


if __name__ == "__main__":
    main()
