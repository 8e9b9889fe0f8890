#!/usr/bin/env python3
"""Headline benchmark: gossip edge-deliveries/s (GTEPS) on a 2^24-node Chung-Lu
power-law overlay (gamma 2.5, mean degree 16) with 4096 concurrent messages
(BASELINE.json config 4), plus the HBM roofline fraction of the expansion kernel.

One step = one complete gossip run: reset the Message-Lists, inject all 4096
messages at their origins (round 0), and run forward-once rounds until no vertex
receives anything new.  value = protocol edge-deliveries (sum of `sends` over all
rounds = 4096 x arcs for a connected overlay) / wall time of the timed steps.

python bench.py [--gpus N] [--steps K] [--warmup W]; N > 1 is launched by
torch.distributed.run (one process per GPU; the data path is RCCL inside
libgossip_hip.so, the control plane is dist.py's own TCP star, which only
distributes the RCCL id and the timings: no PyTorch in this process).
"""
import argparse
import glob
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", choices=("c4", "c5"), default="c4",
                    help="c4: BASELINE config 4 (2^24 x 4096, the headline line); c5: config 5, "
                         "2^26 nodes with 1%%/round crashes, 3-miss detection and seed removal")
    ap.add_argument("--log2n", type=int, default=None)
    ap.add_argument("--dbar", type=float, default=16.0)
    ap.add_argument("--gamma", type=float, default=2.5)
    ap.add_argument("--messages", type=int, default=4096)
    ap.add_argument("--seed", type=int, default=None)
    ap.add_argument("--p-fail", type=float, default=0.01, help="c5: per-round crash probability")
    ap.add_argument("--hub-threshold", type=int, default=4096)
    ap.add_argument("--push-ratio", type=float, default=100.0)
    ap.add_argument("--early-exit", type=int, default=1)
    ap.add_argument("--unfiltered-pct", type=int, default=90,
                    help="pull without the per-arc activity check when >= this %% of vertices send (0 = never)")
    ap.add_argument("--arc-mask-permille", type=int, default=0,
                    help="filtered pull rounds with >= this many senders per 1000 vertices build "
                         "the per-arc activity mask first (0 = always probe per arc)")
    ap.add_argument("--compact-rows", type=int, default=0,
                    help="1: sparse 64-word rounds gather compact Message-Lists (DESIGN.md §3.2)")
    ap.add_argument("--prefilter-pct", type=int, default=20)
    ap.add_argument("--summary-min-n", type=int, default=1 << 25,
                    help="sparse probe rounds of overlays with >= this many vertices read the summary level first")
    ap.add_argument("--split-deg", type=int, default=128,
                    help="degree-split sparse rounds: senders of in-degree < this push, receivers probe the "
                         "gather-order prefix of the others (0 = off; DESIGN.md §3.2)")
    ap.add_argument("--split-max-permille", type=int, default=10,
                    help="degree-split rounds only while fewer than this many vertices per 1000 send")
    ap.add_argument("--flat-max-words", type=int, default=16,
                    help="rows of at most this many words take the edge-parallel pull (<= 32, 0 = never)")
    ap.add_argument("--message-order", choices=("given", "spread"), default="spread",
                    help="bit order of the message table: as drawn, or grouped by spread speed "
                         "(overlay.spread_order)")
    ap.add_argument("--spread-hops", type=int, default=3, help="--message-order spread: key radius (1..3)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--cpu-log2n", type=int, default=None,
                    help="cpu_baseline: overlay size of the oracle's run (all messages, W = 64); default: the "
                         "workload's own size -- the whole C4 run (~30 s on 16 host threads), or the whole C5 "
                         "run with churn (2^26, ~100 s and ~100 GiB of host memory)")
    ap.add_argument("--parallel", choices=("messages", "vertex"), default="messages",
                    help="N > 1: message shards (no data-path collective, default) or the vertex "
                         "partition with a sparse boundary exchange every round (ncclSend/Recv of "
                         "the boundary vertices' new words)")
    ap.add_argument("--shard-assign", choices=("interleaved", "blocked", "wordsnake"), default="blocked",
                    help="message shards: blocks of the table ordered by spread speed as a whole (blocked, "
                         "default: rank 0 the fastest; a rank's receivers complete together), every rank a "
                         "contiguous block of the drawn table ordered inside it (interleaved: every rank gets "
                         "messages of every speed), or the ordered table's 64-message words dealt in snake "
                         "order (wordsnake); DESIGN.md §6, profiles/r04_shard_emulation.txt")
    ap.add_argument("--emulate-shard", default=None, metavar="R/N",
                    help="one process runs rank R's message shard of an N-rank job alone (the per-GPU work "
                         "of the N-GPU run, for projections on a one-GPU box; not a multi-GPU number)")
    ap.add_argument("--profile-steps", action="store_true",
                    help="print per-round stats of the last step to stderr")
    a = ap.parse_args(argv)
    c5 = a.workload == "c5"
    if a.log2n is None:
        a.log2n = 26 if c5 else 24
    if a.cpu_log2n is None:   # the workload itself: C4, or C5 with churn at 2^26
        a.cpu_log2n = a.log2n
    if a.seed is None:
        a.seed = 5 if c5 else 4
    return a


def round_bytes(st, words, nloc):
    """Algorithmic bytes of one expansion launch of the pull:
    per owned vertex 26 B of vertex state read (fpop, deg_live, row_ptr pair,
    state, seenpop, done_at, slot byte) and its 4-B fpop of the next round
    written, per receiver 23 B of per-vertex words committed (seenpop 4, slot
    and written-slot bytes 3, digest read-modify-write 16), per scanned arc the 4-B column id + the 8-B
    activity-bitmap probe (scan 0), or 1 mask bit + the 4-B column id of the
    active arcs only (scan 1, + 8 B of mask words per vertex), or the column id
    alone (scan 2, unfiltered), the neighbour-row bytes the kernel actually
    loaded (8W per gathered row, less the words early-exit rounds skip), per
    receiver seen row read 8W B and per receiver seen row written to the next
    slot 8W B; plus the senders' rows read to build line masks (k_mklm, 8W B
    each) before a filtered 64-word pull."""
    w8 = 8 * words
    scan = st.get("scan", 0) & 3
    if scan == 2:
        arcs = 4 * st["arcs_scanned"]
    elif scan == 1:
        arcs = st["arcs_scanned"] / 8 + 4 * st["rows_gathered"] + 8 * nloc
    else:
        arcs = 12 * st["arcs_scanned"]
    # degree-split rounds (scan bit 32): the push half's accumulator updates,
    # 8 B each (kernel_ms brackets the push half and the clear too)
    split = 8 * st.get("atomics", 0) if st.get("scan", 0) & 32 else 0
    # done-probe rounds (scan bit 64): an 8-B done-bitmap word per scanned arc;
    # receivers committed as aliases of their component row write no row,
    # only their per-vertex words
    if st.get("scan", 0) & 64:
        arcs += 8 * st["arcs_scanned"]
    return (30 * nloc + arcs + st["row_bytes"] + w8 * st["seen_rows_read"]
            + (w8 + 23) * st["rows_written"] + 23 * st.get("aliased", 0) + w8 * st.get("lm_rows", 0) + split)


def message_table(origin, nranks, assign, order, message_shard):
    """The message table of a run in spread order (order(o) -> permutation of
    o, fastest first).  One rank: the whole table ordered.  nranks message
    shards (rank p takes message_shard(m, nranks, p), word-aligned blocks):
    blocked -- the whole table ordered, then cut (each rank's messages spread
    at one speed); interleaved -- each rank's block of the drawn table ordered
    inside; wordsnake -- the ordered table's 64-message words dealt to the
    ranks in snake order.  Always a permutation of origin."""
    m = len(origin)
    nwords = (m + 63) // 64
    if nranks > 1 and assign == "wordsnake" and nwords % nranks:
        # (snake order deals equal word counts; the shard blocks would cut
        # unequal ones, handing ranks part of a neighbour's words)
        raise ValueError(f"wordsnake needs the {nwords} words to divide among {nranks} ranks")
    if nranks > 1 and assign == "interleaved":
        blocks = [message_shard(m, nranks, p) for p in range(nranks)]
    else:
        blocks = [(0, m)]
    out = np.concatenate([origin[lo:hi][order(origin[lo:hi])] for lo, hi in blocks])
    if nranks > 1 and assign == "wordsnake":   # word k of the ordered table to rank snake(k)
        words = [out[64 * k:64 * (k + 1)] for k in range((m + 63) // 64)]
        per = [[] for _ in range(nranks)]
        for k, w in enumerate(words):
            r, lap = k % nranks, k // nranks
            per[r if lap % 2 == 0 else nranks - 1 - r].append(w)
        out = np.concatenate([np.concatenate(x) for x in per if x])
    return out


def engine_config(args):
    """The engine configuration of the timed run (tests/test_full_size.py
    checks a run configured by this very function against the oracle)."""
    cfg = dict(track_digest=1, track_first=0, hub_threshold=args.hub_threshold, push_ratio=args.push_ratio,
               early_exit=args.early_exit, unfiltered_pct=args.unfiltered_pct, flat_max_words=args.flat_max_words,
               arc_mask_permille=args.arc_mask_permille, compact_rows=args.compact_rows,
               prefilter_pct=args.prefilter_pct, summary_min_n=args.summary_min_n, split_deg=args.split_deg,
               split_max_permille=args.split_max_permille)
    if args.workload == "c5":   # Bernoulli crashes of live vertices, stream seeded by the run seed
        cfg.update(churn=1, p_fail=args.p_fail, churn_seed=args.seed, miss_threshold=3)
    return cfg


PMC_TRAFFIC = sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_traffic*.json")))


def pmc_traffic(config):
    """HBM traffic per k_expand launch measured by the two rocprofv3 --pmc
    passes of scripts/gpu_round_profile.sh (FETCH_SIZE x2 + WRITE_SIZE, the
    gfx950 correction of MI355X_MICROARCH.md), from the profiles/pmc_traffic*.json
    whose workload keys match this run (C4: pmc_traffic.json, C5:
    pmc_traffic_c5.json); None when no such measurement is committed."""
    keys = ("n", "arcs", "messages", "words_per_row", "seed", "parallelism", "message_order")
    for path in PMC_TRAFFIC:
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        if all(d["config"].get(k) == config.get(k) for k in keys):
            return d["traffic_bytes_per_launch"], os.path.relpath(path, ROOT)
    return None, None


def dense_round_bytes(n, nnz, words):
    """SURVEY.md §8d dense-pull formula (for reference only)."""
    return 8 * (n + 1) + 4 * nnz + 8 * words * nnz + 24 * words * n


def _host():
    """Host CPU facts for the cpu_baseline object: the threads this process may
    use (OMP_NUM_THREADS, else its affinity set), nproc and the CPU model."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    threads = int(os.environ.get("OMP_NUM_THREADS") or 0) or aff
    return threads, os.cpu_count() or 1, aff, model


def cpu_baseline(args, eng, origin, pkg):
    """CPU legs, timed on this box's host cores (reported beside the GPU
    line, never the target):
      port     oracle/gossip_oracle.c (OpenMP) with the OMP_NUM_THREADS share
               (16 on the GPU box), and -- C4, when the process may use more --
               with every thread of its affinity set on a quarter-size sample
               (`value`: the faster leg; on the GPU box's EPYC 9575F all 256
               threads ran the whole C4 run 3x slower than 16,
               profiles/r06_bench.json), running ALL
               `messages` (W = 64 words per Message-List row, the GPU's layout)
               to quiescence on a 2^cpu_log2n-vertex overlay of the same
               Chung-Lu recipe and seed: by default the workload itself, on
               the overlay the GPU ran (C4 2^24 x 4096: ~30 s on 16 threads;
               C5 2^26 x 4096 with churn, the same crash stream: ~100 s);
      harness  oracle/harness.py, the reference's per-peer Message-List logic
               (sha256 digests in a set per peer, Peer.py:175-216, 395-408) plus
               forwarding, single-core, on BASELINE config 2 (10^4-node BA(m=2),
               64 messages)."""
    from oracle import harness
    from oracle import lib as oracle_lib
    threads, nproc, aff, model = _host()
    if args.cpu_threads:
        threads = args.cpu_threads
    churn = args.workload == "c5"
    ncpu = 1 << args.cpu_log2n
    if ncpu == eng.n and eng.nranks == 1:   # the overlay the GPU just ran
        g = eng.graph()
    else:
        with pkg.GossipEngine(eng.device) as side:   # the same recipe, device-built (bit-identical to the oracle's)
            side.build_chung_lu(ncpu, args.dbar, args.gamma, args.seed)
            g = side.graph()
    o = pkg.overlay.random_origins(ncpu, args.messages, seed=args.seed)

    def leg(g, o, t, log2n, note):
        t0 = time.perf_counter()
        ref = oracle_lib.run(g, o, nthreads=t, want_forwards=False, want_seen=False, churn=churn,
                             p_fail=args.p_fail if churn else 0.0, churn_seed=args.seed)
        dt = time.perf_counter() - t0
        sends = sum(s["sends"] for s in ref["stats"])
        return {"kind": "port", "value": sends / dt / 1e9, "unit": "GTEPS", "cores": t,
                "sample": f"oracle/gossip_oracle.c, Chung-Lu gamma={args.gamma} d={args.dbar:g} seed {args.seed} at "
                          f"2^{log2n} vertices ({g.nnz} arcs{note}), all {len(o)} messages (W = 64), full run"
                          f"{' with churn' if churn else ''} ({ref['rounds']} rounds, {sends} edge-deliveries, "
                          f"{dt:.1f} s, {t} OpenMP threads of {nproc})"}

    # port legs: the OMP_NUM_THREADS share the environment grants (16 on the
    # GPU box) on the workload itself; and, when the process may use more,
    # every thread of its affinity set (SURVEY.md §8d "all host cores") on a
    # quarter-size overlay of the same recipe -- the whole C4 run took 76 s on
    # all 256 threads of the GPU box, 3x the 16-thread leg, against a bounded
    # 10-30 s sample
    legs = [leg(g, o, threads, args.cpu_log2n, ", the GPU run overlay" if ncpu == eng.n else "")]
    if not args.cpu_threads and aff > threads and not churn:
        q = max(args.cpu_log2n - 2, 10)
        with pkg.GossipEngine(eng.device) as side:
            side.build_chung_lu(1 << q, args.dbar, args.gamma, args.seed)
            gq = side.graph()
        legs.append(leg(gq, pkg.overlay.random_origins(1 << q, args.messages, seed=args.seed), aff, q,
                        ", a quarter-size sample of the same recipe"))
    best = max(legs, key=lambda x: x["value"])   # (the fastest leg: 256 threads ran slower than 16 here)
    out = {"value": best["value"], "unit": "GTEPS", "cores": best["cores"], "kind": "port",
           "sample": best["sample"],
           "host": {"nproc": nproc, "affinity": aff, "omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
                    "cpu_model": model}}
    # leg 2: the per-peer Python harness, single core, BASELINE config 2
    h = pkg.overlay.barabasi_albert(10000, 2, seed=2)
    ho = pkg.overlay.random_origins(h.n, 64, seed=2).tolist()
    in_lists = [h.col[h.row_ptr[v]:h.row_ptr[v + 1]].tolist() for v in range(h.n)]
    t0 = time.perf_counter()
    hr = harness.run(h.n, in_lists, False, ho, [0] * len(ho))
    hdt = time.perf_counter() - t0
    hs = sum(s["sends"] for s in hr["stats"])
    out["legs"] = legs + [
        {"kind": "harness", "value": hs / hdt / 1e9, "unit": "GTEPS", "cores": 1,
         "sample": f"oracle/harness.py (per-peer sha256 Message-List sets), 10^4-node BA(m=2), 64 messages, "
                   f"{hr['rounds']} rounds, {hs} edge-deliveries, {hdt:.2f} s, 1 core"},
    ]
    return out


def _fp(a):
    """64-bit fingerprint of an output array (sha256 of its bytes)."""
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()[:16]


def job_record(eng, stats, m_total, job, partitioned):
    """The whole run's record as the line reports it, so that 1-GPU and N-GPU
    lines compare directly: per-round receivers / active counts and
    fingerprints of the per-vertex digest and the per-message coverage /
    forwards (a shard job: the combined job outputs; one GPU: the context's
    own).  None for the vertex partition (each rank holds its slice)."""
    if partitioned:
        return None
    dig = eng.job_digest() if job else eng.digest()
    cov = eng.job_coverage(m_total) if job else eng.coverage()
    try:
        fwd = _fp(eng.job_forwards(m_total) if job else eng.forwards())
    except Exception as e:   # churn without track_msg_forwards: GP_ENOTRACK
        if getattr(e, "status", None) != -6:
            raise
        fwd = None
    return {"rounds": len(stats), "receivers": [int(s["receivers"]) for s in stats],
            "active": [int(s["active"]) for s in stats], "new_bits": [int(s["new_bits"]) for s in stats],
            "digest_fp": _fp(dig), "coverage_fp": _fp(cov), "forwards_fp": fwd}


def main():
    args = parse()
    import _gossip_pkg
    pkg = _gossip_pkg.load()
    dist = pkg.dist
    world, rank, local = dist.env()
    pg = dist.init()
    emu = None
    if args.emulate_shard:   # rank R of an N-rank message-shard job, alone in this process
        if world > 1:
            raise SystemExit("--emulate-shard runs one process")
        er, en = (int(x) for x in args.emulate_shard.split("/"))
        if not (en >= 1 and 0 <= er < en):
            raise SystemExit("--emulate-shard R/N needs 0 <= R < N")
        emu = (er, en)
    n = 1 << args.log2n
    # one GPU per rank; on a smaller box (rehearsal) ranks share devices round-robin
    device = local % max(pkg._lib.device_count(), 1)
    eng = pkg.GossipEngine(device, **engine_config(args))
    churn = args.workload == "c5"
    t0 = time.perf_counter()
    eng.build_chung_lu(n, args.dbar, args.gamma, args.seed)
    _, nnz, _, _ = eng.info()
    setup_s = build_s = time.perf_counter() - t0
    # SURVEY.md §8a A9 on the overlay just built (outside the timed region)
    deg = eng.check_degree(args.gamma)
    t0 = time.perf_counter()
    s_world, s_rank = (emu[1], emu[0]) if emu else (world, rank)   # the message-shard job's ranks
    shards = s_world > 1 and (emu is not None or args.parallel == "messages")
    origin = pkg.overlay.random_origins(n, args.messages, seed=args.seed)
    if args.message_order == "spread":   # bit order by spread speed; setup, untimed
        # blocked (default): the whole table, then cut, so that each rank's
        # messages spread at one speed and its receivers complete together (the
        # N = 8 job's slowest rank 22.3 -> 13.4 ms against interleaved: within
        # each rank's block of the drawn table); DESIGN.md §6
        origin = message_table(origin, s_world if shards else 1, args.shard_assign,
                               lambda o: eng.spread_order(o, hops=args.spread_hops), dist.message_shard)
    if world > 1 and not shards:
        eng.set_partition(rank, world)
        eng.comm_init(dist.share_comm_id(pg, pkg.GossipEngine.comm_unique_id), world, rank)
    if shards:   # this rank's word-aligned block of the 4096 messages
        lo, hi = dist.message_shard(args.messages, s_world, s_rank)
        eng.set_message_shard(origin, None, lo, hi)
    else:
        eng.set_messages(origin)
    # the N-GPU message-shard job combines its ranks' records into the job's
    # (gp_shard_combine, csrc/shard.hip) over RCCL -- one GPU per rank -- or,
    # when ranks share a GPU (a rehearsal on a smaller box: RCCL refuses two
    # ranks per device), over the control plane's all-gather
    job = shards and emu is None
    if job:
        if pkg._lib.device_count() >= world:
            eng.shard_comm_init(dist.share_comm_id(pg, pkg.GossipEngine.comm_unique_id), world, rank)
        else:
            eng.shard_host_init(pg.all_gather_bytes, world, rank)
    setup_s += time.perf_counter() - t0
    combine_ms = []

    def step():   # one whole gossip run, including the per-message coverage / forwards pass
        eng.reset()
        st = eng.run()
        eng.finalize()
        if job:   # the job's record, inside the step: every rank ends with the whole run's outputs
            js, ms = eng.combine()
            combine_ms.append(ms)
            return st, js
        return st, st

    for _ in range(args.warmup):
        step()
    if pg is not None:
        pg.barrier()
    eng.synchronize()
    t0 = time.perf_counter()
    steps = [step() for _ in range(args.steps)]
    eng.synchronize()
    if pg is not None:
        pg.barrier()
    dt = dist.allmax(pg, time.perf_counter() - t0)

    # the whole run's counters: one GPU, the vertex partition (all-reduced every
    # round) and the shard job (gp_shard_combine) all hold them
    runs = [j for _, j in steps]
    own_runs = [o for o, _ in steps]   # this rank's own rounds (its kernels)
    sends = sum(s["sends"] for r in runs for s in r)
    rounds = sum(len(r) for r in runs)
    own_rounds = sum(len(r) for r in own_runs)
    exp_ms = sum(s["expand_ms"] for r in own_runs for s in r)
    exch_ms = sum(s["exchange_ms"] for r in own_runs for s in r)
    # roofline of the dominant kernel set, the pull: k_expand (or
    # k_expand_flat), the hub passes that finish its hub receivers and, in
    # degree-split rounds, the push half and the accumulator clear -- HIP events
    # bracket all of them (kernel_ms), and the algorithmic bytes count all of them
    pulls = [s for r in own_runs for s in r if s["mode"] == 0 and s["kernel_ms"] > 0]
    nbytes = sum(round_bytes(s, eng.words, n) for s in pulls)
    kern_ms = sum(s["kernel_ms"] for s in pulls)
    if world > 1 and not shards:   # counters are global (all-reduced): per-rank share for the per-GPU roofline
        nbytes /= world
    achieved = nbytes / (kern_ms * 1e-3) / 1e9 if kern_ms > 0 else 0.0
    if shards:   # per-GPU roofline: mean over the ranks' own kernels
        achieved = float(dist.allsum(pg, [achieved])[0]) / world
    dense_eq = dense_round_bytes(n, nnz, eng.words) * own_rounds / (1 if shards else world) / (exp_ms * 1e-3) / 1e9
    if args.profile_steps and rank == 0:
        for s in own_runs[-1]:
            print(json.dumps({k: s[k] for k in ("round", "mode", "new_bits", "sends", "active", "receivers",
                                                "arcs_scanned", "rows_gathered", "seen_rows_read",
                                                "rows_written", "row_bytes", "atomics", "done_nb", "lm_rows", "aliased",
                                                "crashed", "reports", "removals", "scan", "expand_ms", "kernel_ms", "exchange_ms")}),
                  file=sys.stderr)
    record = job_record(eng, runs[-1], args.messages, job, world > 1 and not shards)
    comm = None
    if job:
        cn, _, xp = eng.shard_info()
        comm = {"transport": {1: "rccl", 2: "host all-gather (ranks share a GPU)"}.get(xp, "none"),
                "comm_ranks": cn, "combine_ms_per_step": sum(combine_ms[-args.steps:]) / args.steps}
    if rank == 0:
        split = " + the degree-split push half + k_acc_clear" if any(s["scan"] & 32 for s in pulls) else ""
        out = {
            "metric": f"gossip edge-deliveries/s (GTEPS) & HBM roofline %, 2^{args.log2n} nodes x {args.messages} msgs",
            "value": sends / dt / 1e9,
            "unit": "GTEPS",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic (device-built Chung-Lu overlay, seeded origins)",
            "config": {"workload": ("C5: Chung-Lu gamma=2.5 overlay with churn (p_fail per round, 3-miss "
                                    "liveness, seed removal), full forward-once gossip run" if churn else
                                    "C4: Chung-Lu gamma=2.5 overlay, full forward-once gossip run"),
                       "n": n, "arcs": nnz, "mean_degree": nnz / n, "messages": args.messages,
                       "words_per_row": eng.words, "rounds_per_step": rounds / args.steps,
                       "message_order": (f"spread ({args.spread_hops}-hop key)" if args.message_order == "spread"
                                         else "given"),
                       "edge_deliveries_per_step": sends // args.steps, "seed": args.seed,
                       "parallelism": (f"message-shard {emu[0]} of {emu[1]} alone (the per-GPU work of the "
                                       f"{emu[1]}-GPU run, {args.shard_assign})" if emu else
                                       f"message-shard x{world} ({args.shard_assign}), whole-job record combined "
                                       f"in every step over {comm['transport']} (XOR reduce-scatter of the digests "
                                       f"+ all-gather, OR reduce-scatter of the round bitmaps, all-gather of "
                                       f"coverage / forwards / counters)"
                                       if shards else
                                       (f"vertex-partition x{world} (sparse boundary exchange, ncclSend/Recv)"
                                        if world > 1 else "one GPU")),
                       "comm": comm,
                       "job": record,
                       "setup_s": round(setup_s, 2), "build_s": round(build_s, 2),
                       "degree_check": {"gamma_hat": round(deg["gamma_hat"], 4), "kmin": deg["kmin"],
                                        "gamma": args.gamma, "ok": bool(deg["ok"])}},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                         "kernel": (f"k_expand<{eng.words}> (+ k_mklm in line-mask rounds)" if eng.words > 32 else
                                    f"k_expand<{eng.words}> / k_expand_flat<{eng.words}>")
                                   + " + k_hub_partial + k_hub_final" + split
                                   + " per pull launch, HIP events on the engine stream",
                         "launches": len(pulls),
                         "avg_launch_ms": kern_ms / max(len(pulls), 1),
                         "alg_bytes_per_launch": nbytes / max(len(pulls), 1),
                         "expand_ms_per_step": exp_ms / args.steps,
                         "dense_equivalent_GBs": dense_eq,
                         "exchange_ms_per_round": exch_ms / max(own_rounds, 1)},
            "cpu_baseline": None,
        }
        traffic, src = pmc_traffic(out["config"])
        if traffic is not None:
            out["roofline"]["traffic"] = traffic
            out["roofline"]["traffic_source"] = src
            out["roofline"]["traffic_over_alg"] = traffic / out["roofline"]["alg_bytes_per_launch"]
        if world == 1 and not emu and not args.no_cpu_baseline:
            # the GPU line first (stderr), so that a CPU leg killed for memory
            # does not take the measurement with it
            print("gpu line (before cpu_baseline): " + json.dumps(out), file=sys.stderr, flush=True)
            out["cpu_baseline"] = cpu_baseline(args, eng, origin, pkg)
        print(json.dumps(out), flush=True)
    eng.close()
    if pg is not None:
        pg.close()


if __name__ == "__main__":
    main()
