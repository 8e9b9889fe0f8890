"""Child process of tests/test_rccl_standin.py (TEST INFRASTRUCTURE).

Loads the engine built against the in-process RCCL stand-in
(GOSSIP_HIP_LIB = _build/libgossip_hip_rccl_standin.so, tests/native/
rccl_standin.cpp) and runs the vertex partition's real RCCL path --
gp_comm_init, then every round through round_exchange_rccl -> exchange_rccl
(csrc/partition.hip: the count all-gather, the grouped ncclSend / ncclRecv of
the boundary entries, the unpack, the counters' all-reduce), and
gp_finalize_messages' all-reduce -- with P ranks as P threads on one GPU.
Every output is compared with the oracle's one-context run: per-round
counters, dead-node reports, first-receipt matrices, digests, Message-Lists,
coverage and forwards (the reference sends gossip only over real links,
Peer.py:402-404; liveness Peer.py:298-313, Seed.py:358-406).

Prints "cases ok: N" and exits 0 when every case matches; raises otherwise.
The stand-in runs synchronously or, with GP_STANDIN_ASYNC=1, only enqueues
(copies on a side stream ordered by events, as RCCL orders its kernels), so a
missing stream dependency in the engine shows up as a mismatch.

--corrupt: one P = 2 case with GP_STANDIN_CORRUPT set by the caller (the
stand-in overwrites one received boundary entry); every rank must fail the
same round with GP_ERCCL and no rank may hang.  Prints "corrupt ok: ...".
"""
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import _gossip_pkg  # noqa: E402
from oracle import lib as oracle  # noqa: E402

STAT_KEYS = ("injected", "lost", "new_bits", "receivers", "sends", "active", "crashed",
             "reports", "removals", "dup_reports")
# (push_ratio, unfiltered_pct, flat_max_words): always pull (per-receiver
# kernel at every width), adaptive direction with unfiltered dense rounds
MODES = {"pull": (0.0, 0, 0), "adaptive": (10.0, 90, 16)}


def run_ranks(pkg, g, origin, inject, P, crashes, cfg, errors=None):
    """P threads, rank k driving the context that owns partition k.  Rank
    failures raise, or with `errors` (a list) are appended to it as (rank,
    exception) and the ranks' outputs are None."""
    uid = pkg.GossipEngine.comm_unique_id()
    engs = []
    for k in range(P):
        e = pkg.GossipEngine(0, **cfg)
        e.load_graph(g)
        e.set_partition(k, P)
        e.set_messages(origin, inject)
        e.reset()
        engs.append(e)
    by_round = {}
    for v, r in crashes:
        by_round.setdefault(r, []).append(v)
    last = int(np.max(inject)) if inject is not None and len(inject) else 0
    out = [None] * P
    errs = []

    def rank(k):
        try:
            e = engs[k]
            e.comm_init(uid, P, k)
            stats, reports = [], []
            for r in range(254):
                if r in by_round:
                    e.crash(by_round[r])   # every rank gets the same global crash list
                st = e.round()
                stats.append(st)
                rep, nrep = e.reports()
                assert nrep == len(rep)
                reports.extend(map(tuple, rep.tolist()))
                if st["new_bits"] == 0 and r >= last:
                    break
            e.finalize()   # (an all-reduce of coverage / forwards: every rank at once)
            out[k] = dict(stats=stats, reports=reports, first=e.first(), digest=e.digest(), seen=e.seen(),
                          cov=e.coverage(), fwd=e.forwards(), part=e.partition())
        except BaseException as exc:   # surfaced below, after every thread ended
            errs.append((k, exc))

    ts = [threading.Thread(target=rank, args=(k,)) for k in range(P)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for e in engs:
        e.close()
    if errors is not None:
        errors.extend(errs)
    elif errs:
        raise RuntimeError(f"rank failures: {[(k, repr(e)) for k, e in errs]}")
    return out


def check(pkg, g, origin, inject, P, crashes, cfg, ref, by_arcs, tag):
    out = run_ranks(pkg, g, origin, inject, P, crashes, cfg)
    bounds = pkg.dist.partition_bounds(g.n, P, g.row_ptr if by_arcs else None)
    assert [o["part"] for o in out] == bounds, (tag, bounds)
    for o in out:   # counters are all-reduced: every rank holds the global ones
        assert len(o["stats"]) == ref["rounds"], (tag, len(o["stats"]), ref["rounds"])
        for a, b in zip(o["stats"], ref["stats"]):
            for k in STAT_KEYS:
                assert a[k] == b[k], (tag, k, a["round"], a[k], b[k])
        assert np.array_equal(o["cov"], ref["coverage"]), tag
        assert np.array_equal(o["fwd"], ref["forwards"]), tag
    assert sum(s["xchg_rows"] for s in out[0]["stats"]) > 0, tag
    reports = sorted(x for o in out for x in o["reports"])
    assert reports == sorted(map(tuple, ref["reports"].tolist())), tag
    W = out[0]["seen"].shape[1]
    assert np.array_equal(np.concatenate([o["first"] for o in out]), ref["first"]), tag
    assert np.array_equal(np.concatenate([o["digest"] for o in out]), ref["digest"]), tag
    assert np.array_equal(np.concatenate([o["seen"] for o in out]), ref["seen"][:, :W]), tag
    return sum(s["xchg_rows"] for s in out[0]["stats"])


def corrupt(pkg):
    """Every rank fails the round whose received entries the stand-in
    corrupted, with the same status, and the same round."""
    assert os.environ.get("GP_STANDIN_CORRUPT"), "set GP_STANDIN_CORRUPT=rank:k"
    g = pkg.overlay.barabasi_albert(3001, 2, seed=8)
    origin = pkg.overlay.random_origins(g.n, 200, seed=8)
    errs = []
    run_ranks(pkg, g, origin, None, 2, [], dict(track_first=1), errors=errs)
    assert len(errs) == 2, f"expected both ranks to fail, got {[(k, repr(e)) for k, e in errs]}"
    status = {k: getattr(e, "status", None) for k, e in errs}
    msgs = {k: str(e) for k, e in errs}
    assert set(status.values()) == {pkg._lib.GP_ERCCL}, msgs
    rounds = {k: m.split("(round ")[-1] for k, m in msgs.items()}
    assert len(set(rounds.values())) == 1, msgs
    print(f"corrupt ok: ranks=2 status={status[0]} {msgs[0]}", flush=True)


class ThreadAllGather:
    """In-process all-gather of byte strings among P threads (the host
    transport of a shard job, gp_shard_host_init)."""

    def __init__(self, P):
        self.P = P
        self.parts = [None] * P
        self.bar = threading.Barrier(P, timeout=120)

    def fn(self, k):
        def all_gather(b):
            self.parts[k] = b
            self.bar.wait()
            out = list(self.parts)
            self.bar.wait()
            return out
        return all_gather


def run_shard_job(pkg, g, origin, inject, P, crashes, cfg, transport):
    """A message-shard job of P ranks as P threads on one GPU: rank k runs the
    whole overlay for its word-aligned block of the table (dist.message_shard),
    stops when its own messages quiesce, finalizes and joins gp_shard_combine
    over the stand-in RCCL (transport "rccl") or the host all-gather ("host").
    Returns every rank's job record."""
    m = len(origin)
    inj = np.zeros(m, np.int32) if inject is None else np.asarray(inject, np.int32)
    uid = pkg.GossipEngine.comm_unique_id() if transport == "rccl" else None
    hag = ThreadAllGather(P) if transport == "host" else None
    engs = []
    for k in range(P):
        e = pkg.GossipEngine(0, **cfg)
        e.load_graph(g)
        lo, hi = pkg.dist.message_shard(m, P, k)
        e.set_message_shard(origin, inj, lo, hi)
        e.reset()
        engs.append((e, int(inj[lo:hi].max())))
    by_round = {}
    for v, r in crashes:
        by_round.setdefault(r, []).append(v)
    out = [None] * P
    errs = []

    def rank(k):
        try:
            e, last = engs[k]
            if transport == "rccl":
                e.shard_comm_init(uid, P, k)
            else:
                e.shard_host_init(hag.fn(k), P, k)
            info = e.shard_info()
            assert info == (P, k, 1 if transport == "rccl" else 2), info
            reports = set()
            for r in range(254):
                if r in by_round:
                    e.crash(by_round[r])
                st = e.round()
                rep, nrep = e.reports()
                assert nrep == len(rep)
                reports |= set(map(tuple, rep.tolist()))
                if st["new_bits"] == 0 and r >= last:
                    break
            e.finalize()
            job, ms = e.combine()
            fwd = None
            try:
                fwd = e.job_forwards(m)
            except pkg.GossipError as x:
                assert x.status == pkg._lib.GP_ENOTRACK
            out[k] = dict(job=job, ms=ms, digest=e.job_digest(), cov=e.job_coverage(m), fwd=fwd, reports=reports)
        except BaseException as exc:
            errs.append((k, exc))

    ts = [threading.Thread(target=rank, args=(k,)) for k in range(P)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for e, _ in engs:
        e.close()
    if errs:
        raise RuntimeError(f"rank failures: {[(k, repr(e)) for k, e in errs]}")
    return out


def check_shards(pkg, g, origin, inject, P, crashes, cfg, ref, transport, tag):
    """The job record every rank holds equals the oracle's whole run: per-round
    counters (receivers / active as unions), digest, coverage, forwards, and the
    dead-node reports of the ranks together."""
    out = run_shard_job(pkg, g, origin, inject, P, crashes, cfg, transport)
    for o in out:
        assert len(o["job"]) == ref["rounds"], (tag, len(o["job"]), ref["rounds"])
        for a, b in zip(o["job"], ref["stats"]):
            for k in STAT_KEYS:
                assert a[k] == b[k], (tag, k, a["round"], a[k], b[k])
        assert np.array_equal(o["digest"], ref["digest"]), tag
        assert np.array_equal(o["cov"], ref["coverage"]), tag
        if o["fwd"] is not None:
            assert np.array_equal(o["fwd"], ref["forwards"]), tag
        else:
            assert cfg.get("churn") and not cfg.get("track_msg_forwards"), tag
    reports = set().union(*(o["reports"] for o in out))
    assert reports == set(map(tuple, ref["reports"].tolist())), tag
    return max(o["ms"] for o in out)


def shards(pkg):
    """Message-shard jobs through gp_shard_combine: P = 1-4 on a BA overlay
    (200 messages, the reference cadence of 4 inject rounds, with and without
    churn), P = 2, 4, 8 on a Chung-Lu overlay with hubs (4096 messages: rank
    rows of 32, 16, 8 words), both transports."""
    cases = 0
    g = pkg.overlay.barabasi_albert(3001, 2, seed=8)
    origin = pkg.overlay.random_origins(g.n, 200, seed=8)
    inject = (np.arange(200) % 4).astype(np.int32)
    for churn in (False, True):
        kw = dict(churn=True, p_fail=0.02, churn_seed=3) if churn else {}
        crashes = [(int(origin[5]), 1), (17, 2)] if churn else []
        ref = oracle.run(g, origin, inject, crashes=crashes, want_first=True, **kw)
        for P in (1, 2, 3, 4):
            for transport in ("rccl", "host"):
                cfg = dict(track_msg_forwards=int(churn))
                if churn:
                    cfg.update(churn=1, p_fail=0.02, churn_seed=3)
                tag = f"shards ba3001 churn={churn} P={P} {transport}"
                t0 = time.time()
                ms = check_shards(pkg, g, origin, inject, P, crashes, cfg, ref, transport, tag)
                cases += 1
                print(f"ok  {tag}: combine {ms:.3f} ms, {time.time() - t0:.2f} s", flush=True)
    rp, col = oracle.chung_lu(50_000, 10, 2.4, 19)
    g = pkg.CSR(50_000, rp, col, False)
    origin = pkg.overlay.random_origins(g.n, 4096, seed=19)
    for churn in (False, True):
        kw = dict(churn=True, p_fail=0.01, churn_seed=6) if churn else {}
        ref = oracle.run(g, origin, None, nthreads=8, **kw)
        for P in (2, 4, 8):
            for transport in (("rccl", "host") if P == 4 else ("rccl",)):
                cfg = dict(hub_threshold=512)
                if churn:
                    cfg.update(churn=1, p_fail=0.01, churn_seed=6)
                tag = f"shards chung-lu 5e4 x 4096 churn={churn} P={P} {transport}"
                t0 = time.time()
                ms = check_shards(pkg, g, origin, None, P, [], cfg, ref, transport, tag)
                cases += 1
                print(f"ok  {tag}: combine {ms:.3f} ms, {time.time() - t0:.2f} s", flush=True)
    # a rank with no run to combine: every rank fails the combine with the
    # same status (it still joins the header all-gather), none waits forever
    g = pkg.overlay.barabasi_albert(3001, 2, seed=8)
    origin = pkg.overlay.random_origins(g.n, 200, seed=8)
    uid = pkg.GossipEngine.comm_unique_id()
    engs = []
    for k in range(2):
        e = pkg.GossipEngine(0)
        e.load_graph(g)
        lo, hi = pkg.dist.message_shard(200, 2, k)
        e.set_message_shard(origin, None, lo, hi)
        e.reset()
        engs.append(e)
    status = [None, None]

    def fail_rank(k):
        e = engs[k]
        e.shard_comm_init(uid, 2, k)
        if k == 0:
            e.run()
            e.finalize()
        try:
            e.combine()
        except pkg.GossipError as x:
            status[k] = x.status

    ts = [threading.Thread(target=fail_rank, args=(k,)) for k in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in ts), "a rank hung in the combine"
    for e in engs:
        e.close()
    assert status == [pkg._lib.GP_ESTATE] * 2, status
    print(f"shard cases ok: {cases}", flush=True)


def main():
    pkg = _gossip_pkg.load()
    lib_path = pkg._lib.load()._name
    assert "rccl_standin" in os.path.basename(lib_path), lib_path
    print(f"library: {lib_path} (stand-in mode: {'async' if os.environ.get('GP_STANDIN_ASYNC') == '1' else 'sync'})",
          flush=True)
    if "--corrupt" in sys.argv:
        corrupt(pkg)
        return
    if "--shards" in sys.argv:
        shards(pkg)
        return
    cases = 0
    # small BA overlay: every P, slice rule, churn setting and mode
    g = pkg.overlay.barabasi_albert(3001, 2, seed=8)
    origin = pkg.overlay.random_origins(g.n, 200, seed=8)
    inject = (np.arange(200) % 4).astype(np.int32)
    for churn in (False, True):
        kw = dict(churn=True, p_fail=0.02, churn_seed=3) if churn else {}
        crashes = [(int(origin[5]), 1), (17, 2)] if churn else []
        ref = oracle.run(g, origin, inject, crashes=crashes, want_first=True, **kw)
        for mode, (push_ratio, unfiltered_pct, flat_max_words) in MODES.items():
            for by_arcs in (0, 1):
                for P in (2, 3, 4):
                    cfg = dict(track_first=1, track_msg_forwards=int(churn), push_ratio=push_ratio,
                               unfiltered_pct=unfiltered_pct, flat_max_words=flat_max_words,
                               partition_by_arcs=by_arcs)
                    if churn:
                        cfg.update(churn=1, p_fail=0.02, churn_seed=3)
                    tag = f"ba3001 churn={churn} {mode} by_arcs={by_arcs} P={P}"
                    t0 = time.time()
                    rows = check(pkg, g, origin, inject, P, crashes, cfg, ref, by_arcs, tag)
                    cases += 1
                    print(f"ok  {tag}: {rows} boundary entries, {time.time() - t0:.2f} s", flush=True)
    # a Chung-Lu overlay with hubs, W = 64 rows (4096 messages), churn
    rp, col = oracle.chung_lu(50_000, 10, 2.4, 19)
    g = pkg.CSR(50_000, rp, col, False)
    origin = pkg.overlay.random_origins(g.n, 4096, seed=19)
    inject = (np.arange(4096) % 3).astype(np.int32)
    kw = dict(churn=True, p_fail=0.01, churn_seed=6)
    ref = oracle.run(g, origin, inject, want_first=True, nthreads=8, **kw)
    for P, by_arcs in ((2, 1), (4, 0), (8, 1)):   # P = 8: the node's rank count
        cfg = dict(track_first=1, track_msg_forwards=1, churn=1, p_fail=0.01, churn_seed=6, hub_threshold=512,
                   partition_by_arcs=by_arcs)
        tag = f"chung-lu 5e4 x 4096 churn P={P} by_arcs={by_arcs}"
        t0 = time.time()
        rows = check(pkg, g, origin, inject, P, [], cfg, ref, by_arcs, tag)
        cases += 1
        print(f"ok  {tag}: {rows} boundary entries, {time.time() - t0:.2f} s", flush=True)
    print(f"cases ok: {cases}", flush=True)


if __name__ == "__main__":
    main()
