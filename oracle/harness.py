"""Per-peer Message-List harness -- the in-process CPU restatement of the
reference's peer logic with forwarding added as the north star specifies.
TEST INFRASTRUCTURE ONLY (small graphs; pure Python loops).

Each peer keeps, like a reference PeerNode, its own state:
  message_list   set of sha256 digests of the rendered gossip strings
                 ("{ts}:{ip}:{count}", Peer.py:398-399) -- the Message-List
  out links      the peers it sends to (Peer.py:402: outgoing connections;
                 undirected overlays: every link)
  last heartbeat / miss counter per link (Peer.py:298-363, in rounds)
Per round r:
  L  crash draws -> crashed peers stop heartbeating and answering PINGs
     (silent mode, Peer.py:437-439, 367, 202); every live peer holding a link to
     a peer that missed `miss_threshold` heartbeats reports
     "Dead Node: ('ip', port)" (Peer.py:311); the seed removes the first report's
     node and every incident link (Seed.py:380-391), later reports are
     "not found" no-ops (Seed.py:373-375).
  I  messages generated in round r at live origins (gossip_sender, Peer.py:395-400)
  E  every live peer sends each message it first received last round (or
     generated now) to all its links whose far end is not removed
     (Peer.py:402-404); a receiver that is up and has not seen the digest
     adds it to its Message-List and forwards it next round (forward-once).
This is independent code from both the C oracle and the HIP engine: no bit
packing, no CSR tricks, string hashing for dedup.
"""
import datetime
import hashlib
import math

import numpy as np

MASK = (1 << 64) - 1
EPOCH = datetime.datetime(2025, 2, 22, 12, 0, 0)


def splitmix64(x):
    z = (x + 0x9E3779B97F4A7C15) & MASK
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK
    return z ^ (z >> 31)


def draw(seed, stream, idx):
    key = splitmix64(seed ^ splitmix64(stream))
    return splitmix64((key + idx * 0x9E3779B97F4A7C15) & MASK)


def identity(v):
    """Distinct (ip, port) per vertex so the rendered strings are unique."""
    return (f"10.{(v >> 16) & 255}.{(v >> 8) & 255}.{v & 255}", 40001 + (v >> 24))


def render(origin, count, inject_round):
    ts = (EPOCH + datetime.timedelta(seconds=int(inject_round))).strftime("%Y-%m-%d %H:%M:%S")
    return f"{ts}:{identity(origin)[0]}:{count}"


class HarnessPeer:
    def __init__(self, vid):
        self.vid = vid
        self.message_list = set()
        self.first = {}          # message index -> receipt round
        self.outbox = []         # messages to forward this round
        self.up = True
        self.removed = False
        self.miss = 0


def run(n, in_lists, directed, origin, inject_round, churn=False, p_fail=0.0, churn_seed=0,
        miss_threshold=3, crashes=(), max_rounds=254):
    """in_lists[v] = senders to v.  Returns first matrix [n][m] (255 = never),
    per-round stats, per-message coverage/forwards, reports (dead, reporter, r)."""
    m = len(origin)
    out_lists = [[] for _ in range(n)]
    for v in range(n):
        for u in in_lists[v]:
            out_lists[u].append(v)
    # heartbeat links of a peer: both directions (Peer.py:369-392 covers
    # outgoing and incoming connections); one report per link
    links = [list(in_lists[v]) + (list(out_lists[v]) if directed else []) for v in range(n)]
    peers = [HarnessPeer(v) for v in range(n)]
    counts, per_origin = [], {}
    for k in range(m):
        per_origin[origin[k]] = per_origin.get(origin[k], 0) + 1
        counts.append(per_origin[origin[k]])
    digests = [hashlib.sha256(render(origin[k], counts[k], inject_round[k]).encode()).hexdigest()
               for k in range(m)]
    p_thresh = int(math.ldexp(p_fail, 64)) if 0.0 < p_fail < 1.0 else 0
    crash_at = {}
    for v, r in crashes:
        crash_at.setdefault(r, set()).add(v)
    registry_alive = set(range(n))          # seed topology vertices (Seed.py:70-71)
    deg_live = [len(out_lists[v]) for v in range(n)]
    forwards = [0] * m
    stats, reports = [], []
    last_inject = max(inject_round) if m else -1
    liveness = churn or bool(crashes)
    for r in range(max_rounds):
        st = dict(injected=0, lost=0, new_bits=0, receivers=0, sends=0, active=0, crashed=0,
                  reports=0, removals=0, dup_reports=0)
        if liveness:
            for p in peers:
                if p.up and not p.removed:
                    c = p.vid in crash_at.get(r, ())
                    if not c and churn and p_fail >= 1.0:
                        c = True
                    if not c and churn and p_thresh and draw(churn_seed, 0x100 + r, p.vid) < p_thresh:
                        c = True
                    if c:
                        p.up = False
                        p.outbox = []       # crash-stop: pending forwards die with it
                        st["crashed"] += 1
                if not p.up:
                    p.miss = min(p.miss + 1, 255)
            cand = [p for p in peers if not p.up and p.miss == miss_threshold and not p.removed]
            for p in cand:
                lines = [(p.vid, u) for u in links[p.vid] if peers[u].up and not peers[u].removed]
                for dead, reporter in lines:      # the seed: first removes, rest no-ops
                    reports.append((dead, reporter, r))
                    st["reports"] += 1
                    if dead in registry_alive:
                        registry_alive.discard(dead)
                        st["removals"] += 1
                        p.removed = True
                        for u in in_lists[dead]:
                            deg_live[u] -= 1
                    else:
                        st["dup_reports"] += 1
        for k in range(m):
            if inject_round[k] != r:
                continue
            p = peers[origin[k]]
            if not p.up or p.removed:
                st["lost"] += 1
                continue
            p.message_list.add(digests[k])
            p.first[k] = r
            p.outbox.append(k)
            st["injected"] += 1
        inbox = {}
        for p in peers:
            if not p.outbox or not p.up:
                continue
            st["active"] += 1
            for k in p.outbox:
                forwards[k] += deg_live[p.vid]
                st["sends"] += deg_live[p.vid]
                for w in out_lists[p.vid]:
                    q = peers[w]
                    if q.removed:
                        continue          # the seed dropped the link
                    if q.up:
                        inbox.setdefault(w, []).append(k)
            p.outbox = []
        for w, ks in inbox.items():
            q = peers[w]
            new = 0
            for k in ks:
                if digests[k] not in q.message_list:     # Message-List dedup
                    q.message_list.add(digests[k])
                    q.first[k] = r + 1
                    q.outbox.append(k)                   # forward once, next round
                    new += 1
            st["new_bits"] += new
            st["receivers"] += new > 0
        stats.append(st)
        if st["new_bits"] == 0 and r >= last_inject:
            break
    first = np.full((n, m), 255, dtype=np.uint8)
    for p in peers:
        for k, rr in p.first.items():
            first[p.vid, k] = rr
    coverage = (first != 255).sum(axis=0).astype(np.uint64)
    return {"first": first, "stats": stats, "coverage": coverage,
            "forwards": np.array(forwards, dtype=np.uint64), "reports": reports,
            "rounds": len(stats)}
