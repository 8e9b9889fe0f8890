"""Protocol bridge: the reference's Seed/Peer line protocol in front of the
device engine.  Transport-free: lines in, lines out.
Whoever owns the sockets (a test, a localhost front-end) feeds the lines a
seed would read and delivers the lines the bridge returns; the socket, thread
and pickle framing code of the reference stays out of scope.

Line formats (reference file:line):
  peer handshake     "('ip', port)"                    Peer.py:95, parsed Seed.py:273-277
  seed handshake     "I am seed|('ip', port)"          Seed.py:246-262
  peer subset reply  JSON list of [ip, port]           Seed.py:286 (pickle.dumps there; JSON here)
  heartbeat          "Heartbeat from ('ip', port)"     Peer.py:368, Seed.py:263
  ping               "PING"                            Peer.py:307
  dead-node report   "Dead Node: ('ip', port)"         Peer.py:311, parsed Seed.py:358-372
  gossip             "%Y-%m-%d %H:%M:%S:ip:n"          Peer.py:398-399

The seed side is `seed.SeedRegistry` (first-3 subsets, removeDeadNode with
the reference's log lines).  Once every peer has registered, `start()`
freezes the overlay the peers would have wired (each peer sends on the
outgoing links to its subset, Peer.py:233-239, 402), loads it into a
GossipEngine and injects the reference schedule (10 messages per peer, one
every 5 rounds, Peer.py:396-408).  Each `step()` runs one device round and
renders what the reference's sockets would have carried in that second: the
gossip lines each peer receives for the first time, the dead-node reports
live peers send to the seed, and the seed's log lines for them.
"""
import ast
import json

import numpy as np

from . import peer as wire
from .overlay import CSR
from .seed import SeedRegistry

SEED_HELLO = "I am seed|"
HEARTBEAT = "Heartbeat from "
DEAD = "Dead Node:"


def _identity(text):
    """('ip', port) literal -> tuple, or None (ast.literal_eval: data only)."""
    try:
        v = ast.literal_eval(text.strip())
    except (ValueError, SyntaxError):
        return None
    if isinstance(v, tuple) and len(v) == 2 and isinstance(v[0], str) and isinstance(v[1], int):
        return v
    return None


def parse(line):
    """Classify one line of the protocol: returns (kind, payload) with kind in
    hello, seed_hello, heartbeat, ping, dead, gossip, unknown."""
    s = line.strip()
    if s == "PING":
        return "ping", None
    if s.startswith(SEED_HELLO):
        ident = _identity(s[len(SEED_HELLO):])
        return ("seed_hello", ident) if ident else ("unknown", s)
    if s.startswith(HEARTBEAT):
        ident = _identity(s[len(HEARTBEAT):])
        return ("heartbeat", ident) if ident else ("unknown", s)
    if s.startswith(DEAD):
        ident = _identity(s[len(DEAD):])
        return ("dead", ident) if ident else ("unknown", s)
    if s.startswith("("):
        ident = _identity(s)
        return ("hello", ident) if ident else ("unknown", s)
    # gossip: "YYYY-mm-dd HH:MM:SS:<ip>:<n>" -- the timestamp itself holds two colons
    parts = s.rsplit(":", 2)
    if len(parts) == 3 and parts[2].isdigit() and len(parts[0]) == 19:
        return "gossip", (parts[0], parts[1], int(parts[2]))
    return "unknown", s


def render_subset(subset):
    """The seed's reply to a peer handshake (Seed.py:286 sends pickle.dumps;
    the bridge frames it as one JSON line)."""
    return json.dumps([[ip, port] for ip, port in subset]) + "\n"


def parse_subset(line):
    return [tuple(x) for x in json.loads(line)]


class ProtocolBridge:
    def __init__(self, seed=("127.0.0.1", 0), device=0, messages_per_peer=wire.MESSAGES_PER_PEER,
                 period=wire.GOSSIP_PERIOD_ROUNDS, **engine_cfg):
        self.registry = SeedRegistry(*seed)
        self.seed = tuple(seed)
        self.device = device
        self.per_peer = messages_per_peer
        self.period = period
        self.engine_cfg = dict(track_first=1, track_digest=1)
        self.engine_cfg.update(engine_cfg)
        self.peers = []            # registration order = vertex id
        self.vertex = {}           # identity -> vertex id
        self.subsets = []
        self.engine = None
        self.round = 0

    # -- seed side: one incoming line -> reply lines -------------------------
    def handle(self, line):
        kind, arg = parse(line)
        if kind == "hello":
            if self.engine is not None:
                raise RuntimeError("overlay frozen: peers join before start()")
            subset = self.registry.register(arg)
            if subset is None:               # duplicate handshake: the seed closes it
                return []
            self.vertex[arg] = len(self.peers)
            self.peers.append(arg)
            self.subsets.append(list(subset))
            return [render_subset(subset)]
        if kind == "seed_hello":               # Seed.py:258-263: reply, then a heartbeat
            return [f"{SEED_HELLO}{self.seed}\n", wire.heartbeat_message(*self.seed)]
        if kind == "dead":
            self.registry.removeDeadNode(line)
            return []
        return []                              # heartbeats / pings / gossip: nothing for a seed to answer

    # -- the overlay the peers wired ----------------------------------------
    def overlay(self):
        """Directed in-CSR: peer k sends on its outgoing links to every peer of
        its subset but itself (Peer.py:233-239, 402)."""
        src, dst = [], []
        for k, sub in enumerate(self.subsets):
            for ident in sub:
                j = self.vertex.get(tuple(ident))
                if j is not None and j != k:
                    src.append(k)
                    dst.append(j)
        return CSR.from_arcs(len(self.peers), src, dst, directed=True)

    def schedule(self):
        origin, inject, count = wire.c1_schedule(len(self.peers), self.per_peer, self.period)
        return np.array(origin, np.int32), np.array(inject, np.int32), np.array(count, np.int32)

    def start(self):
        from .engine import GossipEngine
        if not self.peers:
            raise RuntimeError("no peer registered")
        self.origin, self.inject, self.count = self.schedule()
        self.engine = GossipEngine(self.device, **self.engine_cfg)
        self.engine.load_graph(self.overlay())
        self.engine.set_messages(self.origin, self.inject)
        self.engine.reset()
        self.round = 0
        self._first = np.full((len(self.peers), len(self.origin)), 255, np.uint8)

    def crash(self, ident):
        """Silent mode for one peer (Peer.py:437-439): from the next round on it
        neither heartbeats nor answers PINGs, nor receives or forwards."""
        self.engine.crash([self.vertex[tuple(ident)]])

    def gossip_line(self, m):
        o = int(self.origin[m])
        return wire.gossip_message(wire.round_time(int(self.inject[m])), self.peers[o][0], int(self.count[m]))

    # -- one round -------------------------------------------------------------
    def step(self):
        """One device round, rendered: deliveries [(to, line)] of this round's
        first receipts, reports [(reporter, line)] sent to the seed, and the
        seed's log lines for them."""
        st = self.engine.round()
        r = st["round"]
        first = self.engine.first()
        new = np.argwhere((first != self._first) & (first == r + 1))   # receipt round r + 1
        self._first = first
        deliveries = [(self.peers[v], self.gossip_line(m)) for v, m in new.tolist()]
        rep, total = self.engine.reports(max(int(st["reports"]), 1))
        if st["overflow"] or total != len(rep):
            # a subset of the Dead Node lines would let the seed log drift from
            # the engine's removals: the engine's report_capacity is too small
            raise RuntimeError(f"round {r}: {total} dead-node reports, the engine kept {len(rep)} "
                               "(raise report_capacity)")
        reports = [(self.peers[int(rp)], wire.dead_node_message(self.peers[int(d)]) + "\n")
                   for d, rp, _ in sorted(rep.tolist(), key=lambda x: (x[0], x[1]))]
        n_log = len(self.registry.logs)
        for _, line in reports:
            self.handle(line)
        self.round = r + 1
        return {"round": r, "stats": st, "deliveries": deliveries, "reports": reports,
                "seed_log": self.registry.logs[n_log:]}

    def run(self, max_rounds=254):
        last = int(self.inject.max())
        for _ in range(max_rounds):
            out = self.step()
            yield out
            if out["stats"]["new_bits"] == 0 and out["round"] >= last:
                return

    def close(self):
        if self.engine is not None:
            self.engine.close()
            self.engine = None
