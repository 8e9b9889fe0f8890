#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ by importing the reference.

This script is the ONLY place that touches /root/reference, and only in the
build container (the reference does not exist on the GPU box).  It drives the
reference's own classes directly (no sockets, no threads): every output here is
the reference's behaviour, captured as data.

Fixtures written (all small, committed):

  powerlaw_join.npz   -- edge lists of the reference-compatible join process:
                         node i calls NetworkBuilder.powerlaw_subset(peers[:i],
                         existing_endpoints, k=2) (demonstrate_powerlaw.py:7-39)
                         under random.seed(s); edges are symmetrised, sorted
                         (u < v) int32 pairs.  SURVEY.md §4.2 P5.
  c1_overlay.json     -- as-run first-3 registration rule: per-peer subsets from
                         Seed.get_peer_subset (Seed.py:127-129), topology after
                         updatePeerConnections (Seed.py:131-149), outgoing sets
                         after Peer.connect_to_peers' self-skip (Peer.py:233-239).
  c1_wire.json        -- wire strings produced by the reference: gossip lines
                         (Peer.py:395-408), heartbeat line (Peer.py:365-371),
                         dead-node report (Peer.py:298-313) and the direct
                         delivery matrix of C1 (who receives each message,
                         Peer.py:402-404).
  c1_remove.json      -- Seed.removeDeadNode transitions (Seed.py:358-406):
                         topology before/after, duplicate report no-op,
                         malformed report, count of broadcasts.

Run from the repo root:  python tests/golden/make_golden.py
"""
import datetime
import json
import os
import random
import sys
import tempfile

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))

JOIN_SIZES = (50, 300, 1000, 2000)
JOIN_SEEDS = (0, 1, 2, 3, 7)
BASE_PORT = 6000


def _import_reference():
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    import demonstrate_powerlaw  # noqa: E402
    import Peer  # noqa: E402
    import Seed  # noqa: E402
    return demonstrate_powerlaw, Peer, Seed


def make_join(dp):
    """Reference join (P5 recipe): O(N^2), a few seconds at N=2000."""
    out = {}
    for n in JOIN_SIZES:
        for s in JOIN_SEEDS:
            random.seed(s)
            peers = [("127.0.0.1", BASE_PORT + i) for i in range(n)]
            index = {p: i for i, p in enumerate(peers)}
            existing = []
            edges = set()
            for i in range(n):
                sel = dp.NetworkBuilder.powerlaw_subset(peers[:i], existing, k=2)
                for p in sorted(sel):  # order-free: only counts matter
                    j = index[p]
                    edges.add((min(i, j), max(i, j)))
                    existing.append(peers[i])
                    existing.append(p)
            arr = np.array(sorted(edges), dtype=np.int32).reshape(-1, 2)
            out[f"n{n}_s{s}"] = arr
            print(f"join n={n} s={s}: {len(arr)} edges", flush=True)
    np.savez_compressed(os.path.join(HERE, "powerlaw_join.npz"), **out)


class _FakeSock:
    def __init__(self, sink, name):
        self.sink, self.name = sink, name

    def sendall(self, data):
        self.sink.append((self.name, data.decode()))

    def close(self):
        pass


class _FixedDT:
    """Stand-in for datetime.datetime inside Peer.py: now() is fixed."""
    _t = datetime.datetime(2025, 2, 22, 12, 0, 0)

    @classmethod
    def now(cls):
        return cls._t


def make_c1(Peer, Seed, workdir):
    seed = Seed.SeedNode("127.0.0.1", 40121)
    logs = []
    seed.log = lambda m: logs.append(m)
    peers = [("127.0.0.1", 40001 + k) for k in range(10)]
    subsets, outgoing = [], []
    for p in peers:
        seed.peer_connections.addNeighbour(p[0], p[1], None)
        sub = seed.get_peer_subset()
        seed.updatePeerConnections(p, sub)
        subsets.append([list(x) for x in sub])
        outgoing.append([peers.index(x) for x in sub if x != p])
    topo = {str(list(k)): sorted(peers.index(x) for x in v)
            for k, v in seed.network_topology.items()}
    json.dump({"peers": [list(p) for p in peers], "subsets": subsets,
               "outgoing": outgoing, "topology": topo},
              open(os.path.join(HERE, "c1_overlay.json"), "w"), indent=1)

    # --- removeDeadNode transitions (Seed.py:358-406) ---
    before = {str(list(k)): sorted(peers.index(x) for x in v)
              for k, v in seed.network_topology.items()}
    bcast = []
    seed.broadcastMessage = lambda m: bcast.append(m)
    logs.clear()
    seed.removeDeadNode("Dead Node: ('127.0.0.1', 40005)")
    after1 = {str(list(k)): sorted(peers.index(x) for x in v)
              for k, v in seed.network_topology.items()}
    logs1, b1 = list(logs), list(bcast)
    logs.clear(); bcast.clear()
    seed.removeDeadNode("Dead Node: ('127.0.0.1', 40005)")
    logs2, b2 = list(logs), list(bcast)
    logs.clear(); bcast.clear()
    seed.removeDeadNode("Dead Node: garbage(")
    logs3 = list(logs)
    logs.clear(); bcast.clear()
    seed.removeDeadNode("Dead Node: ('127.0.0.1', 40001)")   # a hub
    after4 = {str(list(k)): sorted(peers.index(x) for x in v)
              for k, v in seed.network_topology.items()}
    logs4, b4 = list(logs), list(bcast)
    json.dump({"before": before,
               "remove_4": {"after": after1, "logs": logs1, "broadcasts": b1},
               "remove_4_again": {"logs": logs2, "broadcasts": b2},
               "malformed": {"logs": logs3},
               "remove_0": {"after": after4, "logs": logs4, "broadcasts": b4}},
              open(os.path.join(HERE, "c1_remove.json"), "w"), indent=1)

    # --- wire strings + direct-delivery matrix (Peer.py:395-408) ---
    Peer.datetime.datetime = _FixedDT
    Peer.time.sleep = lambda s: None
    deliveries = []   # [origin, count, receiver]
    gossip_lines = {}
    for k, p in enumerate(peers):
        node = Peer.PeerNode(p[0], p[1], os.path.join(workdir, "config.txt"))
        node.log = lambda m: None
        sink = []
        node.peer_connections = {peers[j]: _FakeSock(sink, j) for j in outgoing[k]}
        node.gossip_sender()
        # gossip is sent even with no outgoing link: record the rendered line once
        for name, line in sink:
            cnt = int(line.strip().rsplit(":", 1)[1])
            deliveries.append([k, cnt, name])
            gossip_lines.setdefault(str(k), {})[str(cnt)] = line
    # heartbeat line (Peer.py:365-371): one pass of the loop
    hb_sink = []
    node = Peer.PeerNode("127.0.0.1", 40001, os.path.join(workdir, "config.txt"))
    node.log = lambda m: None
    node.peer_connections = {peers[1]: _FakeSock(hb_sink, 1)}

    def _stop(_s, node=node):
        node.running = False
    Peer.time.sleep = _stop
    node.periodic_peer_heartbeat()
    # dead-node report (Peer.py:298-313): stale outgoing link, PING unanswered
    dn = Peer.PeerNode("127.0.0.1", 40002, os.path.join(workdir, "config.txt"))
    dn.log = lambda m: None
    ping_sink = []
    dn.peer_connections = {peers[0]: _FakeSock(ping_sink, 0)}
    dn.peer_last_heartbeat = {peers[0]: 0.0}
    dn.reported_identity = {peers[0]: peers[0]}
    real_time = Peer.time.time
    Peer.time.time = lambda: 100.0

    def _sleep(s, dn=dn):
        if s >= 10:
            dn.running = False
    Peer.time.sleep = _sleep
    dn.monitor_peer_heartbeats()
    Peer.time.time = real_time
    dead = []
    while not dn.seed_queue.empty():
        dead.append(dn.seed_queue.get())
    json.dump({"gossip_lines": gossip_lines,
               "deliveries": sorted(deliveries),
               "heartbeat": hb_sink[0][1] if hb_sink else None,
               "ping": ping_sink[0][1] if ping_sink else None,
               "dead_report": dead,
               "fixed_now": _FixedDT._t.strftime("%Y-%m-%d %H:%M:%S")},
              open(os.path.join(HERE, "c1_wire.json"), "w"), indent=1)


def main():
    dp, Peer, Seed = _import_reference()
    with tempfile.TemporaryDirectory() as wd:
        cwd = os.getcwd()
        os.chdir(wd)               # SeedNode/PeerNode write config/log files in cwd
        try:
            make_c1(Peer, Seed, wd)
        finally:
            os.chdir(cwd)
    make_join(dp)


if __name__ == "__main__":
    main()
