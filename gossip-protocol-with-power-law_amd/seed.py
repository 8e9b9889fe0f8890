"""Seed registry: host-side mirror of the reference's SeedNode topology logic.

Same method names, argument meaning and error behaviour as Seed.py, minus the
sockets and threads (the transport is replaced by the device engine):
  addNeighbour / removeNeighbour      Seed.py:40-54
  get_peer_subset                     Seed.py:127-129
  updatePeerConnections               Seed.py:131-149
  removeDeadNode                      Seed.py:358-406
The registry is what the engine's dead-node reports are fed into: the first
report for a vertex removes it (and every incident edge), later reports hit
the "not found" branch (Seed.py:373-375).
"""
import ast


class Peer:
    """Seed.py:11-27."""

    def __init__(self, ip, port, socket_obj=None):
        self.ip = ip
        self.port = port
        self.socket = socket_obj
        self.connections = set()

    def add_connection(self, peer_tuple):
        self.connections.add(peer_tuple)

    def __repr__(self):
        return f"Peer({self.ip}, {self.port}, connections={list(self.connections)})"


class SeedNodeConnections:
    """Seed.py:29-54."""

    def __init__(self, ip, port):
        self.ip = ip
        self.port = port
        self.neighbour = {}
        self.count = 0

    def addNeighbour(self, ip, port, socket_obj=None):
        aggregate = (ip, port)
        if aggregate in self.neighbour:
            return False
        self.neighbour[aggregate] = Peer(ip, port, socket_obj)
        self.count += 1
        return True

    def removeNeighbour(self, ip, port):
        aggregate = (ip, port)
        if aggregate in self.neighbour:
            del self.neighbour[aggregate]
            self.count -= 1
            return True
        return False


class SeedRegistry:
    """One logical seed (the sim models the seed mesh as one registry,
    SURVEY.md C11).  `logs` collects the reference's log lines verbatim and
    `broadcasts` the lines it would send to other seeds."""

    def __init__(self, ip="127.0.0.1", port=0):
        self.ip = ip
        self.port = port
        self.peer_connections = SeedNodeConnections(ip, port)
        self.known_peers = []
        self.network_topology = {}
        self.logs = []
        self.broadcasts = []

    def log(self, message):
        self.logs.append(message)

    def broadcastMessage(self, message):
        self.broadcasts.append(message)

    def register(self, peer):
        """Registration handshake minus transport (Seed.py:280-291): add the
        peer, hand it the subset, record the links."""
        if not self.peer_connections.addNeighbour(peer[0], peer[1], None):
            self.log("Duplicate peer connection from " + str(peer))
            return None
        subset = self.get_peer_subset()
        self.updatePeerConnections(peer, subset)
        return subset

    def get_peer_subset(self):
        keys = [k for k in self.peer_connections.neighbour.keys() if k != (self.ip, self.port)]
        return keys[:3] if len(keys) > 3 else keys

    def updatePeerConnections(self, new_peer, subset):
        subset_set = set(subset)
        if new_peer in self.network_topology:
            self.network_topology[new_peer] = self.network_topology[new_peer].union(subset_set)
        else:
            self.network_topology[new_peer] = subset_set
        for p in subset_set:
            if p in self.network_topology:
                self.network_topology[p].add(new_peer)
            else:
                self.network_topology[p] = {new_peer}
        if new_peer in self.peer_connections.neighbour:
            peer_instance = self.peer_connections.neighbour[new_peer]
            for p in subset_set:
                peer_instance.add_connection(p)
                if p in self.peer_connections.neighbour:
                    self.peer_connections.neighbour[p].add_connection(new_peer)

    def removeDeadNode(self, deadMessage):
        """Returns True if the report removed a node, False for the reference's
        no-op branches (malformed report, "not found").  Observable behaviour
        (log lines, the doubled removal/broadcast block Seed.py:393-406) is kept."""
        deadMessage = deadMessage.strip()
        parts = deadMessage.split(":", 1)
        if parts[0] != "Dead Node":
            return False
        try:
            reported = ast.literal_eval(parts[1].strip())
        except Exception as e:
            self.log("Error parsing dead node message: " + str(e))
            return False
        found = None
        for peer in list(self.network_topology.keys()):
            if peer[0] == reported[0] and peer[1] == reported[1]:
                found = peer
                break
        if found is None:
            self.log("Dead node " + str(reported) + " not found in network topology; no broadcast sent.")
            return False
        deadNode = found
        if self.peer_connections.removeNeighbour(deadNode[0], deadNode[1]):
            self.log("Removed dead node from peer_connections: " + str(deadNode))
        else:
            self.log("Dead node " + str(deadNode) + " not found in peer_connections; proceeding with removal.")
        if deadNode in self.network_topology:
            del self.network_topology[deadNode]
        for node in list(self.network_topology.keys()):
            if deadNode in self.network_topology[node]:
                self.network_topology[node].discard(deadNode)
        for _ in range(2):   # the reference runs this block twice (Seed.py:393-406)
            if deadNode in self.known_peers:
                self.known_peers.remove(deadNode)
            self.log("Completely removed dead node: " + str(deadNode))
            self.broadcastMessage(f"Dead Node: {deadNode}\n")
        return True

    def apply_reports(self, report_lines):
        """Feed rendered 'Dead Node: ...' lines (Peer.py:311) in order; returns
        (removals, no-ops) -- the seed-side view of gp_round_stats
        removals / dup_reports."""
        removed = noop = 0
        for line in report_lines:
            if self.removeDeadNode(line):
                removed += 1
            else:
                noop += 1
        return removed, noop
