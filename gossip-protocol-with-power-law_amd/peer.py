"""Peer-side wire formats and identities (renderers only -- the transport is the
device engine).

  gossip line     "{%Y-%m-%d %H:%M:%S}:{ip}:{count}\\n"      Peer.py:398-399
  heartbeat       "Heartbeat from ('ip', port)\\n"            Peer.py:368
  ping            "PING\\n"                                   Peer.py:307
  dead report     "Dead Node: ('ip', port)"  (+"\\n" on send)  Peer.py:311, 148-149

The reference's gossip string carries no port, so two peers on one host that
generate message #n in the same second render identically (SURVEY.md §0
finding 5).  The engine's message identity is therefore (origin vertex, n);
PeerDirectory gives every vertex a distinct (ip, port) so rendered strings stay
unique when they are hashed into a Message-List (oracle/harness.py).
"""
import datetime

TS_FORMAT = "%Y-%m-%d %H:%M:%S"
EPOCH = datetime.datetime(2025, 2, 22, 12, 0, 0)   # synthetic clock of round 0
SECONDS_PER_ROUND = 1                               # C1 cadence: 1 round = 1 s
GOSSIP_PERIOD_ROUNDS = 5                            # Peer.py:408 sleeps 5 s
MESSAGES_PER_PEER = 10                              # Peer.py:397


def timestamp(ts):
    if isinstance(ts, datetime.datetime):
        return ts.strftime(TS_FORMAT)
    return str(ts)


def gossip_message(ts, ip, count):
    return f"{timestamp(ts)}:{ip}:{count}\n"


def heartbeat_message(ip, port):
    return f"Heartbeat from {(ip, port)}\n"


def ping_message():
    return "PING\n"


def dead_node_message(identity):
    return f"Dead Node: {identity}"


def round_time(r):
    return EPOCH + datetime.timedelta(seconds=r * SECONDS_PER_ROUND)


class PeerDirectory:
    """vertex id <-> (ip, port).  Default: every peer on 127.0.0.1 with
    consecutive ports (the reference's localhost setup, readme.md:2-4); with
    distinct_ips=True each vertex gets its own 10.x.y.z address so the rendered
    gossip strings are unique per origin."""

    def __init__(self, n, base_port=40001, ip="127.0.0.1", distinct_ips=False):
        self.n = n
        self.base_port = base_port
        self.ip = ip
        self.distinct_ips = distinct_ips

    def identity(self, v):
        if self.distinct_ips:
            return (f"10.{(v >> 16) & 255}.{(v >> 8) & 255}.{v & 255}", self.base_port + (v >> 24))
        return (self.ip, self.base_port + v)

    def vertex(self, identity):
        ip, port = identity
        if self.distinct_ips:
            a, b, c, d = (int(x) for x in ip.split("."))
            return ((port - self.base_port) << 24) | (b << 16) | (c << 8) | d
        return port - self.base_port


def c1_schedule(n_peers, per_peer=MESSAGES_PER_PEER, period=GOSSIP_PERIOD_ROUNDS):
    """C1 injection schedule: peer k generates message #c (c = 1..10) at round
    period*(c-1) (Peer.py:396-408).  Message id = k*per_peer + (c-1)."""
    origin, inject, count = [], [], []
    for k in range(n_peers):
        for c in range(1, per_peer + 1):
            origin.append(k)
            inject.append(period * (c - 1))
            count.append(c)
    return origin, inject, count
