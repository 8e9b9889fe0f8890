"""Overlay builders -> canonical in-CSR (host side of the seed registry).

The reference wires peers in two ways:
  * as run: Seed.get_peer_subset hands each newly registered peer the first 3
    registered peers (Seed.py:127-129, called at Seed.py:285); the peer connects
    to them except itself (Peer.py:233-239) and sends gossip on those OUTGOING
    links only (Peer.py:402).  -> first3_overlay (directed).
  * degree-weighted selection NetworkBuilder.powerlaw_subset
    (demonstrate_powerlaw.py:7-39), never called by the reference; here driven
    by a join process with the reference's exact RNG call
    sequence.  -> powerlaw_join (undirected, bit-exact with the reference).
Synthetic power-law overlays for the throughput configs:
  * barabasi_albert(n, m, seed)   (BASELINE.json config 2)
  * Chung-Lu: built on the device, GossipEngine.build_chung_lu (configs 3-5).

CSR convention: row v lists In(v) = {u : arc u->v} (the peers whose gossip v
receives), sorted, de-duplicated, no self-loops.
"""
import math
import random
from collections import defaultdict
from dataclasses import dataclass

import numpy as np


@dataclass
class CSR:
    n: int
    row_ptr: np.ndarray   # int64 [n+1]
    col: np.ndarray       # int32 [nnz]
    directed: bool = False

    @property
    def nnz(self):
        return int(self.row_ptr[-1])

    def in_neighbors(self, v):
        return self.col[self.row_ptr[v]:self.row_ptr[v + 1]]

    def in_degree(self):
        return np.diff(self.row_ptr).astype(np.int64)

    def arcs(self):
        """(src, dst) int64 arrays of every arc src->dst."""
        dst = np.repeat(np.arange(self.n, dtype=np.int64), np.diff(self.row_ptr))
        return self.col.astype(np.int64), dst

    def transpose(self):
        src, dst = self.arcs()
        return CSR.from_arcs(self.n, dst, src, directed=True)

    def out_degree(self):
        if not self.directed:
            return self.in_degree()
        return np.bincount(self.col, minlength=self.n).astype(np.int64)

    def edges_undirected(self):
        """Sorted unique (u < v) pairs of an undirected CSR."""
        src, dst = self.arcs()
        keep = src < dst
        e = np.stack([src[keep], dst[keep]], axis=1)
        return e[np.lexsort((e[:, 1], e[:, 0]))]

    @staticmethod
    def from_arcs(n, src, dst, directed):
        src = np.asarray(src, dtype=np.int64)
        dst = np.asarray(dst, dtype=np.int64)
        if src.size and (src.min() < 0 or src.max() >= n or dst.min() < 0 or dst.max() >= n):
            raise ValueError("vertex id out of range")
        if not directed:
            src, dst = np.concatenate([src, dst]), np.concatenate([dst, src])
        keep = src != dst
        src, dst = src[keep], dst[keep]
        key = np.unique(dst * np.int64(n) + src)
        d, s = key // n, key % n
        row_ptr = np.zeros(n + 1, dtype=np.int64)
        np.cumsum(np.bincount(d, minlength=n), out=row_ptr[1:])
        return CSR(n, row_ptr, s.astype(np.int32), bool(directed))

    @staticmethod
    def from_edges(n, edges, directed=False):
        e = np.asarray(edges, dtype=np.int64).reshape(-1, 2)
        return CSR.from_arcs(n, e[:, 0], e[:, 1], directed)


# --------------------------------------------------------------------------
# as-run first-3 rule

def first3_subsets(n_peers):
    """Subset the seed hands peer k (0-based registration order): the first 3
    registered peers, the new peer itself included (Seed.py:127-129 runs after
    addNeighbour, Seed.py:281)."""
    return [list(range(min(3, k + 1))) for k in range(n_peers)]


def first3_overlay(n_peers):
    """Directed overlay k -> j for every j in peer k's subset, j != k
    (Peer.py:233-239 skips itself; gossip flows on outgoing links, Peer.py:402)."""
    src, dst = [], []
    for k, sub in enumerate(first3_subsets(n_peers)):
        for j in sub:
            if j != k:
                src.append(k)
                dst.append(j)
    return CSR.from_arcs(n_peers, src, dst, directed=True)


# --------------------------------------------------------------------------
# degree-weighted selection (demonstrate_powerlaw.py:7-39)

class NetworkBuilder:
    """Mirror of demonstrate_powerlaw.NetworkBuilder with the same signature,
    RNG call sequence and error behaviour (the `except:` fallback to
    random.sample, demonstrate_powerlaw.py:38-39).  Membership of the returned
    list is deterministic for a given `random` state; its ORDER, like the
    reference's list(set(...)), is not part of the contract."""

    @staticmethod
    def powerlaw_subset(peers, existing_connections, k=2, rng=None):
        rng = rng if rng is not None else random._inst
        if not peers:
            return []
        degree_count = defaultdict(int)
        for ip, port in existing_connections:
            degree_count[(ip, port)] += 1
        weights = [degree_count.get(p, 1) for p in peers]
        n = max(k, min(len(peers), 5))
        hi = min(len(peers), n * 3)
        if n > hi:   # randint raises ValueError before drawing -> except branch
            return rng.sample(peers, min(len(peers), n))
        cnt = rng.randint(n, hi)
        cum = np.cumsum(weights)
        total = float(cum[-1])
        idx = [math.floor(rng.random() * total) for _ in range(cnt)]
        pos = np.searchsorted(cum, idx, side="right")
        return list({peers[int(j)] for j in pos})


class _Fenwick:
    def __init__(self, n):
        self.n = n
        self.t = [0] * (n + 1)
        self.total = 0

    def add(self, i, d):
        self.total += d
        i += 1
        while i <= self.n:
            self.t[i] += d
            i += i & -i

    def find(self, x):
        """Smallest index j with prefix(j+1) > x (== bisect_right on the cumsum)."""
        pos, rem = 0, x
        step = 1 << self.n.bit_length()
        while step:
            nxt = pos + step
            if nxt <= self.n and self.t[nxt] <= rem:
                pos = nxt
                rem -= self.t[nxt]
            step >>= 1
        return pos


def powerlaw_join(n, seed, k=2):
    """Join process over NetworkBuilder.powerlaw_subset: peer i selects among
    peers 0..i-1 with weight max(degree, 1) (demonstrate_powerlaw.py:19-27),
    n = max(k, min(i, 5)) (:30), randint(n, min(i, 3n)) THEN choices (:32-35),
    dedup (:37); links are symmetric.  O(log n) per pick (Fenwick tree), with
    the reference's exact `random.Random(seed)` call sequence -- edge-for-edge
    identical to the O(n^2) reference (tests/golden/powerlaw_join.npz)."""
    rng = random.Random(seed)
    fen = _Fenwick(max(n, 1))
    deg = [0] * n
    src, dst = [], []
    for i in range(n):
        L = i
        if L == 0:
            sel = ()
        else:
            nn = max(k, min(L, 5))
            hi = min(L, nn * 3)
            if nn > hi:
                sel = rng.sample(range(L), min(L, nn))
            else:
                cnt = rng.randint(nn, hi)
                total = float(fen.total)
                sel = {fen.find(math.floor(rng.random() * total)) for _ in range(cnt)}
        for j in sel:
            src.append(i)
            dst.append(j)
            # weight = degree once present in existing_connections, else 1
            old_j = max(deg[j], 1)
            deg[j] += 1
            fen.add(j, max(deg[j], 1) - old_j)
            deg[i] += 1
        fen.add(i, max(deg[i], 1))   # peer i becomes selectable for later peers
    return CSR.from_arcs(n, src, dst, directed=False)


# --------------------------------------------------------------------------
# Barabasi-Albert (BASELINE.json config 2)

def barabasi_albert(n, m, seed):
    """Preferential attachment: start from a star on m+1 vertices; vertex s >= m+1
    attaches to m distinct targets drawn uniformly from the endpoint list
    (probability ∝ degree) with random.Random(seed).choice.  This is the
    published networkx 3.x barabasi_albert_graph procedure, so the edge set
    equals nx.barabasi_albert_graph(n, m, seed) (tests/test_overlay.py)."""
    if m < 1 or m >= n:
        raise ValueError("need 1 <= m < n")
    rng = random.Random(seed)
    src = list(range(1, m + 1))
    dst = [0] * m
    repeated = [0] * m + list(range(1, m + 1))
    for s in range(m + 1, n):
        targets = set()
        while len(targets) < m:
            targets.add(rng.choice(repeated))
        for t in targets:
            src.append(s)
            dst.append(t)
        repeated.extend(targets)
        repeated.extend([s] * m)
    return CSR.from_arcs(n, src, dst, directed=False)


def random_origins(n, m, seed):
    """Message origins of the throughput configs: PCG64(seed + 100), SURVEY.md §8d."""
    return np.random.Generator(np.random.PCG64(seed + 100)).integers(0, n, m).astype(np.int32)


def spread_keys(row_ptr, col, origin, hops=2):
    """Host restatement of gp_spread_keys (DESIGN.md §3.4 "message order"):
    arc endpoints within `hops` of each origin -- 1: its degree, 2: the sum of
    its neighbours' degrees, 3: the sum over its neighbours of their hops-2
    key.  u64, exact."""
    rp = np.asarray(row_ptr, dtype=np.int64)
    col = np.asarray(col, dtype=np.int64)
    o = np.asarray(origin, dtype=np.int64)
    if hops not in (1, 2, 3):
        raise ValueError("hops must be 1, 2 or 3")
    val = np.diff(rp).astype(np.uint64)
    for _ in range(hops - 2):   # val <- per-vertex sum of val over the in-list
        val = np.add.reduceat(np.append(val[col], np.uint64(0)), np.minimum(rp[:-1], col.size)) * (np.diff(rp) > 0)
        val = val.astype(np.uint64)
    if hops == 1:
        return val[o]
    return np.array([val[col[rp[v]:rp[v + 1]]].sum(dtype=np.uint64) for v in o], dtype=np.uint64)


def spread_order(keys, inject_round=None):
    """Bit order of a message table that groups messages by how fast they
    spread (DESIGN.md §3.4 "message order"): by inject round, then by spread
    key descending (gp_spread_keys), ties by index.  Messages from
    well-connected origins complete early and then share 128-B lines of the
    Message-List rows, which the late early-exit rounds skip whole.  Returns
    the permutation p: message k of the ordered table is message p[k] of the
    given one."""
    keys = np.asarray(keys, dtype=np.float64)
    idx = np.arange(keys.size)
    r = np.zeros(keys.size, np.int64) if inject_round is None else np.asarray(inject_round, np.int64)
    return np.lexsort((idx, -keys, r))
