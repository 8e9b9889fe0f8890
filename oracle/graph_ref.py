"""Pure-Python/numpy restatement of the Chung-Lu overlay definition
 -- TEST INFRASTRUCTURE, small n only.  Independent of both
oracle/gossip_oracle.c (or_chung_lu) and csrc/graph_build.hip; the three must
produce the same CSR bit for bit."""
import math

import numpy as np

from .harness import MASK, splitmix64


def _key(seed, stream):
    return splitmix64(seed ^ splitmix64(stream))


def _draw(key, idx):
    return splitmix64((key + idx * 0x9E3779B97F4A7C15) & MASK)


def _below(r, n):
    return (r * n) >> 64


def alias_table(n, gamma):
    alpha = 1.0 / (gamma - 1.0)
    q = [max(1, int(math.floor(math.ldexp((i + 1) ** -alpha, 32)))) for i in range(n)]
    T = sum(q)
    prob = [T] * n
    alias = list(range(n))
    p = [qi * n for qi in q]
    small = [i for i in range(n) if p[i] < T]
    large = [i for i in range(n) if p[i] >= T]
    while small and large:
        s = small.pop()
        l = large.pop()
        prob[s] = p[s]
        alias[s] = l
        p[l] -= T - p[s]
        (small if p[l] < T else large).append(l)
    return prob, alias, T


def chung_lu(n, dbar, gamma, seed):
    prob, alias, T = alias_table(n, gamma)
    krel = _key(seed, 2)
    keys = sorted(((_draw(krel, i) >> 32) << 32) | i for i in range(n))
    new_id = [0] * n
    for k, key in enumerate(keys):
        new_id[key & 0xFFFFFFFF] = k
    E = int(math.floor(dbar * n / 2.0))
    kedge = _key(seed, 1)
    arcs = set()
    for e in range(E):
        b = 4 * e
        ends = []
        for h in (0, 2):
            i = _below(_draw(kedge, b + h), n)
            x = _below(_draw(kedge, b + h + 1), T)
            ends.append(i if x < prob[i] else alias[i])
        u, v = ends
        if u == v:
            continue
        a, c = new_id[u], new_id[v]
        arcs.add((a, c))
        arcs.add((c, a))
    arcs = sorted(arcs)
    row_ptr = np.zeros(n + 1, np.int64)
    for a, _ in arcs:
        row_ptr[a + 1] += 1
    np.cumsum(row_ptr, out=row_ptr)
    col = np.array([c for _, c in arcs], dtype=np.int32)
    return row_ptr, col
