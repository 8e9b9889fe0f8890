"""Protocol bridge: the reference's line protocol in
front of the engine.  CPU tests pin the codec and the seed side against the
reference's own fixtures (tests/golden/c1_wire.json, c1_overlay.json); GPU
tests run C1 through the bridge and compare every rendered delivery with the
per-peer sha256 harness (oracle/harness.py) and the dead-node reports with the
C oracle."""
import json
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _golden(name):
    return json.load(open(os.path.join(GOLDEN, name)))


def _bridge(pkg, n=10, **cfg):
    b = pkg.bridge.ProtocolBridge(**cfg)
    replies = [b.handle(str(("127.0.0.1", 40001 + k)) + "\n") for k in range(n)]
    return b, replies


def test_codec_reads_the_reference_lines(pkg):
    br = pkg.bridge
    wire = _golden("c1_wire.json")
    assert br.parse(wire["heartbeat"]) == ("heartbeat", ("127.0.0.1", 40001))
    assert br.parse(wire["ping"]) == ("ping", None)
    assert br.parse(wire["dead_report"][0]) == ("dead", ("127.0.0.1", 40001))
    for per_peer in wire["gossip_lines"].values():
        for count, line in per_peer.items():
            kind, (ts, ip, n) = br.parse(line)
            assert kind == "gossip" and ts == wire["fixed_now"] and ip == "127.0.0.1" and n == int(count)
            assert pkg.peer.gossip_message(ts, ip, n) == line
    assert br.parse("('127.0.0.1', 40007)\n") == ("hello", ("127.0.0.1", 40007))
    assert br.parse("I am seed|('10.0.0.2', 5000)") == ("seed_hello", ("10.0.0.2", 5000))
    for bad in ("__import__('os')", "Dead Node: [1, 2]", "hello", "2025-02-22 12:00:00:x:y"):
        assert br.parse(bad)[0] == "unknown"


def test_seed_side_registration_matches_the_reference(pkg):
    gold = _golden("c1_overlay.json")
    b, replies = _bridge(pkg)
    subsets = [pkg.bridge.parse_subset(r[0]) for r in replies]
    assert [[list(x) for x in s] for s in subsets] == gold["subsets"]
    g = b.overlay()
    ref = pkg.overlay.first3_overlay(10)
    assert np.array_equal(g.row_ptr, ref.row_ptr) and np.array_equal(g.col, ref.col)
    out = [sorted(int(j) for j in np.nonzero([k in g.in_neighbors(j).tolist() for j in range(10)])[0])
           for k in range(10)]
    assert out == gold["outgoing"]
    assert b.handle("('127.0.0.1', 40001)\n") == []          # duplicate handshake
    me = b.handle("I am seed|('127.0.0.1', 7000)\n")
    assert me[0].startswith("I am seed|") and me[1].startswith("Heartbeat from ")


@pytest.mark.gpu
@pytest.mark.parametrize("crashes", [(), ((4, 1), (0, 6), (9, 3))])
def test_c1_through_the_bridge(pkg, oracle, harness, crashes):
    """The multiset of (receiver, gossip line, round) the bridge delivers equals
    the first receipts of the harness's per-peer Message-Lists rendered the
    same way; dead-node reports and the seed's removals match the C oracle.
    (All C1 peers share 127.0.0.1, so a line does not name its origin's port:
    the reference's own collision, SURVEY.md §0 finding 5 -- hence multisets.)"""
    b, _ = _bridge(pkg)
    b.start()
    by_round = {}
    for v, r in crashes:
        by_round.setdefault(r, []).append(v)
    got, reports, seed_log = [], [], []
    for r in range(254):
        for v in by_round.get(r, []):
            b.crash(b.peers[v])
        out = b.step()
        assert out["round"] == r
        for to, line in out["deliveries"]:
            assert pkg.bridge.parse(line)[0] == "gossip"
            got.append((b.vertex[to], line, r + 1))
        for rp, line in out["reports"]:
            kind, dead = pkg.bridge.parse(line)
            assert kind == "dead"
            reports.append((b.vertex[dead], b.vertex[rp], r))
        seed_log += out["seed_log"]
        if out["stats"]["new_bits"] == 0 and r >= int(b.inject.max()):
            break
    g = pkg.overlay.first3_overlay(10)
    in_lists = [g.in_neighbors(v).tolist() for v in range(g.n)]
    h = harness.run(g.n, in_lists, True, b.origin.tolist(), b.inject.tolist(), crashes=crashes)
    want = []
    for k, m in np.argwhere(h["first"] != 255).tolist():
        rr = int(h["first"][k, m])
        if k != int(b.origin[m]):     # a receipt, not the origin's own generation
            want.append((k, b.gossip_line(m), rr))
    assert sorted(got) == sorted(want)
    assert len(got) > 0
    ref = oracle.run(g, b.origin, b.inject, crashes=crashes)
    assert sorted(reports) == sorted(map(tuple, ref["reports"].tolist()))
    removals = sum(s["removals"] for s in ref["stats"])
    assert sum("Completely removed dead node" in x for x in seed_log) == 2 * removals   # Seed.py:393-406 runs twice
    if crashes:
        assert removals >= 2
    b.close()
