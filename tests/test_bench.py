"""bench.py host logic (no GPU): the committed PMC traffic measurements are
picked by workload, and never for a run of another shape."""
import glob
import json
import os

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_pmc_traffic_matches_its_own_workload():
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_traffic*.json")))
    assert files, "no PMC traffic measurement committed under profiles/"
    for path in files:
        d = json.load(open(path))
        traffic, src = bench.pmc_traffic(d["config"])
        assert src == os.path.relpath(path, ROOT)
        assert traffic == d["traffic_bytes_per_launch"]
        assert d["traffic_bytes_per_launch"] >= 0.5 * d["alg_bytes_per_launch"]


def test_pmc_traffic_none_for_other_shape():
    d = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))
    cfg = dict(d["config"], messages=d["config"]["messages"] // 2)
    assert bench.pmc_traffic(cfg) == (None, None)


def test_pmc_traffic_none_for_other_message_order():
    """A measurement taken with one message order is not used for a run of the other."""
    d = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))
    cfg = dict(d["config"], message_order="given")
    assert d["config"]["message_order"] != "given"
    assert bench.pmc_traffic(cfg) == (None, None)


def test_round_bytes_terms():
    """Algorithmic bytes of a pull launch: per-vertex state,
    arcs by scan mode, row bytes, seen rows, written rows with their committed
    words, and the senders' rows k_mklm reads."""
    n, W = 1000, 64
    base = dict(arcs_scanned=0, row_bytes=0, seen_rows_read=0, rows_written=0, scan=0)
    assert bench.round_bytes(base, W, n) == 30 * n
    assert bench.round_bytes(dict(base, arcs_scanned=10), W, n) == 30 * n + 120
    assert bench.round_bytes(dict(base, arcs_scanned=10, scan=2), W, n) == 30 * n + 40
    assert bench.round_bytes(dict(base, row_bytes=777), W, n) == 30 * n + 777
    assert bench.round_bytes(dict(base, seen_rows_read=3), W, n) == 30 * n + 3 * 512
    assert bench.round_bytes(dict(base, rows_written=2), W, n) == 30 * n + 2 * (512 + 23)
    assert bench.round_bytes(dict(base, lm_rows=5), W, n) == 30 * n + 5 * 512
