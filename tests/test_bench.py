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
