#!/usr/bin/env python3
"""Cold-start breakdown: device Chung-Lu build, degree check, set_messages
(first: allocates the run state), reset, first run, finalize.  usage: setup_timing.py log2n"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _gossip_pkg  # noqa: E402


def main():
    log2n = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    pkg = _gossip_pkg.load()
    n = 1 << log2n
    out = {}
    t = time.perf_counter()
    eng = pkg.GossipEngine(0, track_digest=1)
    eng.synchronize()
    out["create"] = time.perf_counter() - t
    t = time.perf_counter()
    eng.build_chung_lu(n, 16.0, 2.5, 4)
    eng.synchronize()
    out["build"] = time.perf_counter() - t
    t = time.perf_counter()
    origin = pkg.overlay.random_origins(n, 4096, seed=4)
    out["origins"] = time.perf_counter() - t
    t = time.perf_counter()
    eng.set_messages(origin)
    eng.synchronize()
    out["set_messages"] = time.perf_counter() - t
    t = time.perf_counter()
    eng.reset()
    eng.synchronize()
    out["reset1"] = time.perf_counter() - t
    t = time.perf_counter()
    eng.run()
    eng.synchronize()
    out["run1"] = time.perf_counter() - t
    t = time.perf_counter()
    eng.finalize()
    out["finalize1"] = time.perf_counter() - t
    t = time.perf_counter()
    eng.reset()
    eng.run()
    eng.finalize()
    eng.synchronize()
    out["step2"] = time.perf_counter() - t
    eng.close()
    print({k: round(v, 4) for k, v in out.items()}, flush=True)


if __name__ == "__main__":
    main()
