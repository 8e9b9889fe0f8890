"""CPU oracle of the gossip hot path -- TEST INFRASTRUCTURE ONLY.

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg, as the checker (never as the product path):
  lib.py         ctypes binding of gossip_oracle.c (Chung-Lu builder + rounds)
  harness.py     per-peer Message-List harness (sha256 dedup, forward-once)
  graph_ref.py   numpy restatement of the Chung-Lu alias/relabel builder
  powerlaw_ref.py literal restatement of NetworkBuilder.powerlaw_subset joins
Parity pins: tests/golden/* (generated from the reference by
tests/golden/make_golden.py).  Multi-hop propagation is not present in the
reference: that part is pinned only by the round-1 direct
delivery matrix of C1 and is otherwise the build's own spec.
"""
