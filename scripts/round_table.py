#!/usr/bin/env python3
"""One line per bench run: ms/step and per-round kernel ms / row GB.  usage: round_table.py tag json err"""
import json
import sys

tag, jf, ef = sys.argv[1:4]
d = json.load(open(jf))
rs = [json.loads(l) for l in open(ef) if l.startswith("{")]
print(f"{tag:10s}", round(d["ms_per_step"], 2), "ms |",
      " ".join(f"r{r['round']}:{'P' if r['mode'] else 'L'}{r['kernel_ms'] or r['expand_ms']:.2f}/{r['row_bytes'] / 1e9:.1f}"
               for r in rs), flush=True)
