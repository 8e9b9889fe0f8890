"""One line per emulated shard run (scripts/gpu_shard_emu.sh): the step time,
rounds, edge-deliveries and each round's mode:kernel ms of the last step."""
import json
import sys

tag, js, err = sys.argv[1:4]
d = json.load(open(js))
rounds = [json.loads(x) for x in open(err) if x.startswith('{"round"')]
per = " ".join(f"{r['mode']}:{r['kernel_ms']:.2f}" for r in rounds)
print(f"{tag:<22s} {d['ms_per_step']:8.2f} ms  rounds {d['config']['rounds_per_step']:.0f}  "
      f"sends {d['config']['edge_deliveries_per_step']} | {per}")
