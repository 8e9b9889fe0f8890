#!/bin/bash
# A/B of bench.py knob sets on one box, alternating: VARIANTS="tag1:args1|tag2:args2" ROUNDS=2 WORKLOAD=c5
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
IFS='|' read -ra VS <<< "$VARIANTS"
for k in $(seq 1 ${ROUNDS:-2}); do
for v in "${VS[@]}"; do
  tag=${v%%:*}; args=${v#*:}
  timeout -k 10 200 python -u bench.py --workload ${WORKLOAD:-c4} --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline --profile-steps $args > gpurun_out/ab/$tag.$k.json 2> gpurun_out/ab/$tag.$k.err || exit 1
  python3 - "$tag" "$k" <<'PY'
import json, sys
tag, k = sys.argv[1:]
d = json.loads(open(f"gpurun_out/ab/{tag}.{k}.json").read())
rs = [json.loads(l) for l in open(f"gpurun_out/ab/{tag}.{k}.err") if l.startswith("{")]
print(f"{tag:12s}", round(d["ms_per_step"], 2), "ms", round(d["roofline"]["frac"], 3), "|",
      " ".join(f"r{r['round']}:{'P' if r['mode'] else 'L'}{r['scan']}:{r['kernel_ms'] or r['expand_ms']:.2f}" for r in rs), flush=True)
PY
done
done
