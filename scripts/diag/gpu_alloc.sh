# bimodal per-process C4 times: default allocator vs GP_ALLOC=contig, alternating processes
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/alloc
for k in 1 2 3 4; do
for mode in default contig; do
  GP_ALLOC=$mode timeout -k 10 120 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --profile-steps > gpurun_out/alloc/$mode.$k.json 2> gpurun_out/alloc/$mode.$k.err || exit 1
  python3 - "$mode" "$k" <<'PY'
import json, sys
m, k = sys.argv[1:]
d = json.loads(open(f"gpurun_out/alloc/{m}.{k}.json").read())
rs = [json.loads(l) for l in open(f"gpurun_out/alloc/{m}.{k}.err") if l.startswith("{")]
print(f"{m:8s}", round(d["ms_per_step"], 2), "ms |", " ".join(f"r{r['round']}:{r['kernel_ms'] or r['expand_ms']:.2f}" for r in rs), flush=True)
PY
done
done
