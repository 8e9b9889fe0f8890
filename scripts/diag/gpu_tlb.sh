# slow / fast C4 processes: UTCL1 translation misses of the pull kernels, 6 processes in a row
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/tlb
mkdir -p $O
A="--steps 1 --warmup 0 --no-cpu-baseline --profile-steps"
for k in 1 2 3 4 5 6; do
  timeout -s KILL 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum --output-format csv -d $O/t$k -o t -- python3 bench.py $A > $O/t$k.json 2> $O/t$k.err || exit 1
  python3 - $k <<'PY'
import csv, glob, json, sys, collections
k = sys.argv[1]
path = glob.glob(f"gpurun_out/tlb/t{k}/**/*counter_collection.csv", recursive=True)[0]
per = collections.defaultdict(dict); names = {}
for r in csv.DictReader(open(path)):
    d = int(r["Dispatch_Id"]); names[d] = r["Kernel_Name"].split("(")[0][-18:]
    per[d][r["Counter_Name"]] = per[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
rs = [json.loads(l) for l in open(f"gpurun_out/tlb/t{k}.err") if l.startswith("{")]
pulls = [r for r in rs if r["mode"] == 0 and r["kernel_ms"] > 0]
ex = [d for d in sorted(per) if "k_expand" in names[d]]
print(k, " | ".join(f"r{r['round']} {r['kernel_ms']:.2f}ms miss {per[d].get('TCP_UTCL1_TRANSLATION_MISS_sum',0)/1e6:.1f}M hit {per[d].get('TCP_UTCL1_TRANSLATION_HIT_sum',0)/1e6:.0f}M" for r, d in zip(pulls, ex)), flush=True)
PY
done
