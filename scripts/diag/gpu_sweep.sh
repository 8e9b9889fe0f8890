# parameter sweep of the C4 bench (no CPU baseline): PARAM=<bench flag> LIST="<values>"
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sweep
PARAM=${PARAM:---push-ratio}
for val in ${LIST:-40 16}; do
  tag=$(echo "$PARAM$val" | tr -c 'a-zA-Z0-9.' '_')
  timeout -k 10 120 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline $PARAM $val --profile-steps $EXTRA > gpurun_out/sweep/$tag.json 2> gpurun_out/sweep/$tag.err || exit 1
  python - "$tag" "$PARAM" "$val" <<'PY'
import json, sys
tag, p, v = sys.argv[1:]
d = json.loads(open(f"gpurun_out/sweep/{tag}.json").read())
rs = [json.loads(l) for l in open(f"gpurun_out/sweep/{tag}.err") if l.startswith("{")]
print(p, v, round(d["value"]), "GTEPS", round(d["ms_per_step"], 2), "ms |",
      " ".join(f"r{r['round']}:{'P' if r['mode'] else 'L'}{r.get('scan', 0)}:{r['expand_ms']:.2f}/{r['kernel_ms']:.2f}/{r.get('row_bytes', 0)/1e9:.1f}G" for r in rs))
PY
done
