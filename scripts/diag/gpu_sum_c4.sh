# summary-probe variant on C4: codegen cost (sum: off below 2^25) and the
# 2^24 threshold (sum24), same box, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sum4
B=gossip-protocol-with-power-law_amd/_build
for k in 1 2; do
for lib in libgossip_hip.so libgossip_hip_sum.so libgossip_hip_sum24.so; do
  GOSSIP_HIP_LIB=$B/$lib timeout -k 10 120 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --profile-steps > gpurun_out/sum4/$lib.$k.json 2> gpurun_out/sum4/$lib.$k.err || exit 1
  python3 - "$lib" $k <<'PY'
import json, sys
lib, k = sys.argv[1:]
d = json.loads(open(f"gpurun_out/sum4/{lib}.{k}.json").read())
rs = [json.loads(l) for l in open(f"gpurun_out/sum4/{lib}.{k}.err") if l.startswith("{")]
print(lib, round(d["value"]), "GTEPS", round(d["ms_per_step"], 2), "ms |",
      " ".join(f"r{r['round']}:{'P' if r['mode'] else 'L'}{r['scan']}:{r['expand_ms']:.2f}" for r in rs))
PY
done
done
