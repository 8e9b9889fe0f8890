# same C4 bench against library variants (GOSSIP_HIP_LIB)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/var
for lib in ${LIBS:-gossip-protocol-with-power-law_amd/_build/libgossip_hip.so}; do
  tag=$(echo $lib | tr '/' '_')
  GOSSIP_HIP_LIB=$lib timeout -k 10 120 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --profile-steps $EXTRA > gpurun_out/var/$tag.json 2> gpurun_out/var/$tag.err || exit 1
  python - "$tag" "$lib" <<'PY'
import json, sys
tag, lib = sys.argv[1:]
d = json.loads(open(f"gpurun_out/var/{tag}.json").read())
rs = [json.loads(l) for l in open(f"gpurun_out/var/{tag}.err") if l.startswith("{")]
print(lib, round(d["value"]), "GTEPS", round(d["ms_per_step"], 2), "ms |",
      " ".join(f"r{r['round']}:{'P' if r['mode'] else 'L'}{r['expand_ms']:.2f}" for r in rs))
PY
done
