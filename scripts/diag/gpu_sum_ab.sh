# summary-probe variant: parity suite with the summary level forced on in every
# filtered round, then C5 A/B (default library vs summary probes), same box
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sum
B=gossip-protocol-with-power-law_amd/_build
GOSSIP_HIP_LIB=$B/libgossip_hip_sumall.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/sum/pytest.log 2>&1
rc=$?; echo "pytest sumall exit $rc"; tail -3 gpurun_out/sum/pytest.log; [ $rc -eq 0 ] || exit $rc
for k in 1 2; do
for lib in libgossip_hip.so libgossip_hip_sum.so; do
  GOSSIP_HIP_LIB=$B/$lib timeout -k 10 200 python -u bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline --profile-steps > gpurun_out/sum/$lib.$k.json 2> gpurun_out/sum/$lib.$k.err || exit 1
  python3 - "$lib" $k <<'PY'
import json, sys
lib, k = sys.argv[1:]
d = json.loads(open(f"gpurun_out/sum/{lib}.{k}.json").read())
rs = [json.loads(l) for l in open(f"gpurun_out/sum/{lib}.{k}.err") if l.startswith("{")]
print(lib, round(d["value"]), "GTEPS", round(d["ms_per_step"], 2), "ms |",
      " ".join(f"r{r['round']}:{'P' if r['mode'] else 'L'}{r['scan']}:{r['expand_ms']:.2f}" for r in rs))
PY
done
done
