# round 5 check: a forwards diagnostic, the whole GPU suite, the C4 bench line,
# and the blocked message shards under the round-4 library (base) and HEAD (r05a)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05a
timeout -k 10 200 python3 -u scripts/diag/fwd_check.py 200 || exit 1
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/r05a/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/r05a/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r05a/bench.json 2> gpurun_out/r05a/bench.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/r05a/bench.json')); print('C4', round(d['ms_per_step'],2), 'ms frac', round(d['roofline']['frac'],3))"
LIBS="gossip-protocol-with-power-law_amd/_ab/base.so gossip-protocol-with-power-law_amd/_ab/r05a.so" bash scripts/diag/gpu_shard_libs.sh
