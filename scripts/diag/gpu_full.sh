# full GPU parity suite, then the C4 headline bench and the C5 churn bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { grep -n "FAIL\|Error" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --profile-steps --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "c4 bench exit $rc"; cat gpurun_out/bench.json; tail -10 gpurun_out/bench.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py --workload c5 --steps 3 --warmup 1 --profile-steps --no-cpu-baseline > gpurun_out/c5_bench.json 2> gpurun_out/c5_bench.err
rc=$?; echo "c5 bench exit $rc"; cat gpurun_out/c5_bench.json; tail -11 gpurun_out/c5_bench.err
exit $rc
