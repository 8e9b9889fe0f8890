set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -40 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --profile-steps > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench exit $rc"; cat gpurun_out/bench.json; tail -20 gpurun_out/bench.err
exit $rc
