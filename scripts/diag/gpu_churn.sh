# churn parity tests (lost-message target drops) + C5 bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -m gpu -k "churn or lost or crashes" > gpurun_out/pytest_churn.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -25 gpurun_out/pytest_churn.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py --workload c5 --steps 3 --warmup 1 --profile-steps --no-cpu-baseline > gpurun_out/c5_bench.json 2> gpurun_out/c5_bench.err
rc=$?; echo "c5 bench exit $rc"; cat gpurun_out/c5_bench.json; tail -12 gpurun_out/c5_bench.err
exit $rc
