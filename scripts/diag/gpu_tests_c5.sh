# selected GPU tests, then the C5 bench line (per-round stats to stderr) and its kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
if [ -n "$1" ]; then
  timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu $1 ${2:+-k "$2"} > gpurun_out/pytest_sel.log 2>&1
  rc=$?; echo "pytest exit $rc"; tail -4 gpurun_out/pytest_sel.log
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python -u bench.py --workload c5 --steps 5 --warmup 2 --profile-steps --no-cpu-baseline > gpurun_out/c5_bench.json 2> gpurun_out/c5_bench.err
rc=$?; echo "c5 bench exit $rc"; cat gpurun_out/c5_bench.json | cut -c1-700; tail -3 gpurun_out/c5_bench.err | cut -c1-300
[ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c5prof -o run -- python3 bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/c5_prof_bench.json 2> gpurun_out/c5_prof.err
rc=$?; echo "prof exit $rc"
exit $rc
