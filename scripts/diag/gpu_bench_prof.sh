# selected GPU tests, the C4 bench line (with the CPU baseline legs) and a rocprofv3 kernel trace of it
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
nproc > gpurun_out/host.txt; lscpu | grep "Model name" >> gpurun_out/host.txt
if [ -n "$1" ]; then
  timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu $1 ${2:+-k "$2"} > gpurun_out/pytest_sel.log 2>&1
  rc=$?; echo "pytest exit $rc"; tail -5 gpurun_out/pytest_sel.log
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --profile-steps > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "c4 bench exit $rc"; cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err
[ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_bench.json 2> gpurun_out/prof.err
rc=$?; echo "prof exit $rc"; cat gpurun_out/prof_bench.json
find gpurun_out/prof -name "*stats*"
exit $rc
