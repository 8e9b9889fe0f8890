# whole GPU suite (incl. full-size C4/C5 parity), then the C4 bench line and a rocprofv3 kernel-trace of it
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
nproc > gpurun_out/host.txt; lscpu | grep "Model name" >> gpurun_out/host.txt
GP_ORACLE_PROGRESS=1 timeout -k 10 1000 python -u -m pytest tests -x -v -s --timeout 1200 --timeout-method thread -m gpu --durations=15 > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -25 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "c4 bench exit $rc"; cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err
exit $rc
