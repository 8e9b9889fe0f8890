# rocprofv3 kernel-trace summary of the C4 bench (copy the summary into profiles/)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --profile-steps > gpurun_out/prof/bench.json 2> gpurun_out/prof/bench.err
rc=$?; echo "prof exit $rc"; cat gpurun_out/prof/bench.json
find gpurun_out/prof -name "*stats*"
exit $rc
