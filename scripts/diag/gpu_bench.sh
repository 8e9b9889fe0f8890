set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
nproc > gpurun_out/host.txt; lscpu | grep "Model name" >> gpurun_out/host.txt
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --profile-steps > gpurun_out/bench.json 2> gpurun_out/bench.err
echo "bench exit $?"
cat gpurun_out/bench.json; tail -20 gpurun_out/bench.err
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_bench.json 2> gpurun_out/prof.err
echo "prof exit $?"
find gpurun_out/prof -name "*stats*" | head
