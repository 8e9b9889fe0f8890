# C5 (2^26 nodes, 1%/round churn) bench on one MI355X, plus the C4 line for comparison
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py --workload c5 --steps 3 --warmup 1 --profile-steps > gpurun_out/c5_bench.json 2> gpurun_out/c5_bench.err
rc=$?; echo "c5 bench exit $rc"; cat gpurun_out/c5_bench.json; tail -20 gpurun_out/c5_bench.err
exit $rc
