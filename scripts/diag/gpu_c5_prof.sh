# C5 evidence: rocprofv3 kernel-trace stats of the churn bench (2^26 nodes)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/c5p
mkdir -p $O
timeout -k 10 500 python -u bench.py --workload c5 --profile-steps > $O/bench.json 2> $O/bench.err || exit 1
cat $O/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --workload c5 --no-cpu-baseline --steps 2 > $O/trace.json 2> $O/trace.err || exit 1
python3 scripts/prof_summary.py $(find $O/trace -name "*kernel_stats.csv" | head -1) "rocprofv3 --kernel-trace --stats -- python3 bench.py --workload c5 --no-cpu-baseline --steps 2" > $O/kernel_stats.md && head -14 $O/kernel_stats.md
