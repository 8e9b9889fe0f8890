# C5 evidence for profiles/: bench line + rounds, rocprofv3 kernel-trace stats
# of the same command, then the two PMC traffic passes (gpu_c5_pmc.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/c5p
mkdir -p $O
ARGS="--workload c5 --steps 3 --warmup 1 --no-cpu-baseline --profile-steps"
timeout -k 10 400 python -u bench.py $ARGS > $O/bench.json 2> $O/bench.err || exit 1
echo "bench ok"; cat $O/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py $ARGS > $O/trace.json 2> $O/trace.err || exit 1
python3 scripts/prof_summary.py $(find $O/trace -name "*kernel_stats.csv" | head -1) "rocprofv3 --kernel-trace --stats -- python3 bench.py $ARGS" > $O/kernel_stats.md && head -14 $O/kernel_stats.md
bash scripts/gpu_c5_pmc.sh
