# Round evidence for profiles/: bench line, rocprofv3 kernel-trace stats of the
# same command, and the two PMC traffic passes (separate runs).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/rp
mkdir -p $O/pmc
timeout -k 10 400 python -u bench.py --profile-steps > $O/bench.json 2> $O/bench.err || exit 1
echo "bench ok"; cat $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --no-cpu-baseline --profile-steps > $O/trace.json 2> $O/trace.err || exit 1
echo "trace ok"
ARGS="--steps 1 --warmup 0 --no-cpu-baseline --profile-steps"
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc/fetch -o fetch -- python3 bench.py $ARGS > $O/pmc/fetch.json 2> $O/pmc/fetch.err || exit 1
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc/write -o write -- python3 bench.py $ARGS > $O/pmc/write.json 2> $O/pmc/write.err || exit 1
echo "pmc ok"
python3 scripts/pmc_summary.py $O/pmc $O/pmc_traffic.json > $O/pmc_traffic.md && cat $O/pmc_traffic.md
python3 scripts/prof_summary.py $(find $O/trace -name "*kernel_stats.csv" | head -1) "rocprofv3 --kernel-trace --stats -- python3 bench.py --no-cpu-baseline" > $O/kernel_stats.md && head -12 $O/kernel_stats.md
