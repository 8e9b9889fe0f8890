# C5 HBM traffic of k_expand: the two rocprofv3 PMC passes (separate runs) of
# one churn run at 2^26 nodes, summarised into pmc_traffic_c5.json
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/c5pmc
mkdir -p $O/pmc
ARGS="--workload c5 --steps 1 --warmup 0 --no-cpu-baseline --profile-steps"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc/fetch -o fetch -- python3 bench.py $ARGS > $O/pmc/fetch.json 2> $O/pmc/fetch.err || exit 1
echo "fetch ok"
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc/write -o write -- python3 bench.py $ARGS > $O/pmc/write.json 2> $O/pmc/write.err || exit 1
echo "pmc ok"
python3 scripts/pmc_summary.py $O/pmc $O/pmc_traffic_c5.json > $O/pmc_traffic_c5.md && cat $O/pmc_traffic_c5.md
