# round 5: HBM traffic of the N = 8 job's shards 7 and 0 run alone (W = 8 rows:
# each 64-B row a 128-B line?) -- the two PMC passes per shard, summed per pull
# launch by scripts/pmc_summary.py against the algorithmic bytes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for S in 7 0; do
  O=gpurun_out/spmc$S
  mkdir -p $O
  ARGS="--steps 1 --warmup 0 --no-cpu-baseline --profile-steps --emulate-shard $S/8"
  timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o fetch -- python3 bench.py $ARGS > $O/fetch.json 2> $O/fetch.err || exit 1
  timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o write -- python3 bench.py $ARGS > $O/write.json 2> $O/write.err || exit 1
  python3 scripts/pmc_summary.py $O > $O/pmc_traffic.md && cat $O/pmc_traffic.md
done
