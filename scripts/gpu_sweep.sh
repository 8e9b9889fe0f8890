# parameter sweep of the C4 bench (no CPU baseline); one JSON line per setting
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sweep
for hd in ${HOT_LIST:-0 32 64 128 256}; do
  timeout -k 10 120 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --hot-degree $hd --profile-steps $EXTRA > gpurun_out/sweep/hot_$hd.json 2> gpurun_out/sweep/hot_$hd.err || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/sweep/hot_$hd.json').read()); print('hot', $hd, round(d['value']), 'GTEPS', round(d['ms_per_step'],2), 'ms')"
done
