set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ep
for s in 1/2 7/8; do
  t=$(echo $s | tr / _)
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ep/$t -o run -- python3 bench.py --emulate-shard $s --shard-assign blocked --steps 3 --warmup 1 --no-cpu-baseline --profile-steps > gpurun_out/ep/$t.json 2> gpurun_out/ep/$t.err || exit 1
  echo "$s ok"
done
