# per-round kernel times of every rank of the emulated N-GPU message-shard jobs (NS="2 4 8"), bench.py --emulate-shard
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sr
for N in ${NS:-2 4 8}; do for R in $(seq 0 $((N - 1))); do
  timeout -k 10 120 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --profile-steps --emulate-shard $R/$N $EXTRA > gpurun_out/sr/n$N.r$R.json 2> gpurun_out/sr/n$N.r$R.err || exit 1
  python3 scripts/round_table.py n$N.r$R gpurun_out/sr/n$N.r$R.json gpurun_out/sr/n$N.r$R.err
done; done
