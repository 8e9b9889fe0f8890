# per-GPU work of the message shards at N = 8 / 4 / 2 (512 / 1024 / 2048 messages) on one MI355X
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for m in ${MSGS:-512 1024 2048}; do
  timeout -k 10 120 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --profile-steps --messages $m $EXTRA > gpurun_out/sh$m.json 2> gpurun_out/sh$m.err || exit 1
  python3 scripts/round_table.py m=$m gpurun_out/sh$m.json gpurun_out/sh$m.err
done
