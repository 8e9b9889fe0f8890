# Per-GPU work of the N-GPU message-shard runs, every rank of the job run alone
# on this box (bench.py --emulate-shard R/N), both shard assignments; the whole
# C4 run alternates with them.  The projected N-GPU time is the max over ranks.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/emu
one() {   # tag, args...
  local tag=$1; shift
  timeout -k 10 120 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --profile-steps "$@" > gpurun_out/emu/$tag.json 2> gpurun_out/emu/$tag.err || exit 1
  python3 scripts/emu_line.py $tag gpurun_out/emu/$tag.json gpurun_out/emu/$tag.err
}
one c4
for N in ${NS:-2 4 8}; do
  for A in ${ASSIGN:-interleaved blocked wordsnake}; do
    for R in $(seq 0 $((N - 1))); do one n${N}_${A:0:5}_r$R --emulate-shard $R/$N --shard-assign $A; done
  done
done
one c4_again
