# A/B of library variants on message-shard ranks run alone (bench.py --emulate-shard),
# alternating on one box: LIBS="a.so b.so" RANKS="1/2 0/2" ROUNDS=2
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/abe
for k in $(seq 1 ${ROUNDS:-2}); do
for s in ${RANKS:-1/2}; do
for lib in $LIBS; do
  tag=$(basename $lib .so)_$(echo $s | tr / _)
  GOSSIP_HIP_LIB=$lib timeout -k 10 200 python -u bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline --profile-steps --emulate-shard $s --shard-assign blocked > gpurun_out/abe/$tag.$k.json 2> gpurun_out/abe/$tag.$k.err || exit 1
  python3 scripts/emu_line.py $tag gpurun_out/abe/$tag.$k.json gpurun_out/abe/$tag.$k.err || exit 1
done
done
done
