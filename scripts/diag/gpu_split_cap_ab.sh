# A/B of the degree-split cap (split_max_permille 10 vs 1000) on every rank of the emulated N = 4 / 8 shard jobs, C4 and C5
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/cap && P=gossip-protocol-with-power-law_amd
for L in $P/_ab/nocap.so $P/_build/libgossip_hip.so; do t=$(basename $L .so)
  for N in 4 8; do for R in $(seq 0 $((N - 1))); do
    GOSSIP_HIP_LIB=$L timeout -k 10 120 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --emulate-shard $R/$N > gpurun_out/cap/$t.$N.$R.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/cap/$t.$N.$R.json')); print('%-14s N=%d r%d %7.2f ms' % ('$t', $N, $R, d['ms_per_step']))"
  done; done
  for W in c4 c5; do GOSSIP_HIP_LIB=$L timeout -k 10 200 python3 bench.py --workload $W --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/cap/$t.$W.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/cap/$t.$W.json')); print('%-14s %s %7.2f ms' % ('$t', '$W', d['ms_per_step']))"; done
done
