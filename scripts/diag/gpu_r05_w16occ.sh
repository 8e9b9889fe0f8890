# round 5: W = 16 flat kernel (the N = 4 shards) -- 32 receivers per wave (LDS 5.1 KB) and 5 / 6 waves per
# SIMD forced (96 / 80 VGPRs, with spills) against HEAD (64 receivers, 9.2 KB, 4 waves); N = 4 ranks 3 and 0
set -o pipefail
cd $GRAFT_REPO_ROOT
L=gossip-protocol-with-power-law_amd/_ab
GOSSIP_HIP_LIB=$L/nr32w5.so timeout -k 10 600 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu -k "width or shard" > gpurun_out/pytest_w16.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_w16.log; [ $rc -eq 0 ] || exit $rc
LIBS="$L/base.so $L/nr32.so $L/nr32w5.so $L/nr32w6.so" ROUNDS=2 STEPS=6 EXTRA="--emulate-shard 3/4" bash scripts/gpu_ab_libs.sh || exit 1
LIBS="$L/base.so $L/nr32.so $L/nr32w5.so $L/nr32w6.so" ROUNDS=1 STEPS=6 EXTRA="--emulate-shard 0/4" bash scripts/gpu_ab_libs.sh
