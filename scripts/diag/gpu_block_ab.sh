# A/B of the pull kernels' block size (GP_EXPAND_BLOCK 256 / 128 / 64 = default), C4, C5 and the slowest emulated shard ranks
set -o pipefail
cd $GRAFT_REPO_ROOT
L="gossip-protocol-with-power-law_amd/_ab/eb256.so gossip-protocol-with-power-law_amd/_ab/eb128.so gossip-protocol-with-power-law_amd/_build/libgossip_hip.so"
LIBS="$L" ROUNDS=2 bash scripts/gpu_ab_libs.sh && LIBS="$L" WORKLOAD=c5 STEPS=2 ROUNDS=2 bash scripts/gpu_ab_libs.sh || exit 1
for S in 7/8 3/4 1/2; do EXTRA="--emulate-shard $S" LIBS="$L" ROUNDS=1 bash scripts/gpu_ab_libs.sh || exit 1; done
