# round 5: flat-kernel rows in flight for W <= 8 (GP_FLAT_RIF_NARROW 3 / 4 / 5)
# on the N = 8 job's ranks 7 and 0, same box, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
L=gossip-protocol-with-power-law_amd/_ab
LIBS="$L/base.so $L/frif4.so $L/frif5.so" ROUNDS=2 STEPS=10 EXTRA="--emulate-shard 7/8" bash scripts/gpu_ab_libs.sh || exit 1
LIBS="$L/base.so $L/frif4.so $L/frif5.so" ROUNDS=2 STEPS=10 EXTRA="--emulate-shard 0/8" bash scripts/gpu_ab_libs.sh
