# round 5: the LDS trim at W = 16 / 32 (N = 4 / 2 message shards; 10,688 -> 9,200 B
# per one-wave block) and the wide rows in flight (6 at HEAD; 4, 8), same box
set -o pipefail
cd $GRAFT_REPO_ROOT
L=gossip-protocol-with-power-law_amd/_ab
for sh in 3/4 0/4 1/2; do
  LIBS="$L/base.so $L/head.so $L/wide4.so $L/wide8.so" ROUNDS=2 STEPS=6 EXTRA="--emulate-shard $sh" bash scripts/gpu_ab_libs.sh || exit 1
done
