# round 3: 3 rows in flight per lane in k_expand (GP_ROWS_IN_FLIGHT 3 vs 4) on C5 and the 2048-message
# shard, and the alive early-exit variant at 8 waves with it (rif3aw8: 64 VGPRs, 8 B/lane scratch)
set -o pipefail
cd $GRAFT_REPO_ROOT
A=gossip-protocol-with-power-law_amd/_ab
echo "== C5"
LIBS="$A/base.so $A/rif3.so $A/rif3aw8.so" WORKLOAD=c5 STEPS=3 ROUNDS=2 timeout -k 10 700 bash scripts/gpu_ab_libs.sh || exit 1
echo "== 2048-message shard"
LIBS="$A/base.so $A/rif3.so" EXTRA="--messages 2048" ROUNDS=2 timeout -k 10 300 bash scripts/gpu_ab_libs.sh || exit 1
echo "== C4"
LIBS="$A/base.so $A/rif3.so" ROUNDS=1 timeout -k 10 300 bash scripts/gpu_ab_libs.sh || exit 1
