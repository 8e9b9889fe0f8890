# round-3 same-box A/B: narrow push (shards), sated vertices (C5)
set -o pipefail
cd $GRAFT_REPO_ROOT
A=gossip-protocol-with-power-law_amd/_ab
echo "== 512-message shard"
LIBS="$A/base.so $A/np1.so $A/nolanes.so" EXTRA="--messages 512" ROUNDS=2 timeout -k 10 300 bash scripts/gpu_ab_libs.sh || exit 1
echo "== 1024-message shard"
LIBS="$A/base.so $A/np1.so $A/nolanes.so" EXTRA="--messages 1024" ROUNDS=2 timeout -k 10 300 bash scripts/gpu_ab_libs.sh || exit 1
echo "== C5"
LIBS="$A/base.so $A/nosate.so" WORKLOAD=c5 ROUNDS=3 timeout -k 10 400 bash scripts/gpu_ab_libs.sh || exit 1
echo "== C4"
LIBS="$A/base.so $A/nolanes.so" ROUNDS=2 timeout -k 10 300 bash scripts/gpu_ab_libs.sh || exit 1
