# 2048-message shard (W = 32): flat kernel in round 2, narrow push at W = 32; plus per-GPU shard times
set -o pipefail
cd $GRAFT_REPO_ROOT
A=gossip-protocol-with-power-law_amd/_ab
LIBS="$A/base.so $A/flat32.so $A/np32.so $A/both.so" EXTRA="--messages 2048" ROUNDS=2 timeout -k 10 400 bash scripts/gpu_ab_libs.sh || exit 1
