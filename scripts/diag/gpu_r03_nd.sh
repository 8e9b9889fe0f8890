# round 3 HEAD: near-done rows in flight (nd1 / nd3 against 2) and line-mask rows in flight (lr2 against 3), C4 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
A=gossip-protocol-with-power-law_amd/_ab
LIBS="$A/base.so $A/nd1.so $A/nd3.so $A/lr2.so" ROUNDS=2 timeout -k 10 500 bash scripts/gpu_ab_libs.sh || exit 1
