# round 3: complete lines (seen rows' complete 128-B lines not read) -- same-box A/B against the same
# source built without them (nocl); C5: the alive early-exit variant asked for 8 waves (nocl_aw8)
set -o pipefail
cd $GRAFT_REPO_ROOT
A=gossip-protocol-with-power-law_amd/_ab
echo "== C4"
LIBS="$A/nocl.so $A/cl.so" ROUNDS=2 timeout -k 10 300 bash scripts/gpu_ab_libs.sh || exit 1
echo "== C5"
LIBS="$A/nocl.so $A/nocl_aw8.so $A/cl.so" WORKLOAD=c5 STEPS=3 ROUNDS=2 timeout -k 10 600 bash scripts/gpu_ab_libs.sh || exit 1
