# round 3: round-2 line-mask pull with short in-lists two receivers at a time (GP_LINES_PAIRS) -- same-box A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
A=gossip-protocol-with-power-law_amd/_ab
echo "== C4"
LIBS="$A/lbase.so $A/lpairs.so" ROUNDS=2 timeout -k 10 300 bash scripts/gpu_ab_libs.sh || exit 1
echo "== C5"
LIBS="$A/lbase.so $A/lpairs.so" WORKLOAD=c5 STEPS=3 ROUNDS=2 timeout -k 10 500 bash scripts/gpu_ab_libs.sh || exit 1
