# round 3: line-mask probe variants (0 nibble, 1 activity bit then nibble, 2 two-bit prefix codes),
# same-box A/B on C4 and C5; then the whole GPU suite and the C4 bench line at HEAD
set -o pipefail
cd $GRAFT_REPO_ROOT
A=gossip-protocol-with-power-law_amd/_ab
echo "== C4"
LIBS="$A/lmp0.so $A/lmp1.so $A/lmp2.so" ROUNDS=2 timeout -k 10 400 bash scripts/gpu_ab_libs.sh || exit 1
echo "== C5"
LIBS="$A/lmp0.so $A/lmp1.so $A/lmp2.so" WORKLOAD=c5 STEPS=3 ROUNDS=1 timeout -k 10 500 bash scripts/gpu_ab_libs.sh || exit 1
bash scripts/gpu_all.sh
