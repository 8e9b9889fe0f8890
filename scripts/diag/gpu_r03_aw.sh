# round 3: alive early-exit variant asked for 8 waves per SIMD (64 VGPRs + 36 B/lane scratch) vs 7 (69 VGPRs), C5 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
A=gossip-protocol-with-power-law_amd/_ab
LIBS="$A/aw0.so $A/aw8.so" WORKLOAD=c5 STEPS=3 ROUNDS=2 timeout -k 10 500 bash scripts/gpu_ab_libs.sh || exit 1
