# round 5: degree-rank probes with the hot ranks dealt across lines
# (GP_PROBE_HOT_LOG2 0 = plain rank order / 16 / 21) against base, C4 then C5
set -o pipefail
cd $GRAFT_REPO_ROOT
L=gossip-protocol-with-power-law_amd/_ab
LIBS="$L/base.so $L/hot0.so $L/hot16.so $L/hot21.so" ROUNDS=2 STEPS=10 bash scripts/gpu_ab_libs.sh || exit 1
LIBS="$L/base.so $L/hot21.so" ROUNDS=2 STEPS=3 WORKLOAD=c5 bash scripts/gpu_ab_libs.sh
