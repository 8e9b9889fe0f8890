# round 5: done in-neighbours probed over the first 2 / 4 / 8 gather-order arcs, C4 then C5, same box
set -o pipefail
cd $GRAFT_REPO_ROOT
L=gossip-protocol-with-power-law_amd/_ab
LIBS="$L/base.so $L/dnb4.so $L/dnb8.so" ROUNDS=2 STEPS=10 bash scripts/gpu_ab_libs.sh || exit 1
LIBS="$L/base.so $L/dnb4.so $L/dnb8.so" ROUNDS=2 STEPS=3 WORKLOAD=c5 bash scripts/gpu_ab_libs.sh
