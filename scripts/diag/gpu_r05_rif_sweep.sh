# round 5: rows in flight re-checked at the round's HEAD -- 64-word rows 3 (base) / 4 / 2,
# line-mask gathers 3 (base) / 4 / 2; C4, same box, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
L=gossip-protocol-with-power-law_amd/_ab
LIBS="$L/base.so $L/rif64_4.so $L/rif64_2.so $L/lrif4.so $L/lrif2.so" ROUNDS=2 STEPS=10 bash scripts/gpu_ab_libs.sh
