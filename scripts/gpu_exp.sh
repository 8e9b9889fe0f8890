set -o pipefail
cd $GRAFT_REPO_ROOT
EXTRA="--sparse-rows 0" PARAM=--hot-degree LIST="0 1000000000 64" bash scripts/gpu_sweep.sh || exit 1
EXTRA="--sparse-rows 0 --hot-degree 1000000000" PASSES="TCC_EA0_RDREQ_sum,TCC_HIT_sum,TCC_MISS_sum" bash scripts/gpu_pmc_passes.sh
