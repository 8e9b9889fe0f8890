set -o pipefail
cd $GRAFT_REPO_ROOT
EXTRA="--sparse-rows 0" PARAM=--push-ratio LIST="40 16 12 8" bash scripts/gpu_sweep.sh || exit 1
EXTRA="--sparse-rows 1" PARAM=--push-ratio LIST="16" bash scripts/gpu_sweep.sh || exit 1
grep -h '"round": 1,' gpurun_out/sweep/*.err
