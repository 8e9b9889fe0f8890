set -o pipefail
cd $GRAFT_REPO_ROOT
PARAM=--sparse-rows LIST="1 0" bash scripts/gpu_sweep.sh || exit 1
grep -h '"round": 2' gpurun_out/sweep/*.err
bash scripts/gpu_prof.sh
