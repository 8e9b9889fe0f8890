# round-3 evidence: churn parity subset, then C4 and C5 bench lines with
# rocprofv3 kernel-trace stats and the two PMC passes each
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -m gpu -k "churn or sated or wide or lost or checkpoint or detection or group" > gpurun_out/pytest_churn.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_churn.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_round_profile.sh || exit 1
bash scripts/gpu_c5_profile.sh || exit 1
