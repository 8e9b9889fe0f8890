# round-3 evidence at HEAD: C4 bench line + rocprofv3 kernel trace + PMC passes, then the same for C5
set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu_round_profile.sh || exit 1
bash scripts/gpu_c5_profile.sh || exit 1
