# round-3 final evidence at HEAD: the whole GPU suite, then the C4 bench line with rocprofv3 kernel stats
# and the two PMC passes, then the same for C5
set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu_all.sh || exit 1
bash scripts/gpu_round_profile.sh || exit 1
bash scripts/gpu_c5_profile.sh || exit 1
