# Round evidence at HEAD (TAG names the round, e.g. TAG=r04): whole GPU suite,
# C4 bench line + rocprofv3 kernel trace + the two PMC passes, the same for C5.
# Outputs under gpurun_out/ (copied to profiles/<TAG>_* afterwards).
set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu_all.sh || exit 1
bash scripts/gpu_round_profile.sh || exit 1
bash scripts/gpu_c5_profile.sh || exit 1
