# round 5: the unfiltered-pull threshold (unfiltered_pct 90 default / 85 / 80) on the N = 2 job's slow
# rank (its round 3 has 88.6 % senders), the N = 4 slow rank and C4, same box, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
VARIANTS="u90:--emulate-shard 1/2|u85:--emulate-shard 1/2 --unfiltered-pct 85|u80:--emulate-shard 1/2 --unfiltered-pct 80" ROUNDS=2 STEPS=5 bash scripts/gpu_ab_args.sh || exit 1
VARIANTS="u90:--emulate-shard 3/4|u80:--emulate-shard 3/4 --unfiltered-pct 80" ROUNDS=2 STEPS=5 bash scripts/gpu_ab_args.sh || exit 1
VARIANTS="u90:|u80:--unfiltered-pct 80" ROUNDS=2 STEPS=5 bash scripts/gpu_ab_args.sh
