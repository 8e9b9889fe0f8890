# round 3: per-GPU work of the message shards at N = 2 / 4 / 8 against the whole C4 run, same box, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
VARIANTS="c4:|m2048:--messages 2048|m1024:--messages 1024|m512:--messages 512" ROUNDS=2 timeout -k 10 500 bash scripts/gpu_ab_args.sh || exit 1
