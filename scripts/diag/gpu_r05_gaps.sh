# round 5: where a step's time goes outside the pull kernels -- kernel traces
# of the whole C4 step and of the N = 8 message shards 0 and 7 run alone
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/gaps
mkdir -p $O
for t in c4 s0 s7; do
  case $t in c4) A="";; s0) A="--emulate-shard 0/8";; s7) A="--emulate-shard 7/8";; esac
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/$t -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --profile-steps $A > $O/$t.json 2> $O/$t.err || exit 1
  echo "$t ok"
done
