#!/bin/bash
# PMC traffic of k_expand per library variant (two passes each), then a timed
# A/B: LIBS="a.so b.so" [WORKLOAD=c4|c5] [ROUNDS=2]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
ARGS="--workload ${WORKLOAD:-c4} --steps 1 --warmup 0 --no-cpu-baseline --profile-steps"
for lib in $LIBS; do
  tag=$(basename $lib .so)
  O=gpurun_out/abpmc/$tag
  mkdir -p $O
  GOSSIP_HIP_LIB=$lib timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o fetch -- python3 bench.py $ARGS > $O/fetch.json 2> $O/fetch.err || exit 1
  GOSSIP_HIP_LIB=$lib timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o write -- python3 bench.py $ARGS > $O/write.json 2> $O/write.err || exit 1
  echo "== $tag"
  python3 scripts/pmc_summary.py $O $O/pmc_traffic.json > $O/pmc_traffic.md && cat $O/pmc_traffic.md || exit 1
done
bash scripts/gpu_ab_libs.sh
