#!/bin/bash
# kernel-trace stats of library variants: LIBS="a.so b.so" WORKLOAD=c4|c5 bash scripts/gpu_kstats_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/kab
for lib in $LIBS; do
  tag=$(basename $lib .so)
  GOSSIP_HIP_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/kab/$tag -o run -- python3 bench.py --workload ${WORKLOAD:-c5} --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline > gpurun_out/kab/$tag.json 2> gpurun_out/kab/$tag.err || exit 1
  f=$(find gpurun_out/kab/$tag -name "*kernel_stats.csv" | head -1)
  echo "== $tag"; python3 scripts/prof_summary.py "$f" 2>/dev/null | head -${TOP:-14}
done
