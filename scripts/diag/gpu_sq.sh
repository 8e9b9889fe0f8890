# SQ counters of k_expand for the current tree and the committed one (_old/)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LEVEL_WAVES SQ_WAVES SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
for tree in ${TREES:-. _old}; do
  out=$GRAFT_REPO_ROOT/gpurun_out/sq/$(echo $tree | tr -d './')x
  mkdir -p $out
  i=0
  for P in "$P1" "$P2"; do
    (cd $tree && timeout -s KILL 180 rocprofv3 --pmc $P --output-format csv -d $out/p$i -o p$i -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $out/p$i.json 2> $out/p$i.err) || exit 1
    i=$((i+1))
  done
  python3 scripts/pmc_table.py $out k_expand > $out/table.md
  echo "== $tree"; cat $out/table.md
done
