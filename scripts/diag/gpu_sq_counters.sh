# SQ / TCC counters per k_expand dispatch of one C4 step (separate passes), tables under gpurun_out/sq
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/sq
mkdir -p $O
ARGS="--steps 1 --warmup 0 --no-cpu-baseline --profile-steps ${EXTRA}"
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES" \
           "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum" \
           "SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_BUSY_CYCLES SQ_INSTS_SMEM"; do
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $O/p$i -o p -- python3 bench.py $ARGS > $O/p$i.json 2> $O/p$i.err || { echo "pass $i failed"; exit 1; }
  i=$((i+1))
done
python3 scripts/pmc_table.py $O k_expand > $O/k_expand.md
cat $O/k_expand.md
