# arbitrary rocprofv3 --pmc passes over one C4 step; PASSES="A1,A2;B1,B2" (';' separates passes)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmcx
export TMPDIR=/tmp
ARGS="--steps 1 --warmup 0 --no-cpu-baseline --profile-steps $EXTRA"
i=0
IFS=';' read -ra PS <<< "$PASSES"
for p in "${PS[@]}"; do
  cs=$(echo $p | tr ',' ' ')
  timeout -s KILL 180 rocprofv3 --pmc $cs --output-format csv -d gpurun_out/pmcx/p$i -o p$i -- python3 bench.py $ARGS > gpurun_out/pmcx/p$i.json 2> gpurun_out/pmcx/p$i.err || exit 1
  i=$((i+1))
done
python3 scripts/pmc_table.py gpurun_out/pmcx k_expand > gpurun_out/pmcx/table.md
cat gpurun_out/pmcx/table.md
