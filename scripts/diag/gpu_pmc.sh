# HBM traffic of the expansion kernels: separate rocprofv3 --pmc passes
# (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950; MI355X_MICROARCH.md)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
ARGS="--steps 1 --warmup 0 --no-cpu-baseline --profile-steps $EXTRA"
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc/fetch -o fetch -- python3 bench.py $ARGS > gpurun_out/pmc/fetch.json 2> gpurun_out/pmc/fetch.err || exit 1
echo "fetch ok"
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc/write -o write -- python3 bench.py $ARGS > gpurun_out/pmc/write.json 2> gpurun_out/pmc/write.err || exit 1
echo "write ok"
python3 scripts/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc/summary.md
cat gpurun_out/pmc/summary.md
