# builder parity + degree tests, C4 and C5 bench lines (setup times), message-shard per-GPU times
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -m gpu -k "builder or degree or c3" > gpurun_out/pytest_misc.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -2 gpurun_out/pytest_misc.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --profile-steps > gpurun_out/c4.json 2> gpurun_out/c4.err || exit 1
python3 scripts/round_table.py c4 gpurun_out/c4.json gpurun_out/c4.err; grep -o '"setup_s": [0-9.]*, "build_s": [0-9.]*' gpurun_out/c4.json
timeout -k 10 300 python3 bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline --profile-steps > gpurun_out/c5.json 2> gpurun_out/c5.err || exit 1
python3 scripts/round_table.py c5 gpurun_out/c5.json gpurun_out/c5.err; grep -o '"setup_s": [0-9.]*, "build_s": [0-9.]*' gpurun_out/c5.json
bash scripts/gpu_shards.sh
