# parity subset at HEAD (64-word paths, churn, partitions, checkpoints, full-size C4/C5), then the C4 bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_full_size.py -x -q --timeout 1200 --timeout-method thread -k "message_widths or wide_rows or spread or full_size or done_in or checkpoint or group_partition or edge_cases or hub_split or churn or sated or lost or detection or finalize or compact" > gpurun_out/gpu_check.txt 2>&1 || { tail -40 gpurun_out/gpu_check.txt; exit 1; }
tail -2 gpurun_out/gpu_check.txt
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
cat gpurun_out/bench.json
