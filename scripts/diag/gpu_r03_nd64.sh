# round 3: no near-done rows-in-flight switch for 64-word rows (nd64) against HEAD -- parity subset, then
# same-box A/B on C4 and the 2048-message shard (unchanged code path at W = 32)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_full_size.py -x -q --timeout 1200 --timeout-method thread -k "message_widths or wide_rows or spread or c4_full or done_in or hub_split or edge_cases" > gpurun_out/gpu_nd64_tests.txt 2>&1 || { tail -40 gpurun_out/gpu_nd64_tests.txt; exit 1; }
tail -2 gpurun_out/gpu_nd64_tests.txt
A=gossip-protocol-with-power-law_amd/_ab
echo "== C4"
LIBS="$A/head.so $A/nd64.so" ROUNDS=3 timeout -k 10 400 bash scripts/gpu_ab_libs.sh || exit 1
