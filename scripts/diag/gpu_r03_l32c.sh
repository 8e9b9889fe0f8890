# round 3: line masks at W = 32 with the early column ids at every width (l32c) against the previous HEAD
# (head) -- parity subset, then same-box A/B on the 2048-message shard and C4
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_full_size.py -x -q --timeout 1200 --timeout-method thread -k "message_widths or wide_rows or spread or c4_full or message_shards or done_in or hub_split or edge_cases or c2_ba or checkpoint" > gpurun_out/gpu_l32_tests.txt 2>&1 || { tail -40 gpurun_out/gpu_l32_tests.txt; exit 1; }
tail -2 gpurun_out/gpu_l32_tests.txt
A=gossip-protocol-with-power-law_amd/_ab
echo "== 2048-message shard"
LIBS="$A/head.so $A/l32c.so" EXTRA="--messages 2048" ROUNDS=3 timeout -k 10 400 bash scripts/gpu_ab_libs.sh || exit 1
