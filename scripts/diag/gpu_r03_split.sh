# round 3: done-in-neighbour receivers in a pass of their own (k_expand<64, ... | SCAN_DNB>, GP_DNB_BATCH pairs
# in flight) -- parity subset, then same-box A/B: nosplit (in the main kernel, one pair at a time), split (4 pairs),
# split2 (2 pairs)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_full_size.py -x -q --timeout 1200 --timeout-method thread -k "done_in or message_widths or wide_rows or spread or c4_full or hub_split or edge_cases or c2_ba or checkpoint or message_shards" > gpurun_out/gpu_split_tests.txt 2>&1 || { tail -40 gpurun_out/gpu_split_tests.txt; exit 1; }
tail -2 gpurun_out/gpu_split_tests.txt
A=gossip-protocol-with-power-law_amd/_ab
echo "== C4"
LIBS="$A/nosplit.so $A/split.so $A/split2.so" ROUNDS=2 timeout -k 10 400 bash scripts/gpu_ab_libs.sh || exit 1
echo "== 2048-message shard"
LIBS="$A/nosplit.so $A/split.so" EXTRA="--messages 2048" ROUNDS=2 timeout -k 10 300 bash scripts/gpu_ab_libs.sh || exit 1
