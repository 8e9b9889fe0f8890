# round 3: done in-neighbours -- GPU parity at HEAD, then same-box A/B (C4, shards)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_full_size.py -x -q --timeout 300 --timeout-method thread -k "done_in or wide_rows or message_widths or c4_full or c2_ba" > gpurun_out/gpu_suite.txt 2>&1 || { tail -30 gpurun_out/gpu_suite.txt; exit 1; }
tail -3 gpurun_out/gpu_suite.txt
A=gossip-protocol-with-power-law_amd/_ab
echo "== C4"
LIBS="$A/base.so $A/dnb.so $A/dnbser.so" ROUNDS=2 timeout -k 10 300 bash scripts/gpu_ab_libs.sh || exit 1
echo "== 2048-message shard"
LIBS="$A/base.so $A/dnb.so" EXTRA="--messages 2048" ROUNDS=2 timeout -k 10 300 bash scripts/gpu_ab_libs.sh || exit 1
echo "== 512-message shard"
LIBS="$A/base.so $A/dnb.so" EXTRA="--messages 512" ROUNDS=2 timeout -k 10 300 bash scripts/gpu_ab_libs.sh || exit 1
