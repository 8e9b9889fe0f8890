# round 3: the first pass's column ids loaded beside the early-exit target (col) vs after it (nocol);
# parity subset, then same-box A/B on C4 and C5
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_full_size.py -x -q --timeout 1200 --timeout-method thread -k "message_widths or wide_rows or spread or c4_full or done_in or churn or sated or hub_split or edge_cases or summary" > gpurun_out/gpu_col_tests.txt 2>&1 || { tail -40 gpurun_out/gpu_col_tests.txt; exit 1; }
tail -2 gpurun_out/gpu_col_tests.txt
A=gossip-protocol-with-power-law_amd/_ab
echo "== C4"
LIBS="$A/nocol.so $A/col.so" ROUNDS=3 timeout -k 10 400 bash scripts/gpu_ab_libs.sh || exit 1
echo "== C5"
LIBS="$A/nocol.so $A/col.so" WORKLOAD=c5 STEPS=3 ROUNDS=2 timeout -k 10 500 bash scripts/gpu_ab_libs.sh || exit 1
