# round 3: packed line-mask entries (gather_lines) -- parity subset, then rows in flight of the
# line-mask gather (lbase = previous HEAD, lr3 / lr4 / lr6), same-box A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_full_size.py -x -q --timeout 1200 --timeout-method thread -k "message_widths or wide_rows or spread or c4_full or churn_random or group_partition_invariance" > gpurun_out/gpu_lrif_tests.txt 2>&1 || { tail -40 gpurun_out/gpu_lrif_tests.txt; exit 1; }
tail -2 gpurun_out/gpu_lrif_tests.txt
A=gossip-protocol-with-power-law_amd/_ab
echo "== C4"
LIBS="$A/lbase.so $A/lr3.so $A/lr4.so $A/lr6.so" ROUNDS=2 timeout -k 10 400 bash scripts/gpu_ab_libs.sh || exit 1
echo "== C5"
LIBS="$A/lbase.so $A/lr3.so $A/lr4.so" WORKLOAD=c5 STEPS=3 ROUNDS=1 timeout -k 10 500 bash scripts/gpu_ab_libs.sh || exit 1
