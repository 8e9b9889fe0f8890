# round 3: line-mask rounds load the receiver's seen row and first column ids up front (se) vs seen row at the
# commit (nose) -- parity subset, then same-box A/B on C4 and C5
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_full_size.py -x -q --timeout 1200 --timeout-method thread -k "message_widths or wide_rows or spread or c4_full or churn or hub_split or edge_cases or c2_ba or checkpoint or group_partition_invariance" > gpurun_out/gpu_se_tests.txt 2>&1 || { tail -40 gpurun_out/gpu_se_tests.txt; exit 1; }
tail -2 gpurun_out/gpu_se_tests.txt
A=gossip-protocol-with-power-law_amd/_ab
echo "== C4"
LIBS="$A/nose.so $A/se.so" ROUNDS=3 timeout -k 10 400 bash scripts/gpu_ab_libs.sh || exit 1
echo "== C5"
LIBS="$A/nose.so $A/se.so" WORKLOAD=c5 STEPS=3 ROUNDS=2 timeout -k 10 500 bash scripts/gpu_ab_libs.sh || exit 1
