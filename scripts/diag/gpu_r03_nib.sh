# round 3: nibble-packed line masks -- parity subset, then same-box A/B against the byte array (C4, C5)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_full_size.py -x -q --timeout 1200 --timeout-method thread -k "message_widths or wide_rows or spread or c4_full or churn_random or group_partition_invariance" > gpurun_out/gpu_nib_tests.txt 2>&1 || { tail -40 gpurun_out/gpu_nib_tests.txt; exit 1; }
tail -2 gpurun_out/gpu_nib_tests.txt
A=gossip-protocol-with-power-law_amd/_ab
echo "== C4"
LIBS="$A/lmbyte.so $A/lmnib.so" ROUNDS=2 timeout -k 10 300 bash scripts/gpu_ab_libs.sh || exit 1
echo "== C5"
LIBS="$A/lmbyte.so $A/lmnib.so" WORKLOAD=c5 STEPS=3 ROUNDS=2 timeout -k 10 500 bash scripts/gpu_ab_libs.sh || exit 1
