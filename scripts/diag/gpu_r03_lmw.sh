# round 3: line masks written by the previous round's commits (no k_mklm pass) -- parity subset, then
# same-box A/B against the same source with GP_LM_WRITE=0 (k_mklm every line-mask round)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_full_size.py -x -q --timeout 1200 --timeout-method thread -k "message_widths or wide_rows or spread or c4_full or done_in or checkpoint or group_partition_invariance or edge_cases or hub_split or c1_ or c2_ba or compact" > gpurun_out/gpu_lmw_tests.txt 2>&1 || { tail -40 gpurun_out/gpu_lmw_tests.txt; exit 1; }
tail -2 gpurun_out/gpu_lmw_tests.txt
A=gossip-protocol-with-power-law_amd/_ab
echo "== C4"
LIBS="$A/nolmw.so $A/lmw.so" ROUNDS=3 timeout -k 10 400 bash scripts/gpu_ab_libs.sh || exit 1
