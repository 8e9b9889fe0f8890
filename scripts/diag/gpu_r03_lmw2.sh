# round 3: written line masks, only in rounds without early exit (lmw2) vs every 64-word pull (lmw) vs
# none (nolmw); parity subset of lmw2 first
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_full_size.py -x -q --timeout 1200 --timeout-method thread -k "message_widths or wide_rows or spread or c4_full or done_in or checkpoint or edge_cases or hub_split or c1_ or c2_ba" > gpurun_out/gpu_lmw2_tests.txt 2>&1 || { tail -40 gpurun_out/gpu_lmw2_tests.txt; exit 1; }
tail -2 gpurun_out/gpu_lmw2_tests.txt
A=gossip-protocol-with-power-law_amd/_ab
echo "== C4"
LIBS="$A/nolmw.so $A/lmw.so $A/lmw2.so" ROUNDS=3 timeout -k 10 500 bash scripts/gpu_ab_libs.sh || exit 1
