# flat record pull (k_expand_rec): compact-row parity tests, then C4 with compact rows on / off, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -m gpu -k "compact or message_widths or c2 or wide_rows" > gpurun_out/pytest_rec.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_rec.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="rows:--compact-rows 0|recs:--compact-rows 1" ROUNDS=3 timeout -k 10 400 bash scripts/gpu_ab_args.sh
