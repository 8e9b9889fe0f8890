# round 5: churn-tail scans probe 4 passes ahead and skip the inactive ones
# (gather_scan SKIP, k_expand<W, SCAN_FILTERED | SCAN_ALIVE>): churn and
# liveness parity incl. the C5 full-size case, then base vs skip on C5
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests -x -q --timeout 600 --timeout-method thread -m gpu -k "churn or crash or c5 or alive or liveness or detect" > gpurun_out/pytest_skip.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_skip.log; [ $rc -eq 0 ] || exit $rc
L=gossip-protocol-with-power-law_amd/_ab
LIBS="$L/base.so $L/skip.so" ROUNDS=3 STEPS=3 WORKLOAD=c5 bash scripts/gpu_ab_libs.sh
