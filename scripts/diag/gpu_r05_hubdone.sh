# round 5: hub chunks of an early-exit round stop once another chunk of their hub covered its target
# (hub_done), base = with the hub prefix clipping: GPU suite
# without the C5 full-size case, then base vs hubdone on C4 and C5
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu -k "not c5_full" > gpurun_out/pytest_hubdone.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_hubdone.log; [ $rc -eq 0 ] || exit $rc
L=gossip-protocol-with-power-law_amd/_ab
LIBS="$L/base.so $L/hubdone.so" ROUNDS=3 STEPS=10 bash scripts/gpu_ab_libs.sh || exit 1
LIBS="$L/base.so $L/hubdone.so" ROUNDS=2 STEPS=3 WORKLOAD=c5 bash scripts/gpu_ab_libs.sh
