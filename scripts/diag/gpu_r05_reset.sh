# round 5: fused per-run reset (k_reset) -- GPU parity suite without the
# full-size cases, then base vs reset1 on C4 and on the N = 8 job's rank 7
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu -k "not full_size" > gpurun_out/pytest_reset.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_reset.log; [ $rc -eq 0 ] || exit $rc
LIBS="gossip-protocol-with-power-law_amd/_ab/base.so gossip-protocol-with-power-law_amd/_ab/reset1.so" ROUNDS=2 STEPS=10 bash scripts/gpu_ab_libs.sh || exit 1
LIBS="gossip-protocol-with-power-law_amd/_ab/base.so gossip-protocol-with-power-law_amd/_ab/reset1.so" ROUNDS=2 STEPS=10 EXTRA="--emulate-shard 7/8" bash scripts/gpu_ab_libs.sh
