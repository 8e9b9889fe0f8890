# round 5: W = 8 flat kernel -- rows in flight 5, LDS trimmed to 5,104 B per
# one-wave block (staging / receiver-side union, one counter row), waves per
# SIMD forced to 8 (non-early-exit) and 6 (early-exit): parity of the most
# aggressive variant on the narrow-row tests, then ranks 7 and 0 of the N = 8 job
set -o pipefail
cd $GRAFT_REPO_ROOT
L=gossip-protocol-with-power-law_amd/_ab
GOSSIP_HIP_LIB=$L/u8e6.so timeout -k 10 600 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu -k "width or shard or churn or hub or flat" > gpurun_out/pytest_flatlds.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_flatlds.log; [ $rc -eq 0 ] || exit $rc
LIBS="$L/base.so $L/r5.so $L/u1.so $L/u8.so $L/u8e6.so" ROUNDS=2 STEPS=10 EXTRA="--emulate-shard 7/8" bash scripts/gpu_ab_libs.sh || exit 1
LIBS="$L/base.so $L/r5.so $L/u1.so $L/u8.so $L/u8e6.so" ROUNDS=2 STEPS=10 EXTRA="--emulate-shard 0/8" bash scripts/gpu_ab_libs.sh
