#!/bin/bash
# parking: churn parity (incl. C5 full size), then C5 A/B park off/on
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -k "${TESTS:-parks or churn or checkpoint or finalize or lost or summary}" > gpurun_out/park_tests.log 2>&1 || { tail -30 gpurun_out/park_tests.log; exit 1; }
tail -3 gpurun_out/park_tests.log
if [ -z "$NO_C5" ]; then
timeout -k 10 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread \
  tests/test_full_size.py -k c5 > gpurun_out/park_c5.log 2>&1 || { tail -30 gpurun_out/park_c5.log; exit 1; }
tail -3 gpurun_out/park_c5.log
fi
P=gossip-protocol-with-power-law_amd/_ab
LIBS="${LIBS:-$P/park0.so $P/park1.so}" WORKLOAD=c5 ROUNDS=2 bash scripts/gpu_ab_libs.sh
