# quick GPU check: selected tests (TESTS), then alternating bench knob sets (VARIANTS, see gpu_ab_args.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  GP_ORACLE_PROGRESS=1 timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest $TESTS -x -v -s --timeout 600 --timeout-method thread -m gpu --durations=10 > gpurun_out/pytest_check.log 2>&1
  rc=$?; echo "pytest exit $rc"; grep -E "passed|failed|error" gpurun_out/pytest_check.log | tail -5
  [ $rc -eq 0 ] || { tail -60 gpurun_out/pytest_check.log; exit $rc; }
fi
if [ -n "$VARIANTS" ]; then
  bash scripts/gpu_ab_args.sh || exit 1
fi
