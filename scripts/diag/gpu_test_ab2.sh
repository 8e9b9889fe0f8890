# GPU parity suite (current build), then an A/B of library variants: LIBS="a.so b.so"
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 500 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/pytest_ab.log 2>&1
  rc=$?; echo "pytest exit $rc"; tail -12 gpurun_out/pytest_ab.log
  [ $rc -eq 0 ] || exit $rc
fi
bash scripts/gpu_ab_libs.sh
