set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_bridge.py -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/pytest_bridge.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -30 gpurun_out/pytest_bridge.log
exit $rc
