set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
PARAM=--messages LIST="2048 1024 512" bash scripts/gpu_sweep.sh || exit 1
EXTRA="--flat-max-words 0" PARAM=--messages LIST="1024 512" bash scripts/gpu_sweep.sh || exit 1
EXTRA="--flat-max-words 32" PARAM=--messages LIST="2048" bash scripts/gpu_sweep.sh || exit 1
