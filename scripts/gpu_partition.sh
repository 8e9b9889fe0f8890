# GPU parity subset, then the C4 vertex-partition exchange volumes at P = 2, 4, 8 (group mode, one GPU)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/part
if [ -n "$1" ]; then
  timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu $1 ${2:+-k "$2"} > gpurun_out/pytest_sel.log 2>&1
  rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/pytest_sel.log
  [ $rc -eq 0 ] || exit $rc
fi
for P in ${PARTS:-2 4 8}; do
  timeout -k 10 300 python -u scripts/partition_c4.py $P > gpurun_out/part/p$P.jsonl 2> gpurun_out/part/p$P.err
  rc=$?; echo "P=$P exit $rc"; tail -2 gpurun_out/part/p$P.jsonl; tail -2 gpurun_out/part/p$P.err
  [ $rc -eq 0 ] || exit $rc
done
