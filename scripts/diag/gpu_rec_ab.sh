# GPU parity suite, then C4 A/B of Message-List records (--compact-rows 0 / 1), alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py} -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/pytest_rec.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -15 gpurun_out/pytest_rec.log
[ $rc -eq 0 ] || exit $rc
for x in 0 1 0 1; do
  timeout -k 10 120 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --profile-steps --compact-rows $x $EXTRA > gpurun_out/cml$x.json 2> gpurun_out/cml$x.err || exit 1
  python3 scripts/round_table.py cml=$x gpurun_out/cml$x.json gpurun_out/cml$x.err
done
