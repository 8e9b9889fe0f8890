# round 3: message order -- parity (spread tests, full-size C4/C5 on the ordered table), C5 A/B of the key radius
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_full_size.py -x -v -s --timeout 1200 --timeout-method thread -k "spread or full_size" > gpurun_out/gpu_order_tests.txt 2>&1 || { tail -40 gpurun_out/gpu_order_tests.txt; exit 1; }
grep -E "PASS|FAIL|passed|failed|oracle|whole run" gpurun_out/gpu_order_tests.txt | tail -30
echo "== C5"
VARIANTS="given:--message-order given|h2:--message-order spread --spread-hops 2|h3:--message-order spread --spread-hops 3" WORKLOAD=c5 STEPS=3 ROUNDS=2 timeout -k 10 600 bash scripts/gpu_ab_args.sh || exit 1
