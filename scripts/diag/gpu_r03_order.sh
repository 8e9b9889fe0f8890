# round 3: message order (gp_spread_keys + overlay.spread_order) -- parity, then same-box A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "spread" > gpurun_out/gpu_order_tests.txt 2>&1 || { tail -40 gpurun_out/gpu_order_tests.txt; exit 1; }
tail -3 gpurun_out/gpu_order_tests.txt
echo "== C4"
VARIANTS="given:--message-order given|h1:--message-order spread --spread-hops 1|h2:--message-order spread --spread-hops 2|h3:--message-order spread --spread-hops 3" ROUNDS=2 timeout -k 10 600 bash scripts/gpu_ab_args.sh || exit 1
echo "== 2048-message shard"
VARIANTS="given:--message-order given --messages 2048|h2:--message-order spread --messages 2048|h3:--message-order spread --spread-hops 3 --messages 2048" ROUNDS=2 timeout -k 10 300 bash scripts/gpu_ab_args.sh || exit 1
echo "== C5"
VARIANTS="given:--message-order given|h2:--message-order spread|h3:--message-order spread --spread-hops 3" WORKLOAD=c5 STEPS=3 ROUNDS=2 timeout -k 10 600 bash scripts/gpu_ab_args.sh || exit 1
