set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for cfg in "0 1 12 1 512" "0 1 12 0 512" "0 1 12 1 100000" "0 0 12 1 512" "10 1 12 1 512"; do
  timeout -k 10 150 python scripts/debug_repeat.py $cfg > gpurun_out/rep.txt 2>&1 || { echo "cfg $cfg FAILED/TIMEOUT"; cat gpurun_out/rep.txt; exit 1; }
  echo "cfg $cfg: $(grep -c ' ok ' gpurun_out/rep.txt) ok, $(grep -vc ' ok ' gpurun_out/rep.txt) other"; grep -v ' ok ' gpurun_out/rep.txt | head -3
done
