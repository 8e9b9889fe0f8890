set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters.txt 2>&1
echo "list exit $?"
grep -c . gpurun_out/counters.txt
