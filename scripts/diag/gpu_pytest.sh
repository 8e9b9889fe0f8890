#!/bin/bash
# usage: scripts/gpu_pytest.sh <log name> <timeout s> <pytest args...>
# runs one pytest process on the GPU box with a hard time limit, log under gpurun_out/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
name=$1; shift
lim=$1; shift
timeout -k 10 "$lim" python -u -m pytest -x -v --timeout 300 --timeout-method thread "$@" > "gpurun_out/$name.log" 2>&1
rc=$?
echo "pytest exit $rc"
grep -E "passed|failed|error" "gpurun_out/$name.log" | tail -3
exit $rc
