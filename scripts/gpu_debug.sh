set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u scripts/debug_seq.py 3 1 512 2>&1 | grep -c "DIFF at"
timeout -k 10 300 python -u scripts/debug_seq.py 2 1 100000 2>&1 | grep -c "DIFF at"
