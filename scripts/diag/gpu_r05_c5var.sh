# round 5: run-to-run spread of C5's round 3 (73-84 ms across processes with one library): 5 bench
# processes on one box, per-round kernel ms of each
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/c5var
for k in 1 2 3 4 5; do
  timeout -k 10 200 python -u bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline --profile-steps > gpurun_out/c5var/$k.json 2> gpurun_out/c5var/$k.err || exit 1
  python3 scripts/emu_line.py run$k gpurun_out/c5var/$k.json gpurun_out/c5var/$k.err
done
