# Library variants on the blocked message shards of the N = 2 / 4 / 8 jobs and
# the whole C4 run, one process per library (scripts/diag/shard_study.py):
# LIBS="a.so b.so" [RANGES=...]
set -o pipefail
cd $GRAFT_REPO_ROOT
R=${RANGES:-0:8,8:8,16:8,24:8,32:8,40:8,48:8,56:8,0:16,16:16,32:16,48:16,0:32,32:32,0:64}
for k in 1 2; do
for lib in $LIBS; do
  tag=$(basename $lib .so)
  mkdir -p gpurun_out/sl/$tag.$k
  GOSSIP_HIP_LIB=$lib timeout -k 10 300 python3 -u scripts/diag/shard_study.py --no-arrival --sizes "" \
      --ranges $R --out gpurun_out/sl/$tag.$k > gpurun_out/sl/$tag.$k/log.txt 2>&1 || { tail gpurun_out/sl/$tag.$k/log.txt; exit 1; }
  python3 - gpurun_out/sl/$tag.$k/shards.jsonl "$tag" <<'PY'
import json, sys
rs = [json.loads(l) for l in open(sys.argv[1])]
print(f"{sys.argv[2]:10s}", " ".join(f"{r['w0']}:{r['words']}={r['ms']:.2f}" for r in rs), flush=True)
PY
done
done
