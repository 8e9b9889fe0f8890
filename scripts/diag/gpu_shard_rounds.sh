# per-GPU work of the N = 2/4/8 message shards on one MI355X (2048/1024/512 msgs), per-round stats
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for m in 512 1024 2048; do
  timeout -k 10 200 python -u bench.py --messages $m --steps 3 --warmup 1 --profile-steps --no-cpu-baseline > gpurun_out/shard_$m.json 2> gpurun_out/shard_$m.err || exit $?
  echo "== $m"; python -c "import json;d=json.load(open('gpurun_out/shard_$m.json'));print(d['ms_per_step'], d['roofline']['frac'])"
  grep round gpurun_out/shard_$m.err | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['round'],d['mode'],d['scan'],round(d['expand_ms'],2),round(d['kernel_ms'],2),d['arcs_scanned'],d['rows_gathered'],d['seen_rows_read'],d['rows_written'],d['row_bytes'])"
done
