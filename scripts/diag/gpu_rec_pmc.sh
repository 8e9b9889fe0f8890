# round 2 with compact rows (k_expand_rec) vs full rows (k_expand<64,0>): HBM traffic and SQ stall counters
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/recpmc
mkdir -p $O
A="--steps 1 --warmup 0 --no-cpu-baseline --profile-steps"
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES"
for cr in 0 1; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f$cr -o f -- python3 bench.py $A --compact-rows $cr > $O/f$cr.json 2> $O/f$cr.err || exit 1
  timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d $O/s$cr -o s -- python3 bench.py $A --compact-rows $cr > $O/s$cr.json 2> $O/s$cr.err || exit 1
  echo "cr=$cr ok"
done
python3 - <<'PY'
import csv, glob, collections
for cr in (0, 1):
    for tag in ("f", "s"):
        path = glob.glob(f"gpurun_out/recpmc/{tag}{cr}/**/*counter_collection.csv", recursive=True)[0]
        per = collections.defaultdict(dict)
        names = {}
        for r in csv.DictReader(open(path)):
            k = int(r["Dispatch_Id"]); names[k] = r["Kernel_Name"].split("(")[0][:40]
            per[k][r["Counter_Name"]] = per[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        for k in sorted(per):
            if "k_expand" in names[k]:
                print(cr, tag, k, names[k], {c: round(v) for c, v in sorted(per[k].items())})
PY
