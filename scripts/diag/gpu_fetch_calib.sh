# FETCH_SIZE calibration for the engine's access widths (scripts/diag/fetch_calib.hip)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/calib
mkdir -p $O
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o calib -- ./scripts/diag/fetch_calib > $O/run.txt 2>&1 || { tail -20 $O/run.txt; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d $O/req -o calib -- ./scripts/diag/fetch_calib > $O/run2.txt 2>&1 || tail -5 $O/run2.txt
timeout -s KILL 60 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/hit -o calib -- ./scripts/diag/fetch_calib > $O/run3.txt 2>&1 || tail -5 $O/run3.txt
for f in $(find $O -name "*counter_collection.csv"); do echo "== $f"; python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    print(r.get("Kernel_Name", "")[:40], r.get("Counter_Name"), r.get("Counter_Value"))
PY
done
