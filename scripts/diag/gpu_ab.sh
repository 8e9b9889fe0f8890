# A/B: committed tree (_old/) vs working tree, same box
set -o pipefail
cd $GRAFT_REPO_ROOT
for k in 1 2; do
for tree in _old .; do
  (cd $tree && timeout -k 10 120 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --profile-steps $EXTRA > /tmp/ab.json 2> /tmp/ab.err) || exit 1
  python3 - "$tree" <<'PY'
import json, sys
d = json.loads(open("/tmp/ab.json").read())
rs = [json.loads(l) for l in open("/tmp/ab.err") if l.startswith("{")]
print(sys.argv[1], round(d["value"]), "GTEPS", round(d["ms_per_step"], 2), "ms |",
      " ".join(f"r{r['round']}:{'P' if r['mode'] else 'L'}{r['expand_ms']:.2f}" for r in rs))
PY
done
done
