# round 3: knob sweep at HEAD (after message order + line masks), same box, alternating: build knobs
# (rows in flight, near-done rows in flight, done-neighbour probes, early-exit threshold) and bench knobs
set -o pipefail
cd $GRAFT_REPO_ROOT
A=gossip-protocol-with-power-law_amd/_ab
echo "== C4 build knobs"
LIBS="$A/base.so $A/rif3.so $A/rif5.so $A/nd1.so $A/nd3.so $A/dnb1.so $A/dnb4.so $A/ee8.so $A/ee32.so" ROUNDS=2 timeout -k 10 800 bash scripts/gpu_ab_libs.sh || exit 1
echo "== C4 bench knobs"
VARIANTS="base:|unf80:--unfiltered-pct 80|unf97:--unfiltered-pct 97|pre10:--prefilter-pct 10|pre35:--prefilter-pct 35|push50:--push-ratio 50|push200:--push-ratio 200" ROUNDS=2 timeout -k 10 600 bash scripts/gpu_ab_args.sh || exit 1
