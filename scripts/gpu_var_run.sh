set -o pipefail
cd $GRAFT_REPO_ROOT
V=gossip-protocol-with-power-law_amd/_variants
LIBS="$V/w0.so $V/w8.so" EXTRA="--sparse-rows 0" bash scripts/gpu_variants.sh || exit 1
LIBS="$V/w0.so $V/w8.so" EXTRA="--sparse-rows 1" bash scripts/gpu_variants.sh || exit 1
