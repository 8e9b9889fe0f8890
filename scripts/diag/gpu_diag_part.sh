# the k_arcmask store reproducer, GPU parity subset, C4 vertex-partition volumes
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/part
timeout -k 10 300 ./scripts/diag/arcmask_repro 22 6 > gpurun_out/arcmask_repro.log 2>&1
echo "arcmask_repro exit $?"; tail -8 gpurun_out/arcmask_repro.log
bash scripts/gpu_partition.sh "$@"
