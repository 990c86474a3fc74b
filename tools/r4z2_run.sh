# Round-4 final evidence, part 2 (GPU box): PMC traffic / MFMA busy and the SQ issue profiles.
set -o pipefail
D=gpurun_out/r4z
mkdir -p $D
export TMPDIR=/tmp
bash tools/gpu_pmc.sh || exit $?
PRESET=mf128 bash tools/gpu_pmc.sh || exit $?
STAGE=grid_bw bash tools/pmc_sq.sh || exit $?
STAGE=field_bw bash tools/pmc_sq.sh || exit $?
for f in pmc_traffic.json pmc_traffic_mf128.json pmc_mfma.txt pmc_mfma_mf128.txt pmc_sq_grid_bw.txt pmc_sq_field_bw.txt; do cp gpurun_out/$f $D/; done
