# r5f: issue profile of the march alone (kbench march: AABB, clamp, noise, march_wave, scan, expand):
# kernel trace + SQ counter passes (tools/pmc_sq.sh)
set -o pipefail
mkdir -p gpurun_out
STAGE=march bash tools/pmc_sq.sh && cat gpurun_out/pmc_sq_march.txt | grep -A40 "march_wave"
python3 tools/kstats.py gpurun_out/pmc_sq_march/ktr march
