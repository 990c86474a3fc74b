# r5n: PMC traffic / MFMA busy for the lego preset and the T2^20 table (tools/gpu_pmc.sh), and the
# test-time render FPS (tools/render_fps.py) on the current tree.
set -o pipefail
mkdir -p gpurun_out/r5n
export TMPDIR=/tmp
timeout -k 10 500 bash tools/gpu_pmc.sh > gpurun_out/r5n/pmc_lego.log 2>&1 || { tail -20 gpurun_out/r5n/pmc_lego.log; exit 1; }
LOG2T=20 timeout -k 10 500 bash tools/gpu_pmc.sh > gpurun_out/r5n/pmc_T20.log 2>&1 || { tail -20 gpurun_out/r5n/pmc_T20.log; exit 1; }
timeout -k 10 300 python tools/render_fps.py > gpurun_out/r5n/render_fps.json 2> gpurun_out/r5n/render_fps.err || { tail -20 gpurun_out/r5n/render_fps.err; exit 1; }
cat gpurun_out/r5n/render_fps.json
