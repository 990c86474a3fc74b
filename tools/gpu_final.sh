#!/bin/bash
# Round-end session: the whole GPU check (tests, smoke, benches, render FPS, kernel stats), then the
# PMC passes (traffic, atomics, MFMA busy).  Each GPU step has its own time limit; && chains them.
set -o pipefail
STEPS=${STEPS:-200} bash tools/gpu_check.sh > gpurun_out/check.out 2>&1 || { tail -30 gpurun_out/check.out; exit 1; }
tail -12 gpurun_out/check.out | cut -c1-400
bash tools/gpu_pmc.sh > gpurun_out/pmc.out 2>&1 || { tail -20 gpurun_out/pmc.out; exit 1; }
cat gpurun_out/pmc_mfma.txt | head -20
