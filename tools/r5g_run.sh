# r5g: the march's empty-cell jumps by pointer doubling -- bit-exact march tests (vren, configs,
# engine), the march's SQ profile, kbench march vs the previous commit, and a bench A/B.
set -o pipefail
D=gpurun_out/r5g
mkdir -p $D
timeout -k 10 500 python -u -m pytest tests/test_gpu_vren.py tests/test_gpu_configs.py tests/test_gpu_engine.py -q --maxfail=5 --timeout 120 --timeout-method thread -p no:cacheprovider > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
tail -1 $D/tests.log
STAGE=march bash tools/pmc_sq.sh && grep -A34 "^march_wave" gpurun_out/pmc_sq_march.txt | grep "=" ; python3 tools/kstats.py gpurun_out/pmc_sq_march/ktr march
MFNERF_LIB=$PWD/mf-nerf_amd/csrc/var/head.so timeout -k 10 120 python tools/kbench.py march
timeout -k 10 120 python tools/kbench.py march
LIBS="- mf-nerf_amd/csrc/var/head.so" STEPS=300 TESTS=tests/test_gpu_vren.py bash tools/ab_libs.sh
