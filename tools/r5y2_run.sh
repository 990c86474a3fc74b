# r5y2: tests for the 3840-record accumulate stage (two chunks per Lego partition now), the issue
# profile of the planar forward encode, and the TA / TCP / TCC counter names on this box.
set -o pipefail
D=gpurun_out/r5y2
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_field.py tests/test_gpu_configs.py tests/test_gpu_engine.py tests/test_gpu_optim.py tests/test_gpu_dp.py -q --maxfail=3 --timeout 120 --timeout-method thread -p no:cacheprovider > $D/tests.log 2>&1 || { tail -60 $D/tests.log; exit 1; }
tail -1 $D/tests.log
STAGE=grid_fw_planar bash tools/pmc_sq.sh && tail -30 gpurun_out/pmc_sq_grid_fw_planar.txt
timeout -s KILL 60 rocprofv3 -L > $D/counters.txt 2>&1; grep -oE "\b(TA|TCP|TD)_[A-Z0-9_]+" $D/counters.txt | sort -u > $D/ta_tcp.txt; wc -l $D/ta_tcp.txt
