set -o pipefail
D=gpurun_out/r4i
mkdir -p $D
export TMPDIR=/tmp
ok() { rc=$?; [ $rc -le 1 ] || exit $rc; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider --deselect tests/test_gpu_parity_train.py::test_training_psnr_matches_reference > $D/tests.log 2>&1; ok
B="timeout -k 10 200 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --roofline-every 1000"
for rep in 1 2; do
for V in "composite 1 1 1" "composite 2 1 1" "composite 4 1 1" "field_bw 1 1 1" "field_bw 2 1 1" "composite 1 0 1" "composite 1 1 0" "field_bw 1 0 1"; do
  set -- $V
  MFNERF_GATE_AT=$1 MFNERF_MARCH_RPW=$2 MFNERF_SLAB_TAIL=$3 MFNERF_GATE_RIDE=$4 $B > $D/ab.json 2> $D/ab.err || exit $?
  python -c "import json;d=json.load(open('$D/ab.json'));print('gate=$1 rpw=$2 slab=$3 ride=$4',d['ms_per_step'],d['grid_bw_ms'])" >> $D/ab.txt
done
done
