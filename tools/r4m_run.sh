set -o pipefail
D=gpurun_out/r4m
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 120 python -c "import torch; print('priority_range', torch.cuda.Stream.priority_range()); s=torch.cuda.Stream(priority=torch.cuda.Stream.priority_range()[0]); print('least', s.priority)" > $D/prio.txt 2>&1 || exit $?
B="timeout -k 10 200 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --roofline-every 1000"
for rep in 1 2 3; do
for V in "normal" "low"; do
  MFNERF_SIDE_PRIORITY=$V $B > $D/ab.json 2> $D/ab.err || exit $?
  python -c "import json;d=json.load(open('$D/ab.json'));print('prio=$V',d['ms_per_step'],d['grid_bw_ms'])" >> $D/ab.txt
done
done
