#!/bin/bash
# A/B of an environment knob on one box: alternating benches with $VAR=$A and $VAR=$B.
set -o pipefail
mkdir -p gpurun_out
for v in $A $B $A $B; do
  env $VAR=$v timeout -k 10 200 python bench.py --steps ${STEPS:-300} --warmup 30 --no-cpu-baseline > gpurun_out/abe_$v.json 2> gpurun_out/abe_$v.err || { tail -20 gpurun_out/abe_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/abe_$v.json'));print('$VAR=$v',d['ms_per_step'],d['value'])"
done
