#!/bin/bash
# Benches over a list of environment settings (CONFIGS: space-separated "VAR=v,VAR2=w" items), twice each.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
for c in $CONFIGS; do
  env ${c//,/ } timeout -k 10 200 python bench.py --steps ${STEPS:-300} --warmup 30 --no-cpu-baseline > gpurun_out/abm.json 2> gpurun_out/abm.err || { tail -20 gpurun_out/abm.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/abm.json'));print('$c',d['ms_per_step'],d['value'])"
done
done
