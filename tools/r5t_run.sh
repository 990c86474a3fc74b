# r5t: HIP runtime launch settings A/B on the default bench (300 steps, twice): the per-node graph
# launch (bench.py's default DEBUG_CLR_GRAPH_PACKET_CAPTURE=0) vs the captured-packet path (=1), and
# kernel arguments in device memory (HIP_FORCE_DEV_KERNARG=1).
set -o pipefail
D=gpurun_out/r5t
mkdir -p $D
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 300 --warmup 30 --no-cpu-baseline > $D/$name.json 2> $D/$name.err || { tail -20 $D/$name.err; exit 1; }
  python -c "import json;d=json.load(open('$D/$name.json'));print('$name',d['ms_per_step'])"
}
for rep in 1 2; do
  run default
  run packet DEBUG_CLR_GRAPH_PACKET_CAPTURE=1
  run devkernarg HIP_FORCE_DEV_KERNARG=1
done
