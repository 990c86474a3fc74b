set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/eng.log 2>&1 || { tail -40 gpurun_out/eng.log; exit 1; }
tail -2 gpurun_out/eng.log
for g in 1 0 1 0; do
MFNERF_GATED_MARCH=$g timeout -k 10 200 python bench.py --steps 400 --warmup 30 --no-cpu-baseline > gpurun_out/b$g.json 2>gpurun_out/b$g.err || { tail -20 gpurun_out/b$g.err; exit 1; }
echo "gated=$g"; python -c "import json;d=json.load(open('gpurun_out/b$g.json'));print(d['ms_per_step'],d['value'])"
done
