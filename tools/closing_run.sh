#!/bin/bash
# Closing evidence of a tree (GPU box), one parameterised runner in place of the per-call scripts:
#   D=gpurun_out/<id> STEPS="tests smoke bench mf128 T20 dp train30k timeline" bash tools/closing_run.sh
# Each step has its own time limit; any failure -- a failing pytest (exit 1 included), a crash, a
# time limit -- stops the run there, so no bench / 30k-step evidence is produced for a tree whose GPU
# suite failed.  Outputs under $D.
set -o pipefail
D=${D:-gpurun_out/closing}
mkdir -p $D
export TMPDIR=/tmp
STEPS=${STEPS:-"tests smoke bench mf128 T20 dp timeline"}
line() { python -c "import json;d=json.load(open('$1'));print('$(basename $1 .json)',d['ms_per_step'],d['value'],d.get('grid_bw_ms'),d.get('density_update_ms'),d['roofline']['frac'])"; }
for s in $STEPS; do
  case $s in
    tests)
      export MFNERF_PARITY_OUT=$GRAFT_REPO_ROOT/$D/parity_train.json
      timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread -p no:cacheprovider > $D/tests.log 2>&1 || { tail -40 $D/tests.log; exit 1; }
      tail -1 $D/tests.log ;;
    smoke)
      timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
      tail -1 $D/smoke.log ;;
    bench)
      timeout -k 10 400 python bench.py > $D/bench.json 2> $D/bench.err || { tail -20 $D/bench.err; exit 1; }
      line $D/bench.json ;;
    mf128)
      timeout -k 10 200 python bench.py --no-cpu-baseline --preset mf128 > $D/bench_mf128.json 2> $D/bench_mf128.err || { tail -20 $D/bench_mf128.err; exit 1; }
      line $D/bench_mf128.json ;;
    T20)
      timeout -k 10 200 python bench.py --no-cpu-baseline --log2-T 20 > $D/bench_T20.json 2> $D/bench_T20.err || { tail -20 $D/bench_T20.err; exit 1; }
      line $D/bench_T20.json ;;
    dp)
      timeout -k 10 200 python bench.py --no-cpu-baseline --dp-rehearse > $D/bench_dp_rehearse.json 2> $D/bench_dp_rehearse.err || { tail -20 $D/bench_dp_rehearse.err; exit 1; }
      line $D/bench_dp_rehearse.json ;;
    train30k)
      timeout -k 10 400 python tools/train_30k.py > $D/train30k.json 2> $D/train30k.err || { tail -20 $D/train30k.err; exit 1; }
      tail -c 400 $D/train30k.json ;;
    timeline)
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$D/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 40 --warmup 10 --no-cpu-baseline > $GRAFT_REPO_ROOT/$D/prof.log 2>&1) || { tail -20 $D/prof.log; exit 1; }
      python3 tools/step_timeline.py $D/prof > $D/timeline.txt && head -30 $D/timeline.txt ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
