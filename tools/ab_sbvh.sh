#!/bin/bash
# spatial splits A/B: parity (SBVH tests), kernel times with / without bvhSpatial, frame bench both ways
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/sbvh"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "spatial or variants or deep_stack" > "$OUT/tests.log" 2>&1 || { echo TESTFAIL; tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
SP="--pre-setting bvhSpatial=${ALPHA:-1e-5} --pre-setting bvhSpatialBudget=${BUDGET:-1}"
for rep in 1 2; do
  timeout -k 10 120 python3 tools/trace_kernel_bench.py --set both --iters 20 > "$OUT/off.log" 2>&1 || exit 1
  echo "off $(tail -1 "$OUT/off.log" | cut -c1-160)"
  timeout -k 10 120 python3 tools/trace_kernel_bench.py --set both --iters 20 $SP > "$OUT/on.log" 2>&1 || exit 1
  echo "on  $(tail -1 "$OUT/on.log" | cut -c1-160)"
done
for cfg in off on; do
  if [ $cfg = on ]; then A="--setting bvhSpatial=${ALPHA:-1e-5} --setting bvhSpatialBudget=${BUDGET:-1}"; else A=""; fi
  timeout -k 10 200 python3 bench.py --steps 20 --no-cpu-baseline --no-config4 $A > "$OUT/bench_$cfg.json" 2> "$OUT/bench_$cfg.log" || exit 1
  python3 -c "import json;d=json.load(open('$OUT/bench_$cfg.json'));print('bench $cfg',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['detail']['traceTime0_ms'],d['detail']['traceTime1_ms'],d['detail']['shadeTime_ms'],d['detail']['setup_s'])"
done
