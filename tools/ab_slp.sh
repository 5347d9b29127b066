#!/bin/bash
# A/B: kernels with / without SLP vectorisation (gpuab/slp = SLP on), traversal versions 4 / 5
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/abslp"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "not fullsize" > "$OUT/tests.log" 2>&1 || { echo TESTFAIL; tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
for rep in 1 2; do for lib in noslp slp; do for v in 4 5; do
  if [ $lib = slp ]; then export LH2_CORE_LIB="$ROOT/gpuab/slp/libRenderCore_MI355X.so"; else unset LH2_CORE_LIB; fi
  timeout -k 10 120 python3 tools/trace_kernel_bench.py --set bounce --iters 20 --setting traceVersion=$v > "$OUT/tkb_${lib}_$v.log" 2>&1 || exit 1
  echo "$lib v$v $(tail -1 "$OUT/tkb_${lib}_$v.log" | cut -c1-80)"
done; done; done
unset LH2_CORE_LIB
for lib in noslp slp; do for v in 4 5; do
  if [ $lib = slp ]; then export LH2_CORE_LIB="$ROOT/gpuab/slp/libRenderCore_MI355X.so"; else unset LH2_CORE_LIB; fi
  timeout -k 10 300 python3 tools/bench_configs.py --configs 3,5 --frames 5 --setting traceVersion=$v > "$OUT/configs_${lib}_v$v.jsonl" 2>"$OUT/configs_${lib}_v$v.log" || exit 1
  python3 -c "
import json
for l in open('$OUT/configs_${lib}_v$v.jsonl'):
    d=json.loads(l); print('$lib v$v', d['config'], d['ms_per_frame'], d['Mrays_s'], 'shade', d['shadeTime_ms'], 'shadow', d['shadowTraceTime_ms'])"
done; done
unset LH2_CORE_LIB
for v in 4 5; do timeout -k 10 200 python3 bench.py --steps 20 --no-cpu-baseline --no-config4 --setting traceVersion=$v > "$OUT/bench_$v.json" 2> "$OUT/bench_$v.log" || { tail -20 "$OUT/bench_$v.log"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_$v.json'));print('bench v$v',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['detail']['traceTime0_ms'],d['detail']['traceTime1_ms'],d['detail']['shadeTime_ms'])"; done
timeout -k 10 300 python3 bench.py > "$OUT/bench_full.json" 2> "$OUT/bench_full.log" || { tail -20 "$OUT/bench_full.log"; exit 1; }
cat "$OUT/bench_full.json"
