#!/bin/bash
# A/B of the in-tree core library ("new") against variant builds gpuab/<name>/libRenderCore_MI355X.so:
# parity subset on the new library, then kernel times (trace_kernel_bench, both ray sets) alternating
# between the libraries, then bench.py.  usage (through gpurun): bash tools/ab_libs.sh name...
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/ab"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1 || { echo TESTFAIL; tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
for rep in 1 2 3; do for lib in new "$@"; do
  if [ "$lib" = new ]; then unset LH2_CORE_LIB; else export LH2_CORE_LIB="$ROOT/gpuab/$lib/libRenderCore_MI355X.so"; fi
  timeout -k 10 120 python3 tools/trace_kernel_bench.py --set both --iters 20 ${TKB_ARGS:-} > "$OUT/$lib.log" 2>&1 || exit 1
  echo "$lib $(tail -1 "$OUT/$lib.log" | cut -c1-160)"
done; done
unset LH2_CORE_LIB
timeout -k 10 200 python3 bench.py --steps 20 --no-cpu-baseline --no-config4 > "$OUT/bench.json" 2> "$OUT/bench.log" || exit 1
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('bench',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['roofline']['frac'],d['detail']['traceTime0_ms'],d['detail']['traceTime1_ms'],d['detail']['shadeTime_ms'])"
