#!/bin/bash
# Round-5 W8 evaluation (through gpurun from the repo root): the GPU suite, the unit bounce launch (tools/trace_kernel_bench.py
# --set bounce: bench.py's roofline kernel) on the BVH4 and on the W8, then bench.py (configs 2, 2-restart, 3, 4) and the config-4
# rank shares at N = 1 and 8 alternating traceWide (tools/ab_setting.sh).  Every GPU step has its own time limit; chained.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/w8eval"
mkdir -p "$OUT"
cd "$ROOT"
if [ "${TESTS:-1}" != "0" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
  tail -1 "$OUT/gpu_tests.log"
fi
for w in ${KB_VALUES:-0 1}; do
  timeout -k 10 200 python3 tools/trace_kernel_bench.py --set bounce --iters 20 --setting "traceWide=$w" > "$OUT/kb_$w.txt" 2>&1
  tail -3 "$OUT/kb_$w.txt"
done
SETTING="${SETTING:-traceWide}" VALUES="${VALUES:-0 1}" REPS="${REPS:-2}" TAG=w8eval/ab bash tools/ab_setting.sh
echo "w8 eval done"
