#!/bin/bash
# Round-5 W8 evaluation (through gpurun from the repo root): the GPU suite, the unit bounce launch (tools/trace_kernel_bench.py
# --set bounce: bench.py's roofline kernel) on the BVH4 and on the W8 and with the W8 variant libraries under gpuab/ (when
# built), then bench.py (configs 2, 2-restart, 3, 4) and the config-4 rank shares at N = 1 and 8 alternating traceWide, then
# shadowOccluders (tools/ab_setting.sh).  Every GPU step has its own time limit; a failing step ends the batch.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/w8eval"
mkdir -p "$OUT"
cd "$ROOT"
if [ "${TESTS:-1}" != "0" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
  tail -1 "$OUT/gpu_tests.log"
fi
export LH2_BLUENOISE="$ROOT/lighthouse2_amd/data/bluenoise.bin"   # the variant libraries under gpuab/ have no data/ beside them
for rep in 1 2; do
  for w in 0 1; do
    timeout -k 10 200 python3 tools/trace_kernel_bench.py --set bounce --iters 20 --setting "traceWide=$w" > "$OUT/kb_${w}_$rep.txt" 2>&1
    echo "traceWide=$w $(tail -1 "$OUT/kb_${w}_$rep.txt" | cut -c1-200)"
  done
  for lib in $(ls gpuab 2>/dev/null); do
    LH2_CORE_LIB="$ROOT/gpuab/$lib/libRenderCore_MI355X.so" timeout -k 10 200 python3 tools/trace_kernel_bench.py --set bounce --iters 20 --setting traceWide=1 > "$OUT/kb_${lib}_$rep.txt" 2>&1
    echo "$lib $(tail -1 "$OUT/kb_${lib}_$rep.txt" | cut -c1-200)"
  done
done
if [ -d gpuab/stats ]; then
  LH2_CORE_LIB="$ROOT/gpuab/stats/libRenderCore_MI355X.so" timeout -k 10 200 python3 tools/trace_kernel_bench.py --set bounce --iters 2 --setting traceWide=0 > "$OUT/kb_stats_w0.txt" 2>&1
  grep LH2_TRACE_STATS "$OUT/kb_stats_w0.txt" | tail -1
fi
SETTING=traceWide VALUES="0 1" REPS="${REPS:-2}" TAG=w8eval/ab bash tools/ab_setting.sh
SETTING=shadowOccluders VALUES="1 0" REPS=1 TAG=w8eval/occ bash tools/ab_setting.sh
echo "w8 eval done"
