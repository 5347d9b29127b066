#!/bin/bash
# Round 5: the GPU suite at the new defaults, then the launch drain of the bounce closest-hit launch (through gpurun from the
# repo root): per-wave start / queue-dry / end times (gpuab/tt: -DLH2_TRACE_TIMES), and the unit bounce launch with a
# 15-entry LDS stack (gpuab/st15) against the in-tree 16, alternating.  Every GPU step has its own time limit; a failing
# step ends the batch.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/drain"
mkdir -p "$OUT"
cd "$ROOT"
if [ "${TESTS:-1}" != "0" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
  tail -1 "$OUT/gpu_tests.log"
fi
export LH2_BLUENOISE="$ROOT/lighthouse2_amd/data/bluenoise.bin"
kb() {   # name, lib ("" in-tree), scene, tris, extra args...
  local name="$1" lib="$2" sc="$3" tris="$4"; shift 4
  if [ -n "$lib" ]; then export LH2_CORE_LIB="$ROOT/gpuab/$lib/libRenderCore_MI355X.so"; else unset LH2_CORE_LIB; fi
  timeout -k 10 300 python3 tools/trace_kernel_bench.py --set bounce --iters 20 --scene "$sc" --tris "$tris" "$@" > "$OUT/kb_${name}.txt" 2>&1
  unset LH2_CORE_LIB
  echo "$name $(grep '^{' "$OUT/kb_${name}.txt" | tail -1 | cut -c1-100)"
}
for s in config2:100000 room:1000000; do
  sc="${s%%:*}"; n="${s#*:}"
  LH2_CORE_LIB="$ROOT/gpuab/tt/libRenderCore_MI355X.so" LH2_TRACE_TIMES_OUT="$OUT/tt_$sc.bin" timeout -k 10 300 \
    python3 tools/trace_kernel_bench.py --set bounce --iters 3 --scene "$sc" --tris "$n" > "$OUT/tt_$sc.json" 2>&1
  python3 tools/trace_times.py "$OUT/tt_$sc.bin" > "$OUT/tt_$sc.txt"
  echo "== $sc"; cat "$OUT/tt_$sc.txt"
done
for r in 1 2; do
  kb "c2_16_$r" "" config2 100000
  kb "c2_15_$r" st15 config2 100000
  kb "room_16_$r" "" room 1000000
  kb "room_15_$r" st15 room 1000000
done
echo "drain batch done"
