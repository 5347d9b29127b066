#!/bin/bash
# Round 6: register-pressure variants of the BVH4 loops (gpuab/v1: barycentrics packed at each closer hit; v2: + the padded
# closest distance recomputed where used; v3: + the node's reference load issued in the node step, not with the early
# loads), through gpurun: the bounce kernel alone at 7 and 8 waves per SIMD, then frames (tools/r06_ablib.sh).
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/r06regs"
mkdir -p "$OUT"
cd "$ROOT"
export LH2_BLUENOISE="$ROOT/lighthouse2_amd/data/bluenoise.bin"
for rep in 1 2; do for lib in new v1 v2 v3; do for w in 7 8; do
  if [ "$lib" = new ]; then unset LH2_CORE_LIB; else export LH2_CORE_LIB="$ROOT/gpuab/$lib/libRenderCore_MI355X.so"; fi
  b=$(timeout -k 10 180 python3 tools/trace_kernel_bench.py --set bounce --iters 100 --setting unitTraceWaves=$w 2>/dev/null | tail -1)
  echo "$lib w$w $(echo "$b" | python3 -c "import json,sys;d=json.load(sys.stdin)['bounce'];print(d['ms'],d['Mrays_s'])")"
done; done; done | tee "$OUT/kernel.txt"
unset LH2_CORE_LIB
TAG=r06regs REPS=2 bash tools/r06_ablib.sh ${FRAMES:-v1 v3 v3:traceWaves=8 v2:traceWaves=8}
