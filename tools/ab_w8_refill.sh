#!/bin/bash
# v6 bounce launch: 7 vs 8 waves/SIMD (gpuab/w8, blocksPerCU 8), refill threshold sweep
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/w8"
mkdir -p "$OUT"
cd "$ROOT"
for rep in 1 2; do
  timeout -k 10 120 python3 tools/trace_kernel_bench.py --set bounce --iters 20 > "$OUT/base.log" 2>&1 || exit 1; echo "w7 $(tail -1 "$OUT/base.log" | cut -c1-80)"
  LH2_CORE_LIB="$ROOT/gpuab/w8/libRenderCore_MI355X.so" timeout -k 10 120 python3 tools/trace_kernel_bench.py --set bounce --iters 20 --setting blocksPerCU=8 > "$OUT/w8.log" 2>&1 || exit 1; echo "w8 $(tail -1 "$OUT/w8.log" | cut -c1-80)"
  LH2_CORE_LIB="$ROOT/gpuab/w8/libRenderCore_MI355X.so" timeout -k 10 120 python3 tools/trace_kernel_bench.py --set bounce --iters 20 --setting blocksPerCU=7 > "$OUT/w8b7.log" 2>&1 || exit 1; echo "w8lib_b7 $(tail -1 "$OUT/w8b7.log" | cut -c1-80)"
done
for r in 24 32 40 48 56; do
  timeout -k 10 120 python3 tools/trace_kernel_bench.py --set bounce --iters 20 --refill $r > "$OUT/r$r.log" 2>&1 || exit 1; echo "refill $r $(tail -1 "$OUT/r$r.log" | cut -c1-80)"
done
