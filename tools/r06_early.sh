#!/bin/bash
# Round 6: the early node loads of lanes without a node, out of bounds (LH2_EARLY_OOB 1, in-tree "new") against node 0's
# record (gpuab/early0), through gpurun: the LH2_TRACE_STATS build's iteration counts (gpuab/stats), the bounce kernel
# alone (tools/ab_kernel_libs.sh) and frames (tools/r06_ablib.sh).
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/r06early"
mkdir -p "$OUT"
cd "$ROOT"
export LH2_BLUENOISE="$ROOT/lighthouse2_amd/data/bluenoise.bin"
LH2_CORE_LIB="$ROOT/gpuab/stats/libRenderCore_MI355X.so" timeout -k 10 120 python3 tools/trace_kernel_bench.py --set bounce --iters 1 > "$OUT/stats.json" 2> "$OUT/stats.err"
grep "LH2_TRACE_STATS" "$OUT/stats.err"
bash tools/ab_kernel_libs.sh early0 | tee "$OUT/kernel.txt"
TAG=r06early REPS=2 bash tools/r06_ablib.sh early0
