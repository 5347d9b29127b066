#!/bin/bash
# Tail hand-off threshold: GPU suite, closest-hit microbenchmark and frame per tailLanes.  -> gpurun_out/tail/
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/tail"; mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || exit 1
for t in 0 8 16 24 32 48; do
  timeout -k 10 120 python3 tools/trace_kernel_bench.py --set bounce --setting tailLanes=$t > "$OUT/kb_$t.json" 2>>"$OUT/err.log" || exit 1
  timeout -k 10 180 python3 bench.py --no-cpu-baseline --setting tailLanes=$t 2>>"$OUT/err.log" | tail -1 > "$OUT/bench_$t.json" || exit 1
done
echo tail done
