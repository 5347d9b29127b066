#!/bin/bash
# GPU suite with a forced traversal version, then the closest-hit microbenchmark for versions 2 and 4.
# usage (on the GPU box): bash tools/ab_trace_version.sh   -> gpurun_out/tv/
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/tv"; mkdir -p "$OUT"; cd "$ROOT"
LH2_TRACE_VERSION=4 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests_v4.log" 2>&1 || exit 1
for rep in 1 2; do
  for v in 2 4; do
    timeout -k 10 120 python3 tools/trace_kernel_bench.py --set both --setting traceVersion=$v > "$OUT/kb_v${v}_$rep.json" 2>>"$OUT/err.log" || exit 1
  done
done
echo tv done
