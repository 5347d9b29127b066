#!/bin/bash
# BVH4 traversal tuning on the config-2 bounce rays: refill x leafBatch per leaf size.  -> gpurun_out/sw4/
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/sw4"; mkdir -p "$OUT"; cd "$ROOT"
for leaf in 1 2 4; do
  timeout -k 10 240 python3 tools/trace_kernel_bench.py --set bounce --sweep --iters 5 --pre-setting bvhMaxLeaf=$leaf --setting traceVersion=4 > "$OUT/leaf$leaf.jsonl" 2>>"$OUT/err.log" || exit 1
done
echo sw4 done
