#!/bin/bash
# refill threshold sweep of the bounce-ray launch for traceVersion 4 and 5
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p "$ROOT/gpurun_out/refill"
for v in 4 5; do for r in ${REFILLS:-8 16 24 32 40 48 56}; do
  timeout -k 10 120 python3 "$ROOT/tools/trace_kernel_bench.py" --set bounce --iters 20 --setting traceVersion=$v --refill $r > "$ROOT/gpurun_out/refill/v${v}_r$r.log" 2>&1 || exit 1
  echo "v$v refill $r $(tail -1 "$ROOT/gpurun_out/refill/v${v}_r$r.log")"
done; done
