#!/bin/bash
# config-4 rank shares at 1/2/4/8 ranks (tools/config4_shares.py) and the bounce-launch refill x leafBatch grid
# (tools/trace_kernel_bench.py --sweep) -> gpurun_out/$STEP/
set -euo pipefail
OUT="$GRAFT_REPO_ROOT/gpurun_out/${STEP:-shares}"
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
for r in 1 2 4 8; do
  timeout -k 10 240 python3 tools/config4_shares.py --ranks $r --frames 10 2>/dev/null | tail -1 >> "$OUT/shares.jsonl"
done
cat "$OUT/shares.jsonl"
timeout -k 10 400 python3 tools/trace_kernel_bench.py --set bounce --sweep --iters 30 > "$OUT/sweep.jsonl" 2>/dev/null
echo done
