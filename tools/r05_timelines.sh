#!/bin/bash
# Round 5 (through gpurun from the repo root): the N = 8 rank share's per-launch kernel timelines with the W8 loop
# (traceWide 1) and the BVH4 loop (0), rocprofv3 --kernel-trace (tools/share_timeline.sh), and the config-4 shares
# N = 1, 2, 4, 8 at the defaults.  Every GPU step has its own time limit; a failing step ends the batch.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/tl5"
mkdir -p "$OUT"
cd "$ROOT"
for w in 0 1; do
  bash tools/share_timeline.sh 8 --setting traceWide=$w > "$OUT/share8_w$w.txt" 2>&1
  cp "$ROOT/gpurun_out/share8/timeline.txt" "$OUT/timeline_w$w.txt"
  rm -rf "$ROOT/gpurun_out/share8"
  head -3 "$OUT/share8_w$w.txt"
done
cd "$ROOT"
timeout -k 10 300 python3 tools/config4_shares.py > "$OUT/config4_shares.jsonl" 2> "$OUT/config4_shares.err"
cat "$OUT/config4_shares.jsonl"
echo "timelines done"
