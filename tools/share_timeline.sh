#!/bin/bash
# Kernel timeline of one rank's share of the config-4 frame (tools/config4_shares.py, rank 0's bands of N):
# rocprofv3 --kernel-trace of 10 frames -> gpurun_out/share<N>/, then tools/frame_timeline.py on the median
# frame.  usage (through gpurun): bash tools/share_timeline.sh [N] [extra config4_shares.py args]
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
N="${1:-8}"; shift || true
OUT="$ROOT/gpurun_out/share$N"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT" -o run --output-format csv -- \
  python3 "$ROOT/tools/config4_shares.py" --ranks "$N" --frames 10 "$@" > "$OUT/shares.jsonl" 2> "$OUT/shares.err"
python3 "$ROOT/tools/overlap_timeline.py" "$(find "$OUT" -name "*kernel_trace.csv" | head -1)" 3 > "$OUT/timeline.txt"
cat "$OUT/shares.jsonl" "$OUT/timeline.txt"
