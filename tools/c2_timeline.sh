#!/bin/bash
# Kernel timeline of config-2 frames (the bench line's workload): rocprofv3 --kernel-trace of bench.py with configs 3 / 4 / 5
# and the CPU baseline off -> gpurun_out/c2tl/, then tools/overlap_timeline.py on three frames from the middle of the run
# (through gpurun from the repo root).
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/c2tl"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --no-cpu-baseline --no-configs --no-config4 --steps 40 --kernel-iters 2 > "$OUT/bench.json" 2> "$OUT/bench.err"
python3 "$ROOT/tools/overlap_timeline.py" "$(find "$OUT" -name "*kernel_trace.csv" | head -1)" 3 > "$OUT/timeline.txt"
cat "$OUT/timeline.txt"
