#!/bin/bash
# rocprofv3 kernel statistics of config-3 frames (lit room, depth 4)
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/c3prof"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/stats" -o run -- python3 "$ROOT/tools/bench_configs.py" --configs 3 --frames 10 > "$OUT/c3.jsonl" 2> "$OUT/c3.log" || exit 1
cat "$OUT/c3.jsonl"
head -20 "$OUT/stats/run_kernel_stats.csv" | cut -d, -f1-4
