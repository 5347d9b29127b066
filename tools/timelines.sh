#!/bin/bash
# Kernel timelines (rocprofv3 --kernel-trace) of the config-4 N=8 rank share and of config-3 frames, each with the
# given settings, plus the config-5 builders and the gather cost (through gpurun).  usage: SETS="earlyShade=1 earlyShade=0"
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-tl}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for s in ${SETS:-none=0}; do
  n="${s//=/_}"
  timeout -k 10 200 rocprofv3 --kernel-trace -d "$OUT/s8_$n" -o run --output-format csv -- \
    python3 "$ROOT/tools/config4_shares.py" --ranks 8 --frames 10 --setting "$s" > "$OUT/s8_$n.jsonl" 2> "$OUT/s8_$n.err"
  python3 "$ROOT/tools/overlap_timeline.py" "$(find "$OUT/s8_$n" -name '*kernel_trace.csv' | head -1)" 2 > "$OUT/s8_$n.txt"
  timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/c3_$n" -o run --output-format csv -- \
    python3 "$ROOT/tools/bench_configs.py" --configs 3 --frames 10 --setting "$s" > "$OUT/c3_$n.jsonl" 2> "$OUT/c3_$n.err"
  python3 "$ROOT/tools/overlap_timeline.py" "$(find "$OUT/c3_$n" -name '*kernel_trace.csv' | head -1)" 2 > "$OUT/c3_$n.txt"
  echo "== $s"; cat "$OUT/s8_$n.jsonl" "$OUT/s8_$n.txt" "$OUT/c3_$n.jsonl" "$OUT/c3_$n.txt"
done
cd "$ROOT"
if [ "${EXTRA:-1}" != "0" ]; then
  timeout -k 10 200 python3 tools/gather_cost.py > "$OUT/gather_cost.json" 2> "$OUT/gather_cost.err"; cat "$OUT/gather_cost.json"
  timeout -k 10 500 python3 tools/config5_builders.py > "$OUT/config5_builders.jsonl" 2> "$OUT/config5_builders.err"; cat "$OUT/config5_builders.jsonl"
fi
echo "timelines done"
