#!/bin/bash
# Round 6: config 5 with packet primaries (setting packetPrimary 1: the fused camera + packet launch and its frame overlap)
# against the per-ray primaries (the default for a scene beyond the Infinity Cache), two interleaved rounds (through gpurun).
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/r06c5pk"
mkdir -p "$OUT"
cd "$ROOT"
export LH2_BLUENOISE="$ROOT/lighthouse2_amd/data/bluenoise.bin"
for r in 1 2; do
  for v in ${VALUES:--1 1}; do
    timeout -k 10 300 python3 tools/bench_configs.py --configs 5 --setting packetPrimary=$v ${EXTRA_SET:+--setting $EXTRA_SET} > "$OUT/c5_${v}_$r.json" 2> "$OUT/c5_${v}_$r.err"
    python3 - "$OUT/c5_${v}_$r.json" "packetPrimary=$v r$r" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l)
        print(sys.argv[2], d["config"], d["ms_per_frame"], "trace0", d["traceTime0_ms"], "trace1", d["traceTime1_ms"], "shade", d["shadeTime_ms"], flush=True)
PY
  done
done
echo "r06 c5pk done"
