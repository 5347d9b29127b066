#!/bin/bash
# Round 6: config 5 A/B over (library, setting) pairs, REPS interleaved rounds (through gpurun).
# usage: bash tools/r06_c5ab.sh new:traceWaves=0 einst:traceWaves=7 ...   (new = the in-tree library, else gpuab/<name>/)
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-r06c5ab}"
mkdir -p "$OUT"
cd "$ROOT"
export LH2_BLUENOISE="$ROOT/lighthouse2_amd/data/bluenoise.bin"
for r in $(seq 1 "${REPS:-2}"); do
  for v in "$@"; do
    lib="${v%%:*}"; set_="${v#*:}"
    if [ "$lib" = new ]; then unset LH2_CORE_LIB; else export LH2_CORE_LIB="$ROOT/gpuab/$lib/libRenderCore_MI355X.so"; fi
    n="${v//[:=,]/_}_$r"
    timeout -k 10 300 python3 tools/bench_configs.py --configs ${CONFIGS:-5} --setting "$set_" > "$OUT/c_$n.json" 2> "$OUT/c_$n.err"
    python3 - "$OUT/c_$n.json" "$v r$r" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l)
        print(f"{sys.argv[2]:32s}", d["config"], d["ms_per_frame"], "trace0", d["traceTime0_ms"], "trace1", d["traceTime1_ms"], "shade", d["shadeTime_ms"], flush=True)
PY
  done
done
echo "r06 c5ab done"
