#!/bin/bash
# Round-5 W8 / occluder-sharing evaluation, second pass (through gpurun from the repo root):
#   unit bounce launches (tools/trace_kernel_bench.py --set bounce) on config 2 and on the room: BVH4 (traceWide 0), the in-tree W8,
#   and the W8 variant library gpuab/w8l1only; then frames (bench.py configs 2, 2-restart, 3, 4 + config-4 shares N = 1, 8) for
#   traceWide 0 / 1 and, at traceWide 0, shadowOccluders 0 / 1 and the occluder variants gpuab/occR (previous occluder only),
#   gpuab/occB (broadcast only).  Every GPU step has its own time limit; a failing step ends the batch.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/w8eval2"
mkdir -p "$OUT"
cd "$ROOT"
export LH2_BLUENOISE="$ROOT/lighthouse2_amd/data/bluenoise.bin"
kb() {   # name, lib ("" in-tree), scene, tris, settings...
  local name="$1" lib="$2" sc="$3" tris="$4"; shift 4
  local args=(); for s in "$@"; do args+=(--setting "$s"); done
  if [ -n "$lib" ]; then export LH2_CORE_LIB="$ROOT/gpuab/$lib/libRenderCore_MI355X.so"; else unset LH2_CORE_LIB; fi
  timeout -k 10 300 python3 tools/trace_kernel_bench.py --set bounce --iters 20 --scene "$sc" --tris "$tris" "${args[@]}" > "$OUT/kb_${name}.txt" 2>&1
  unset LH2_CORE_LIB
  echo "$name $(tail -1 "$OUT/kb_${name}.txt" | cut -c1-120)"
}
frames() {   # name, lib, settings...
  local name="$1" lib="$2"; shift 2
  local args=(); for s in "$@"; do args+=(--setting "$s"); done
  if [ -n "$lib" ]; then export LH2_CORE_LIB="$ROOT/gpuab/$lib/libRenderCore_MI355X.so"; else unset LH2_CORE_LIB; fi
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-config5 --no-config4 "${args[@]}" > "$OUT/bench_$name.json" 2> "$OUT/bench_$name.log"
  timeout -k 10 200 python3 tools/config4_shares.py --ranks 1,8 "${args[@]}" > "$OUT/shares_$name.jsonl" 2> "$OUT/shares_$name.err"
  unset LH2_CORE_LIB
  python3 - "$OUT/bench_$name.json" "$OUT/shares_$name.jsonl" "$name" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
sh = [json.loads(l) for l in open(sys.argv[2]) if l.strip()]
g = lambda k: (d.get(k) or {}).get("ms_per_frame")
c3 = d["config3"]["coreStats_ms"]
print(sys.argv[3], "c2", d["value"], d["ms_per_step"], "| c2r", g("config2_restart"), "| c3", g("config3"), c3, "| c4", (sh[0] if sh else {}).get("ms_per_frame"),
      "| shares", [s["ms_per_frame"] for s in sh], "ratio", round(sh[0]["ms_per_frame"] / sh[-1]["ms_per_frame"], 3), flush=True)
PY
}
kb c2_bvh4 "" config2 100000 traceWide=0
kb c2_w8 "" config2 100000 traceWide=1
kb c2_w8l1only w8l1only config2 100000 traceWide=1
kb room_bvh4 "" room 1000000 traceWide=0
kb room_w8 "" room 1000000 traceWide=1
frames w0 "" traceWide=0
frames w1 "" traceWide=1
frames occ0 "" traceWide=0 shadowOccluders=0
frames occR "occR" traceWide=0 shadowOccluders=1
frames occB "occB" traceWide=0 shadowOccluders=1
echo "w8 eval2 done"
