#!/bin/bash
# Round 5: the drain merge (LH2_DRAIN_MERGE, gpuab/mg: with a 15-entry LDS stack) through gpurun from the repo root: the GPU
# suite on the variant library, per-wave drain times (gpuab/mgtt), the unit bounce launch (in-tree / st15 / mg, alternating)
# and frames (bench.py configs 2, 3 + config-4 shares N = 1, 8) in-tree vs mg.  Every GPU step has its own time limit; a
# failing step ends the batch.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/merge"
mkdir -p "$OUT"
cd "$ROOT"
export LH2_BLUENOISE="$ROOT/lighthouse2_amd/data/bluenoise.bin"
if [ "${TESTS:-1}" != "0" ]; then
  LH2_CORE_LIB="$ROOT/gpuab/mg/libRenderCore_MI355X.so" timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests_mg.log" 2>&1 || true
  tail -1 "$OUT/gpu_tests_mg.log"
  grep -E "FAILED|ERROR" "$OUT/gpu_tests_mg.log" | head -20 || true
  if ! tail -1 "$OUT/gpu_tests_mg.log" | grep -q " passed"; then echo "suite did not finish"; exit 1; fi
fi
kb() {   # name, lib ("" in-tree), scene, tris
  local name="$1" lib="$2" sc="$3" tris="$4"; shift 4
  if [ -n "$lib" ]; then export LH2_CORE_LIB="$ROOT/gpuab/$lib/libRenderCore_MI355X.so"; else unset LH2_CORE_LIB; fi
  timeout -k 10 300 python3 tools/trace_kernel_bench.py --set bounce --iters 20 --scene "$sc" --tris "$tris" "$@" > "$OUT/kb_${name}.txt" 2>&1
  unset LH2_CORE_LIB
  echo "$name $(grep '^{' "$OUT/kb_${name}.txt" | tail -1 | cut -c1-100)"
}
for s in config2:100000 room:1000000; do
  sc="${s%%:*}"; n="${s#*:}"
  LH2_CORE_LIB="$ROOT/gpuab/mgtt/libRenderCore_MI355X.so" LH2_TRACE_TIMES_OUT="$OUT/tt_mg_$sc.bin" timeout -k 10 300 \
    python3 tools/trace_kernel_bench.py --set bounce --iters 3 --scene "$sc" --tris "$n" > "$OUT/tt_mg_$sc.json" 2>&1
  python3 tools/trace_times.py "$OUT/tt_mg_$sc.bin" > "$OUT/tt_mg_$sc.txt"
  echo "== merge $sc"; cat "$OUT/tt_mg_$sc.txt"
done
for r in 1 2; do
  kb "c2_16_$r" "" config2 100000
  kb "c2_mg_$r" mg config2 100000
  kb "room_16_$r" "" room 1000000
  kb "room_mg_$r" mg room 1000000
done
frames() {   # name, lib
  local name="$1" lib="$2"
  if [ -n "$lib" ]; then export LH2_CORE_LIB="$ROOT/gpuab/$lib/libRenderCore_MI355X.so"; else unset LH2_CORE_LIB; fi
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-config5 --no-config4 > "$OUT/bench_$name.json" 2> "$OUT/bench_$name.log"
  timeout -k 10 200 python3 tools/config4_shares.py --ranks 1,8 > "$OUT/shares_$name.jsonl" 2> "$OUT/shares_$name.err"
  unset LH2_CORE_LIB
  python3 - "$OUT/bench_$name.json" "$OUT/shares_$name.jsonl" "$name" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
sh = [json.loads(l) for l in open(sys.argv[2]) if l.strip()]
g = lambda k: (d.get(k) or {}).get("ms_per_frame")
c3 = d["config3"]["coreStats_ms"]
print(sys.argv[3], "c2", d["value"], d["ms_per_step"], "| c2r", g("config2_restart"), "| c3", g("config3"), c3, "| shares", [s["ms_per_frame"] for s in sh],
      "ratio", round(sh[0]["ms_per_frame"] / sh[-1]["ms_per_frame"], 3), flush=True)
PY
}
frames base_1 ""
frames mg_1 mg
frames base_2 ""
frames mg_2 mg
echo "merge batch done"
