#!/bin/bash
# Round 5 A/B of the in-tree library ("new") against variant builds gpuab/<name>/libRenderCore_MI355X.so (through gpurun from
# the repo root): the unit bounce launch on config 2 and the room, then frames (bench.py configs 2, 2-restart, 3) and the
# config-4 shares N = 1, 8, alternating, R rounds.  Optional GPU tests first (TESTS="<pytest args>").
# usage: bash tools/r05_ab_libs.sh TAG R name...
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
TAG="$1"; R="$2"; shift 2
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
export LH2_BLUENOISE="$ROOT/lighthouse2_amd/data/bluenoise.bin"
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
  tail -1 "$OUT/gpu_tests.log"
fi
uselib() { if [ "$1" = new ]; then unset LH2_CORE_LIB; else export LH2_CORE_LIB="$ROOT/gpuab/$1/libRenderCore_MI355X.so"; fi; }
for r in $(seq 1 "$R"); do
  for lib in new "$@"; do
    uselib "$lib"
    for s in config2:100000 room:1000000; do
      sc="${s%%:*}"; n="${s#*:}"
      timeout -k 10 300 python3 tools/trace_kernel_bench.py --set bounce --iters 50 --scene "$sc" --tris "$n" > "$OUT/kb_${lib}_${sc}_$r.txt" 2>&1
      echo "$lib kb $sc $(grep '^{' "$OUT/kb_${lib}_${sc}_$r.txt" | tail -1 | cut -c1-70)"
    done
  done
done
for r in $(seq 1 "$R"); do
  for lib in new "$@"; do
    uselib "$lib"
    n="${lib}_$r"
    # C5=1: config 5 too (the instanced loops; ~10 s more per bench)
    timeout -k 10 300 python3 bench.py --no-cpu-baseline $([ -n "${C5:-}" ] || echo --no-config5) --no-config4 > "$OUT/bench_$n.json" 2> "$OUT/bench_$n.log"
    timeout -k 10 200 python3 tools/config4_shares.py --ranks 1,8 > "$OUT/shares_$n.jsonl" 2> "$OUT/shares_$n.err"
    python3 - "$OUT/bench_$n.json" "$OUT/shares_$n.jsonl" "$n" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
sh = [json.loads(l) for l in open(sys.argv[2]) if l.strip()]
g = lambda k: (d.get(k) or {}).get("ms_per_frame")
c3 = d["config3"]["coreStats_ms"]
print(sys.argv[3], "c2", d["value"], d["ms_per_step"], "| c2r", g("config2_restart"), "| c3", g("config3"), c3, "| c5", g("config5"), "| shares", [s["ms_per_frame"] for s in sh],
      "ratio", round(sh[0]["ms_per_frame"] / sh[-1]["ms_per_frame"], 3), flush=True)
PY
  done
done
unset LH2_CORE_LIB
echo "ab libs $TAG done"
