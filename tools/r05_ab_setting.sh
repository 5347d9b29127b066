#!/bin/bash
# Round 5 A/B of one core setting on frames (through gpurun from the repo root): optional GPU tests first (TESTS="<pytest
# args>"), then bench.py (configs 2, 2-restart, 3) + the config-4 shares N = 1, 8, alternating the values, R rounds.
# usage: bash tools/r05_ab_setting.sh NAME "v1 v2 ..." [R]
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
NAME="$1"; VALS="$2"; R="${3:-2}"
OUT="$ROOT/gpurun_out/ab_$NAME"
mkdir -p "$OUT"
cd "$ROOT"
export LH2_BLUENOISE="$ROOT/lighthouse2_amd/data/bluenoise.bin"
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
  tail -1 "$OUT/gpu_tests.log"
fi
for r in $(seq 1 "$R"); do
  for v in $VALS; do
    n="${v}_$r"
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-config5 --no-config4 --setting "$NAME=$v" > "$OUT/bench_$n.json" 2> "$OUT/bench_$n.log"
    timeout -k 10 200 python3 tools/config4_shares.py --ranks 1,8 --setting "$NAME=$v" > "$OUT/shares_$n.jsonl" 2> "$OUT/shares_$n.err"
    python3 - "$OUT/bench_$n.json" "$OUT/shares_$n.jsonl" "$NAME=$n" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
sh = [json.loads(l) for l in open(sys.argv[2]) if l.strip()]
g = lambda k: (d.get(k) or {}).get("ms_per_frame")
c3 = d["config3"]["coreStats_ms"]
print(sys.argv[3], "c2", d["value"], d["ms_per_step"], "| c2r", g("config2_restart"), "| c3", g("config3"), c3, "| shares", [s["ms_per_frame"] for s in sh],
      "ratio", round(sh[0]["ms_per_frame"] / sh[-1]["ms_per_frame"], 3), flush=True)
PY
  done
done
echo "ab $NAME done"
