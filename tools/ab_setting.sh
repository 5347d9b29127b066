#!/bin/bash
# A/B of one core setting (through gpurun): bench.py (config 2, config2_restart, 3, 4, 4 in-core; no config 5, no CPU
# baseline) and the config-4 rank shares at N = 1 and 8, alternating the values.  usage: SETTING=name VALUES="1 0" REPS=2
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-ab}"
mkdir -p "$OUT"
cd "$ROOT"
for rep in $(seq 1 "${REPS:-2}"); do
  for v in ${VALUES:-1 0}; do
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-config5 --setting "$SETTING=$v" > "$OUT/bench_${v}_$rep.json" 2> "$OUT/bench_${v}_$rep.log"
    timeout -k 10 200 python3 tools/config4_shares.py --ranks 1,8 --setting "$SETTING=$v" > "$OUT/shares_${v}_$rep.jsonl" 2> "$OUT/shares_${v}_$rep.err"
    python3 - "$OUT/bench_${v}_$rep.json" "$OUT/shares_${v}_$rep.jsonl" "$SETTING=$v" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
sh = [json.loads(l) for l in open(sys.argv[2]) if l.strip()]
g = lambda k: (d.get(k) or {}).get("ms_per_frame")
print(sys.argv[3], "c2", d["value"], d["ms_per_step"], "| c2r", g("config2_restart"), "| c3", g("config3"), "| c4", g("config4"),
      "| shares", [s["ms_per_frame"] for s in sh], "ratio", round(sh[0]["ms_per_frame"] / sh[-1]["ms_per_frame"], 3), flush=True)
PY
  done
done
echo "ab done"
