#!/bin/bash
# Round-4 measurement batch (through gpurun from the repo root): GPU suite, bench.py, config-4 rank shares,
# the N=8 share's kernel timeline, config-5 builders.  STEPS selects parts (default all): t b s l c
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-r04}"
mkdir -p "$OUT"
cd "$ROOT"
STEPS="${STEPS:-tbslc}"
if [[ -n "${FIRST:-}" ]]; then
  timeout -k 10 120 python -u -m pytest tests -m gpu -x -q --timeout 100 --timeout-method thread -k "$FIRST" > "$OUT/gpu_first.log" 2>&1
  tail -1 "$OUT/gpu_first.log"
fi
if [[ "$STEPS" == *t* ]]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
  tail -1 "$OUT/gpu_tests.log"
fi
if [[ "$STEPS" == *b* ]]; then
  timeout -k 10 400 python3 bench.py --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.log"
  python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('bench',d['value'],d['ms_per_step'],{k:(d[k] or {}).get('ms_per_frame') for k in ('config2_restart','config3','config4','config4_incore','config5')}, (d['config5'] or {}).get('setup_s'))"
fi
if [[ "$STEPS" == *s* ]]; then
  timeout -k 10 300 python3 tools/config4_shares.py > "$OUT/shares.jsonl" 2> "$OUT/shares.err"
  cat "$OUT/shares.jsonl"
fi
if [[ "$STEPS" == *l* ]]; then
  TAGDIR="$OUT" bash tools/share_timeline.sh 8 > "$OUT/share8.txt" 2>&1
  tail -14 "$OUT/share8.txt"
fi
if [[ "$STEPS" == *c* ]]; then
  timeout -k 10 500 python3 tools/config5_builders.py --builders "${BUILDERS:-cpu_sbvh,cpu_sbvh_1e-5,cpu_sah,gpu_ploc}" > "$OUT/config5_builders.jsonl" 2> "$OUT/config5_builders.err"
  cat "$OUT/config5_builders.jsonl"
fi
echo "batch done"
