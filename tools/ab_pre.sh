#!/bin/bash
# kernel-time A/B of BVH build settings: each argument is one configuration, a comma-separated list
# of name=value settings applied before the scene is loaded ("" = defaults); TESTS=1 first runs
# the parity tests selected by TESTK.  -> gpurun_out/abpre/
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/abpre"
mkdir -p "$OUT"
cd "$ROOT"
if [ -n "${TESTK:-}" ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "$TESTK" > "$OUT/tests.log" 2>&1 || { echo TESTFAIL; tail -30 "$OUT/tests.log"; exit 1; }
  tail -1 "$OUT/tests.log"
fi
for rep in 1 2; do
  i=0
  for cfg in "$@"; do
    args=(); IFS=',' read -ra kvs <<< "$cfg"; for kv in "${kvs[@]}"; do [ -n "$kv" ] && args+=(--pre-setting "$kv"); done
    timeout -k 10 150 python3 tools/trace_kernel_bench.py --set both --iters 20 ${TKB_TRIS:+--tris $TKB_TRIS} "${args[@]}" > "$OUT/c$i.log" 2>&1 || exit 1
    python3 - "$OUT/c$i.log" "$cfg" <<'PY'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
d = json.loads(line)
print(f"{sys.argv[2]:60s} primary {d['primary']['ms']:.4f} bounce {d['bounce']['ms']:.4f}")
PY
    i=$((i+1))
  done
done
