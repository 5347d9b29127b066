#!/bin/bash
# Config-2 only A/B (bench.py, no other configs), variants interleaved, REPS rounds: VARIANTS="base name=value,..."
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-abc2}"
mkdir -p "$OUT"
cd "$ROOT"
for rep in $(seq 1 "${REPS:-3}"); do
  for v in ${VARIANTS:-base}; do
    args=()
    if [ "$v" != "base" ]; then IFS=',' read -ra kvs <<< "$v"; for kv in "${kvs[@]}"; do args+=(--setting "$kv"); done; fi
    n="${v//[=,]/_}_$rep"
    timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-configs --no-config4 "${args[@]}" > "$OUT/c2_$n.json" 2> "$OUT/c2_$n.err"
    python3 -c "import json,sys; d=json.load(open('$OUT/c2_$n.json')); print(f\"{sys.argv[1]:40s} c2 {d['ms_per_step']:.4f} {d['value']:.0f}\", flush=True)" "$v"
  done
done
echo "ab_c2 done"
