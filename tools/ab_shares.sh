#!/bin/bash
# N = 1 / N = 8 config-4 rank shares only (tools/config4_shares.py), variants interleaved, REPS rounds (through gpurun).
# usage: VARIANTS="base sideBlocks=4 sideBlocks=4,finalShadowBlocks=6" REPS=3 bash tools/ab_shares.sh
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-abs}"
mkdir -p "$OUT"
cd "$ROOT"
for rep in $(seq 1 "${REPS:-3}"); do
  for v in ${VARIANTS:-base}; do
    args=()
    if [ "$v" != "base" ]; then IFS=',' read -ra kvs <<< "$v"; for kv in "${kvs[@]}"; do args+=(--setting "$kv"); done; fi
    n="${v//[=,]/_}_$rep"
    timeout -k 10 200 python3 tools/config4_shares.py --ranks "${RANKS:-1,8}" "${args[@]}" > "$OUT/sh_$n.jsonl" 2> "$OUT/sh_$n.err"
    python3 - "$OUT/sh_$n.jsonl" "$v" <<'PY'
import json, sys
sh = [json.loads(l) for l in open(sys.argv[1]) if l.strip()]
print(f"{sys.argv[2]:40s} " + " ".join(f"N{s['ranks']} {s['ms_per_frame']:.4f}" for s in sh) + f" ratio {sh[0]['ms_per_frame'] / sh[-1]['ms_per_frame']:.3f}", flush=True)
PY
  done
done
echo "ab_shares done"
