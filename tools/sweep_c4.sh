#!/bin/bash
# Settings A/B on config 4's per-rank share (tools/config4_shares.py, RANKS default 8), two interleaved rounds.
# usage: RANKS=8 bash tools/sweep_c4.sh "name=value,..." ...   ("" = defaults)  -> gpurun_out/sweep_c4.jsonl
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p "$ROOT/gpurun_out"; cd "$ROOT"
for rep in 1 2; do
  for cfg in "$@"; do
    args=(); IFS=',' read -ra kvs <<< "$cfg"; for kv in "${kvs[@]}"; do [ -n "$kv" ] && args+=(--setting "$kv"); done
    r=$(timeout -k 10 120 python3 tools/config4_shares.py --ranks ${RANKS:-8} --frames 10 "${args[@]}" 2>>"$ROOT/gpurun_out/sweep_c4.err") || exit 1
    while read -r l; do echo "{\"cfg\": \"$cfg\", \"rep\": $rep, \"res\": $l}" >> "$ROOT/gpurun_out/sweep_c4.jsonl"; done <<< "$r"
    echo "$cfg rep $rep done"
  done
done
