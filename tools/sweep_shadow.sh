#!/bin/bash
# Shadow-launch settings on config 3 (tools/bench_configs.py, 6 frames), two interleaved rounds.
# usage: bash tools/sweep_shadow.sh "name=value,..." ...   ("" = defaults)  -> gpurun_out/sweep_shadow.jsonl
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p "$ROOT/gpurun_out"; cd "$ROOT"
for rep in 1 2; do
  for cfg in "$@"; do
    args=(); IFS=',' read -ra kvs <<< "$cfg"; for kv in "${kvs[@]}"; do [ -n "$kv" ] && args+=(--setting "$kv"); done
    r=$(timeout -k 10 120 python3 tools/bench_configs.py --configs ${CONFIGS:-3} --frames 6 "${args[@]}" 2>>"$ROOT/gpurun_out/sweep_shadow.err") || exit 1
    while read -r l; do echo "{\"cfg\": \"$cfg\", \"rep\": $rep, \"res\": $l}" >> "$ROOT/gpurun_out/sweep_shadow.jsonl"; done <<< "$r"
    echo "$cfg rep $rep done"
  done
done
