#!/bin/bash
# Frame A/B of core settings: each argument is one configuration, a comma-separated list of
# name=value settings ("" = defaults); 2 interleaved rounds of bench.py.  -> gpurun_out/ab_settings.jsonl
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p "$ROOT/gpurun_out"; cd "$ROOT"
for rep in 1 2; do
  for cfg in "$@"; do
    args=(); IFS=',' read -ra kvs <<< "$cfg"; for kv in "${kvs[@]}"; do [ -n "$kv" ] && args+=(--setting "$kv"); done
    b=$(timeout -k 10 180 python3 bench.py --no-cpu-baseline "${args[@]}" 2>>"$ROOT/gpurun_out/ab_settings.err" | tail -1) || exit 1
    echo "{\"cfg\": \"$cfg\", \"rep\": $rep, \"bench\": $b}" | tee -a "$ROOT/gpurun_out/ab_settings.jsonl"
  done
done
