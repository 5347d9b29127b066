#!/bin/bash
# A/B of setting combinations (through gpurun): per variant (comma-separated name=value list, "base" = defaults;
# lib=<name> loads the variant build gpuab/<name>/libRenderCore_MI355X.so, tools/build_variant.sh) the
# config-4 rank shares at N = 1 and 8, config 3 (tools/bench_configs.py) and config 2 (bench.py, no other configs),
# the variants interleaved, REPS rounds.  usage: VARIANTS="base sideBlocks=3 sideBlocks=3,pathTailBlocks=2" REPS=2
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-abm}"
mkdir -p "$OUT"
cd "$ROOT"
for rep in $(seq 1 "${REPS:-2}"); do
  for v in ${VARIANTS:-base}; do
    args=()
    unset LH2_CORE_LIB
    if [ "$v" != "base" ]; then IFS=',' read -ra kvs <<< "$v"; for kv in "${kvs[@]}"; do
      if [[ "$kv" == lib=* ]]; then export LH2_CORE_LIB="$ROOT/gpuab/${kv#lib=}/libRenderCore_MI355X.so"; else args+=(--setting "$kv"); fi
    done; fi
    n="${v//[=,]/_}_$rep"
    timeout -k 10 200 python3 tools/config4_shares.py --ranks 1,8 "${args[@]}" > "$OUT/sh_$n.jsonl" 2> "$OUT/sh_$n.err"
    timeout -k 10 200 python3 tools/bench_configs.py --configs 3 --frames 10 "${args[@]}" > "$OUT/c3_$n.jsonl" 2> "$OUT/c3_$n.err"
    timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-configs --no-config4 "${args[@]}" > "$OUT/c2_$n.json" 2> "$OUT/c2_$n.err"
    python3 - "$OUT" "$n" "$v" <<'PY'
import json, sys
o, n, v = sys.argv[1:]
sh = [json.loads(l) for l in open(f"{o}/sh_{n}.jsonl") if l.strip()]
c3 = json.loads(open(f"{o}/c3_{n}.jsonl").readline())
c2 = json.load(open(f"{o}/c2_{n}.json"))
print(f"{v:40s} N1 {sh[0]['ms_per_frame']:.4f} N8 {sh[-1]['ms_per_frame']:.4f} ratio {sh[0]['ms_per_frame'] / sh[-1]['ms_per_frame']:.3f} | c3 {c3['ms_per_frame']:.4f} | c2 {c2['ms_per_step']:.4f} {c2['value']:.0f}", flush=True)
PY
  done
done
unset LH2_CORE_LIB
echo "ab_multi done"
