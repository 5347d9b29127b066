#!/bin/bash
# A/B of the in-tree library ("new") against gpuab/<name>/libRenderCore_MI355X.so builds on the three
# workloads the round's targets are on, two alternating rounds, one line per run:
#   name  config-2 Mrays/s  frame ms  bounce-trace ms | config-3 frame ms | config-4 N=8 rank share ms
# usage (through gpurun): bash tools/ab_all.sh name...   [AB_SETTINGS="k=v ..." applies to every run]
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"
export LH2_BLUENOISE="$ROOT/lighthouse2_amd/data/bluenoise.bin"
st=""; for kv in ${AB_SETTINGS:-}; do st="$st --setting $kv"; done
for rep in 1 2; do for lib in new "$@"; do
  if [ "$lib" = new ]; then export LH2_CORE_LIB="$ROOT/lighthouse2_amd/libRenderCore_MI355X.so"; else export LH2_CORE_LIB="$ROOT/gpuab/$lib/libRenderCore_MI355X.so"; fi
  b=$(timeout -k 10 180 python3 bench.py --no-cpu-baseline --no-config4 --no-configs --steps 30 $st 2>/dev/null | tail -1) || exit 1
  c2=$(echo "$b" | python3 -c "import json,sys;d=json.load(sys.stdin);print(d['value'],d['ms_per_step'],d['detail']['traceTime1_ms'])")
  c3=$(timeout -k 10 240 python3 tools/bench_configs.py --configs 3 --frames 10 $st 2>/dev/null | tail -1 | python3 -c "import json,sys;d=json.load(sys.stdin);print(d['ms_per_frame'])") || exit 1
  c8=$(timeout -k 10 240 python3 tools/config4_shares.py --ranks 8 --frames 10 $st 2>/dev/null | tail -1 | python3 -c "import json,sys;d=json.load(sys.stdin);print(d['ms_per_frame'])") || exit 1
  echo "$lib $c2 | $c3 | $c8"
done; done
