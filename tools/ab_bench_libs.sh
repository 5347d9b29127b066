#!/bin/bash
# bench.py (config 2, no config 4 / CPU baseline) with the in-tree library ("new") and variant builds
# gpuab/<name>/libRenderCore_MI355X.so, two alternating rounds -> one line per run on stdout
# usage (through gpurun): bash tools/ab_bench_libs.sh name...
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"
export LH2_BLUENOISE="$ROOT/lighthouse2_amd/data/bluenoise.bin"
for rep in 1 2; do for lib in new "$@"; do
  if [ "$lib" = new ]; then unset LH2_CORE_LIB; else export LH2_CORE_LIB="$ROOT/gpuab/$lib/libRenderCore_MI355X.so"; fi
  b=$(timeout -k 10 180 python3 bench.py --no-cpu-baseline --no-config4 --no-configs --steps 30 2>/dev/null | tail -1) || exit 1
  echo "$lib $(echo "$b" | python3 -c "import json,sys;d=json.load(sys.stdin);print(d['value'],d['ms_per_step'],d['detail']['traceTime0_ms'],d['detail']['traceTime1_ms'],d['detail']['shadeTime_ms'])")"
done; done
