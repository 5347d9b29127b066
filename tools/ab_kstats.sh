#!/bin/bash
# per-kernel time of config-2 frames (bench.py) and config-3 frames (tools/bench_configs.py) under rocprofv3
# --kernel-trace --stats, for the in-tree library ("new") and gpuab/<name> builds -> gpurun_out/$STEP/ks_<lib>_<cfg>/
# usage (through gpurun): STEP=... bash tools/ab_kstats.sh name...
set -euo pipefail
ROOT="$GRAFT_REPO_ROOT"
OUT="$ROOT/gpurun_out/${STEP:-kstats}"
mkdir -p "$OUT"
export LH2_BLUENOISE="$ROOT/lighthouse2_amd/data/bluenoise.bin"
cd /tmp && export TMPDIR=/tmp
for lib in new "$@"; do
  if [ "$lib" = new ]; then export LH2_CORE_LIB="$ROOT/lighthouse2_amd/libRenderCore_MI355X.so"; else export LH2_CORE_LIB="$ROOT/gpuab/$lib/libRenderCore_MI355X.so"; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/ks_${lib}_c2" -o run -- python3 "$ROOT/bench.py" --no-cpu-baseline --no-config4 --no-configs --steps 30 > "$OUT/ks_${lib}_c2.json" 2>/dev/null
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/ks_${lib}_c3" -o run -- python3 "$ROOT/tools/bench_configs.py" --configs 3 --frames 20 > "$OUT/ks_${lib}_c3.json" 2>/dev/null
done
echo kstats done
