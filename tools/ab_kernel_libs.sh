#!/bin/bash
# Bounce-ray traversal kernel alone (tools/trace_kernel_bench.py --set bounce, config-2 scene) with the in-tree
# library ("new") and variant builds gpuab/<name>/libRenderCore_MI355X.so, three alternating rounds -> one
# line per run: name, bounce ms (mean of --iters launches), Mrays/s
# usage (through gpurun): bash tools/ab_kernel_libs.sh name...
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"
export LH2_BLUENOISE="$ROOT/lighthouse2_amd/data/bluenoise.bin"
for rep in 1 2 3; do for lib in new "$@"; do
  if [ "$lib" = new ]; then unset LH2_CORE_LIB; else export LH2_CORE_LIB="$ROOT/gpuab/$lib/libRenderCore_MI355X.so"; fi
  b=$(timeout -k 10 180 python3 tools/trace_kernel_bench.py --set bounce --iters 200 2>/dev/null | tail -1) || exit 1
  echo "$lib $(echo "$b" | python3 -c "import json,sys;d=json.load(sys.stdin)['bounce'];print(d['ms'],d['Mrays_s'])")"
done; done
