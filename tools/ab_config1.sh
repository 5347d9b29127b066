#!/bin/bash
# config 1 (tools/config1_plumbing.py: restart every frame) for the in-tree library ("new", also with the settings in
# C1_SETTINGS, one run per space-separated entry) and gpuab/<name> builds
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export LH2_BLUENOISE="$GRAFT_REPO_ROOT/lighthouse2_amd/data/bluenoise.bin"
run() { timeout -k 10 200 python3 tools/config1_plumbing.py --cpu-seconds 1 "$@" 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['mi355x_core']['ms_per_frame'])"; }
for rep in 1 2; do
  export LH2_CORE_LIB="$GRAFT_REPO_ROOT/lighthouse2_amd/libRenderCore_MI355X.so"
  echo "new $(run)"
  for st in ${C1_SETTINGS:-}; do echo "new:$st $(run --setting $st)"; done
  for lib in "$@"; do export LH2_CORE_LIB="$GRAFT_REPO_ROOT/gpuab/$lib/libRenderCore_MI355X.so"; echo "$lib $(run)"; done
done
