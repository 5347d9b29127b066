#!/bin/bash
# Round 6 debug call: tools/dbg/gather_check.py on the main library and the A/B variants
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"
export LH2_BLUENOISE="$ROOT/lighthouse2_amd/data/bluenoise.bin"
for v in main nobehind bfsorder; do
  lib="$ROOT/lighthouse2_amd/libRenderCore_MI355X.so"; [ "$v" != main ] && lib="$ROOT/gpuab/$v/libRenderCore_MI355X.so"
  echo "== $v"
  LH2_CORE_LIB="$lib" timeout -k 10 120 python3 tools/dbg/gather_check.py
done
echo "dbg done"
