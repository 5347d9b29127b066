#!/bin/bash
# Config-3 frame and config-4 N=8 rank share (tools/bench_configs.py, tools/config4_shares.py) for setting
# combinations, one line each: "settings | config-3 ms | share ms".  usage (through gpurun):
#   bash tools/ab_overlap_settings.sh "k=v k=v" "k=v" ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export LH2_BLUENOISE=$PWD/lighthouse2_amd/data/bluenoise.bin
for s in "$@"; do
  st=""; for kv in $s; do st="$st --setting $kv"; done
  c3=$(timeout -k 10 240 python3 tools/bench_configs.py --configs 3 --frames 10 $st 2>/dev/null | tail -1 | python3 -c "import json,sys;d=json.load(sys.stdin);print(d['ms_per_frame'])") || exit 1
  c8=$(timeout -k 10 240 python3 tools/config4_shares.py --ranks 8 --frames 10 $st 2>/dev/null | tail -1 | python3 -c "import json,sys;d=json.load(sys.stdin);print(d['ms_per_frame'])") || exit 1
  echo "$s | $c3 | $c8"
done
