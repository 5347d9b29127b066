#!/bin/bash
# A/B of the persistent trace grid (setting traceBlocksPerCU: 0 = the occupancy limit) on config 2 and config 3 frames -> gpurun_out/r03q_tbpc/ab.txt
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$ROOT"; mkdir -p gpurun_out/r03q_tbpc
export LH2_BLUENOISE="$ROOT/lighthouse2_amd/data/bluenoise.bin"
for rep in 1 2; do for v in 0 6 5 4; do
  st=""; [ "$v" != 0 ] && st="--setting traceBlocksPerCU=$v"
  c2=$(timeout -k 10 180 python3 bench.py --no-cpu-baseline --no-config4 --no-configs --steps 30 $st 2>/dev/null | tail -1 | python3 -c "import json,sys;d=json.load(sys.stdin);print(d['value'],d['ms_per_step'],d['detail']['traceTime1_ms'])") || exit 1
  c3=$(timeout -k 10 240 python3 tools/bench_configs.py --configs 3 --frames 10 $st 2>/dev/null | tail -1 | python3 -c "import json,sys;d=json.load(sys.stdin);print(d['ms_per_frame'])") || exit 1
  echo "tbpc=$v $c2 | $c3" | tee -a gpurun_out/r03q_tbpc/ab.txt
done; done
