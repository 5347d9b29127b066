#!/bin/bash
# VALU issue peak per instruction mix (through gpurun, tools/valu_rate built on the CPU beforehand):
#   gpurun_out/valu/rate.jsonl   tools/valu_rate, every mode at 1/2/4/8 waves per SIMD
#   gpurun_out/valu/pmc/         SQ_INSTS_VALU / SQ_ACTIVE_INST_VALU / GRBM_GUI_ACTIVE of the mix kernel
# then on the CPU: python3 tools/valu_rate_summary.py --tag <tag>  ->  profiles/<tag>_valu_rate.jsonl
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/valu"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 "$ROOT/tools/valu_rate" > "$OUT/rate.jsonl"
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --kernel-trace -d "$OUT/pmc" -o run \
  --output-format csv -- "$ROOT/tools/valu_rate" --mode mix > "$OUT/pmc.log" 2>&1
echo "valu_rate done"
