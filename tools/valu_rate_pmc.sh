#!/bin/bash
# What SQ_ACTIVE_INST_VALU counts (through gpurun, tools/valu_rate built on the CPU): one rocprofv3 --pmc pass per
# instruction class at 8 waves per SIMD, with SQ_INSTS_VALU, SQ_ACTIVE_INST_VALU, SQ_BUSY_CYCLES, SQ_WAVE_CYCLES and
# GRBM_GUI_ACTIVE, so the counter's cycles per VALU instruction can be set beside the probe's s_memtime cycles (a 2-cycle
# class and a 4-cycle class tell whether it counts issue cycles or per-wave occupancy).  -> gpurun_out/valu_pmc/<mode>/
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/valu_pmc"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for m in ${MODES:-add fma fmac pkfma mix}; do
  timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --kernel-trace \
    -d "$OUT/$m" -o run --output-format csv -- "$ROOT/tools/valu_rate" --mode "$m" --waves 8 > "$OUT/$m.log" 2>&1
done
echo "valu pmc done"
