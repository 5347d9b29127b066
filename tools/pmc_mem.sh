#!/bin/bash
# Memory-pipeline counters of the bounce traversal kernel (tools/trace_kernel_bench.py --set bounce), one
# rocprofv3 --pmc pass per counter group -> gpurun_out/pmc_mem/<pass>/; summary: tools/summarize_pmc_mem.py
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/pmc_mem"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export LH2_BLUENOISE="$ROOT/lighthouse2_amd/data/bluenoise.bin"
run() {
  local name="$1"; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace -d "$OUT/$name" -o run --output-format csv -- \
    python3 "$ROOT/tools/trace_kernel_bench.py" --set bounce --iters 5 > "$OUT/$name.log" 2>&1
}
run p1 TA_TA_BUSY TA_BUFFER_TOTAL_CYCLES TD_TD_BUSY TD_TC_STALL GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_INST_LEVEL_VMEM SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_WAVE_CYCLES SQ_BUSY_CYCLES
run p2 TCP_TCP_LATENCY TCP_PENDING_STALL_CYCLES TCP_TCC_READ_REQ_LATENCY TCP_TCC_READ_REQ TA_TCP_STATE_READ TA_ADDR_STALLED_BY_TC_CYCLES SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE
run p3 TCP_TOTAL_CACHE_ACCESSES TCP_TCR_TCP_STALL_CYCLES TCP_READ_TAGCONFLICT_STALL_CYCLES TCP_TCP_TA_DATA_STALL_CYCLES TA_DATA_STALLED_BY_TC_CYCLES TA_BUFFER_READ_WAVEFRONTS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE
echo "pmc mem done"
