#!/bin/bash
# Where the bounce traversal's waves spend their time: three SQ counter passes (issue, wait, memory
# latency levels) on the closest-hit microbenchmark; summarise with tools/pmc_latency.py.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/lat"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
SET="${SET:-bounce}"
LIB="${LIB:-}"
if [ -n "$LIB" ]; then export LH2_CORE_LIB="$ROOT/gpuab/$LIB/libRenderCore_MI355X.so"; fi
run() { timeout -k 10 120 rocprofv3 --pmc "$@" -f csv -d "$OUT/$P" -o run -- python3 "$ROOT/tools/trace_kernel_bench.py" --set "$SET" --iters 3 > "$OUT/$P.log" 2>&1; }
P=p1 run SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM &&
P=p2 run SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_ACTIVE_INST_VALU2 SQ_LDS_BANK_CONFLICT &&
P=p3 run SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_IFETCH SQ_WAVES
echo latency passes done
