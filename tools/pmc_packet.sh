#!/bin/bash
# instruction mix of the packet kernel on the config-2 primary rays (one --pmc pass)
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/pmcpk"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES \
    -f csv -d "$OUT/p1" -o run -- python3 "$ROOT/tools/trace_kernel_bench.py" --set primary --iters 3 --setting unitCoherent=1 > "$OUT/p1.log" 2>&1
echo packet pmc done
