#!/bin/bash
# VALU lane utilisation of the closest-hit kernel: SQ_THREAD_CYCLES_VALU / (64 x SQ_ACTIVE_INST_VALU),
# one --pmc pass per ray set (primary, bounce).
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/lanes"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for SET in primary bounce; do
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD \
    -f csv -d "$OUT/$SET" -o run -- python3 "$ROOT/tools/trace_kernel_bench.py" --set "$SET" --iters 3 > "$OUT/$SET.log" 2>&1
done
echo lanes done
