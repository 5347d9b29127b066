#!/bin/bash
# SQ counter pass on the closest-hit microbenchmark (primary rays); one --pmc pass per group.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/sq"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
SET="${SET:-primary}"
timeout -k 10 120 rocprofv3 --list-avail > "$OUT/avail.txt" 2>&1 || true
timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES \
    -f csv -d "$OUT/p1" -o run -- python3 "$ROOT/tools/trace_kernel_bench.py" --set "$SET" --iters 3 > "$OUT/p1.log" 2>&1 &&
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD TCP_TCC_READ_REQ_sum TCC_HIT_sum \
    -f csv -d "$OUT/p2" -o run -- python3 "$ROOT/tools/trace_kernel_bench.py" --set "$SET" --iters 3 > "$OUT/p2.log" 2>&1
echo sq done
