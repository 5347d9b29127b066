#!/bin/bash
# VALU issue probe (tools/valu_rate) + SQ counters of the bounce-ray kernel per traceVersion
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/sqv"
mkdir -p "$OUT"
timeout -k 10 60 "$ROOT/tools/valu_rate" > "$OUT/valu_rate.jsonl" 2>&1 || exit 1
cat "$OUT/valu_rate.jsonl"
cd /tmp && export TMPDIR=/tmp
for v in ${VERSIONS:-4 5}; do
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE \
    -f csv -d "$OUT/v$v/sq1" -o run -- python3 "$ROOT/tools/trace_kernel_bench.py" --set bounce --iters 5 --setting traceVersion=$v > "$OUT/v$v.sq1.log" 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS \
    -f csv -d "$OUT/v$v/sq2" -o run -- python3 "$ROOT/tools/trace_kernel_bench.py" --set bounce --iters 5 --setting traceVersion=$v > "$OUT/v$v.sq2.log" 2>&1 || exit 1
done
echo sqv done
