#!/bin/bash
# k_shade counters on the config-2 bench frame (two --pmc passes)
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/pmcsh"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR \
    -f csv -d "$OUT/p1" -o run -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --kernel-iters 1 > "$OUT/p1.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -f csv -d "$OUT/p2" -o run -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --kernel-iters 1 > "$OUT/p2.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -f csv -d "$OUT/p3" -o run -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --kernel-iters 1 > "$OUT/p3.log" 2>&1
echo shade pmc done
