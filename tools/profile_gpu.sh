#!/bin/bash
# Round profile on the MI355X box (run through gpurun from the repo root):
#   1. bench.py (JSON line)                           -> gpurun_out/prof/bench.json
#   2. rocprofv3 --kernel-trace --stats of bench.py, config 2 only (the roofline kernel's launches are the
#      config-2 frames' and bench.py's own timed ones)   -> gpurun_out/prof/stats/
#   3. two separate --pmc passes (FETCH_SIZE, WRITE_SIZE; the TCC block cannot hold both) on the
#      closest-hit microbenchmark on the bounce rays (bench.py's roofline kernel)
#                                                           -> gpurun_out/prof/pmc_fetch, pmc_write
# Every GPU step has its own time limit and the steps are chained with &&.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/prof"
mkdir -p "$OUT"
STEPS="${STEPS:-20}"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 "$ROOT/bench.py" --steps "$STEPS" > "$OUT/bench.json" 2> "$OUT/bench.log" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/stats" -o run -- \
    python3 "$ROOT/bench.py" --steps "$STEPS" --no-cpu-baseline --no-config4 --no-configs > "$OUT/bench_prof.json" 2> "$OUT/bench_prof.log" &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -f csv -d "$OUT/pmc_fetch" -o run -- \
    python3 "$ROOT/tools/trace_kernel_bench.py" --set bounce --iters 10 > "$OUT/pmc_fetch.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -f csv -d "$OUT/pmc_write" -o run -- \
    python3 "$ROOT/tools/trace_kernel_bench.py" --set bounce --iters 10 > "$OUT/pmc_write.log" 2>&1
echo "profile done"
