#!/bin/bash
# One GPU round trip for an iteration (run through gpurun from the repo root):
#   1. pytest -m gpu                                  -> gpurun_out/quick/gpu_tests.log
#   2. bench.py (no CPU baseline)                     -> gpurun_out/quick/bench.json
#   3. rocprofv3 --kernel-trace --stats of bench.py   -> gpurun_out/quick/stats/
# TESTS=0 skips step 1.  Every GPU step has its own time limit; steps are chained with &&.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/quick"
mkdir -p "$OUT"
cd "$ROOT"
if [ "${TESTS:-1}" != "0" ]; then
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 "$ROOT/bench.py" --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.log" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/stats" -o run -- \
    python3 "$ROOT/bench.py" --steps 10 --no-cpu-baseline > "$OUT/bench_prof.json" 2> "$OUT/bench_prof.log"
echo "quick done"
