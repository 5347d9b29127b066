#!/bin/bash
# Round batch (through gpurun from the repo root): GPU suite, bench + rocprofv3 kernel stats + PMC
# traffic (profile_gpu.sh; bench.py also times configs 3, 4 in-core and 5), SQ / config-3 / config-5 counter passes
# (pmc_round.sh), config 1.
# Every GPU step has its own time limit; a failing step ends the batch.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/prof"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
tail -1 "$OUT/gpu_tests.log"
bash "$ROOT/tools/profile_gpu.sh"
bash "$ROOT/tools/pmc_round.sh"
cd "$ROOT"
timeout -k 10 300 python3 tools/config1_plumbing.py --cpu-seconds 10 > "$OUT/config1.json" 2> "$OUT/config1.log"
echo "round batch done"
