#!/bin/bash
# End-of-iteration GPU batch (through gpurun from the repo root): GPU suite, profile (bench, rocprofv3
# kernel stats, PMC passes), config 1 (SoftRasterizer reference beside the core), configs 3 and 5.
# Every GPU step has its own time limit; steps are chained with && so a failure ends the batch.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/prof"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
tail -1 "$OUT/gpu_tests.log"
bash "$ROOT/tools/profile_gpu.sh"
cd "$ROOT"
timeout -k 10 300 python3 tools/config1_plumbing.py --cpu-seconds 10 > "$OUT/config1.json" 2> "$OUT/config1.log"
timeout -k 10 600 python3 tools/bench_configs.py --configs 3,5 > "$OUT/configs_3_5.jsonl" 2> "$OUT/configs_3_5.log"
echo "round profile done"
