#!/bin/bash
# Round-5 end measurement (through gpurun from the repo root): tools/round_batch.sh (GPU suite, bench.py + rocprofv3 kernel stats
# + PMC traffic, SQ / config-3 / config-5 counter passes, config 1), then the config-4 shares N = 1, 2, 4, 8 and the N = 8
# share's kernel timeline.  Every GPU step has its own time limit; a failing step ends the batch.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"
bash tools/round_batch.sh
cd "$ROOT"
mkdir -p gpurun_out/r05end
timeout -k 10 300 python3 tools/config4_shares.py > gpurun_out/r05end/config4_shares.jsonl 2> gpurun_out/r05end/config4_shares.err
cat gpurun_out/r05end/config4_shares.jsonl
bash tools/share_timeline.sh 8 > gpurun_out/r05end/share8.txt 2>&1
cp gpurun_out/share8/timeline.txt gpurun_out/r05end/share8_timeline.txt
head -3 gpurun_out/r05end/share8.txt
echo "r05 round done"
