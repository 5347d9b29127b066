#!/bin/bash
# Round-6 end measurement (through gpurun from the repo root), part 1: tools/round_batch.sh (GPU suite, bench.py + rocprofv3
# kernel stats + PMC traffic, SQ / config-3 / config-5 counter passes, config 1).  Part 2 is tools/r06_round2.sh.  Every GPU
# step has its own time limit; a failing step ends the batch.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"
export LH2_BLUENOISE="$ROOT/lighthouse2_amd/data/bluenoise.bin"
bash tools/round_batch.sh
echo "r06 round part 1 done"
