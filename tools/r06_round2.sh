#!/bin/bash
# Round-6 end measurement, part 2 (through gpurun from the repo root): the config-4 shares N = 1, 2, 4, 8, the N = 8 share's
# kernel timeline, and config 5's touched records (gpuab/touch: the LH2_TOUCH build) for the HBM lower bound.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$ROOT"
export LH2_BLUENOISE="$ROOT/lighthouse2_amd/data/bluenoise.bin"
OUT="$ROOT/gpurun_out/r06end"
mkdir -p "$OUT"
timeout -k 10 300 python3 tools/config4_shares.py > "$OUT/config4_shares.jsonl" 2> "$OUT/config4_shares.err"
cat "$OUT/config4_shares.jsonl"
bash tools/share_timeline.sh 8 > "$OUT/share8.txt" 2>&1
cp gpurun_out/share8/timeline.txt "$OUT/share8_timeline.txt"
tail -2 "$OUT/share8_timeline.txt"
if [ -n "${TOUCH:-1}" ]; then
  LH2_CORE_LIB="$ROOT/gpuab/touch/libRenderCore_MI355X.so" timeout -k 10 300 python3 tools/bench_configs.py --configs 5 --frames 1 --warmup 1 \
    > "$OUT/c5_touch.json" 2> "$OUT/c5_touch.err"
  grep -c "LH2_TOUCH " "$OUT/c5_touch.err"
fi
echo "r06 round part 2 done"
