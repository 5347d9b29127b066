#!/bin/bash
# The shade launch's wave time by stage (through gpurun from the repo root): config 3 frames with a -DLH2_SHADE_TIMES build
# (gpuab/stt, built by `make EXTRA=-DLH2_SHADE_TIMES OUT=gpuab/stt/libRenderCore_MI355X.so`), summarised by
# tools/shade_times.py.  Diagnostic only: the marks' own cost is in the times.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/stt"
mkdir -p "$OUT"
cd "$ROOT"
export LH2_BLUENOISE="$ROOT/lighthouse2_amd/data/bluenoise.bin"
LH2_CORE_LIB="$ROOT/gpuab/stt/libRenderCore_MI355X.so" timeout -k 10 300 python3 tools/bench_configs.py --configs 3 --frames 10 \
  > "$OUT/config3.json" 2> "$OUT/config3.err"
grep LH2_SHADE_TIMES "$OUT/config3.err" | tail -1 > "$OUT/times.txt"
python3 tools/shade_times.py "$OUT/times.txt" | tee "$OUT/summary.txt"
if [ -n "${C2:-}" ]; then
  # config 2 (no lights: k_shade<false, true>): the bench line's frames alone
  LH2_CORE_LIB="$ROOT/gpuab/stt/libRenderCore_MI355X.so" timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-configs --no-config4 \
    --steps 20 > "$OUT/config2.json" 2> "$OUT/config2.err"
  grep LH2_SHADE_TIMES "$OUT/config2.err" | tail -1 > "$OUT/times_c2.txt"
  echo "config 2:"; python3 tools/shade_times.py "$OUT/times_c2.txt" | tee "$OUT/summary_c2.txt"
fi
