#!/bin/bash
# Round 6, second GPU call (through gpurun from the repo root): the GPU suite; the VALU probe's new VOP2 / VOPC classes and
# the counter calibration (tools/valu_rate_pmc.sh); the bench; config 5 with and without the per-ray primary frame overlap
# (gpuab/nocamahead: -DLH2_CAM_AHEAD=0), two interleaved rounds; config 5's touched records (gpuab/touch: -DLH2_TOUCH).
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/r06b"
mkdir -p "$OUT"
cd "$ROOT"
export LH2_BLUENOISE="$ROOT/lighthouse2_amd/data/bluenoise.bin"
if [ -n "${TESTS:-1}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
  tail -1 "$OUT/gpu_tests.log"
fi
timeout -k 10 180 "$ROOT/tools/valu_rate" > "$OUT/valu_rate.jsonl"
bash tools/valu_rate_pmc.sh
cd "$ROOT"
timeout -k 10 400 python3 bench.py --cpu-seconds 5 > "$OUT/bench.json" 2> "$OUT/bench.log"
echo "bench: $(python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['config3']['ms_per_frame'], d['config4']['ms_per_frame'], d['config5']['ms_per_frame'])")"
for r in 1 2; do
  for v in on off; do
    lib="$ROOT/lighthouse2_amd/libRenderCore_MI355X.so"; [ "$v" = off ] && lib="$ROOT/gpuab/nocamahead/libRenderCore_MI355X.so"
    LH2_CORE_LIB="$lib" timeout -k 10 200 python3 tools/bench_configs.py --configs 5 > "$OUT/c5_${v}_$r.json" 2> "$OUT/c5_${v}_$r.err"
    echo "camAhead $v round $r: $(tail -1 "$OUT/c5_${v}_$r.json" | cut -c1-220)"
  done
done
LH2_CORE_LIB="$ROOT/gpuab/touch/libRenderCore_MI355X.so" timeout -k 10 300 python3 tools/bench_configs.py --configs 5 --frames 1 --warmup 1 \
  > "$OUT/c5_touch.json" 2> "$OUT/c5_touch.err"
grep -c LH2_TOUCH "$OUT/c5_touch.err"
echo "r06 batch2 done"
