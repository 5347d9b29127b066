#!/bin/bash
# Round 6: sample-inner primary storage (CameraParams::tiled 2) through gpurun.  The parity tests that cover it, then
# config 5 (and 3 as a control) with the in-tree library ("new") against gpuab/si0 (LH2_SAMPLE_INNER 0), two rounds.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/r06si"
mkdir -p "$OUT"
cd "$ROOT"
export LH2_BLUENOISE="$ROOT/lighthouse2_amd/data/bluenoise.bin"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread \
  -k "sample_inner or camera_rays or instanced_animated or converging" > "$OUT/tests.log" 2>&1
tail -1 "$OUT/tests.log"
for r in 1 2; do
  for v in new si0; do
    lib="$ROOT/lighthouse2_amd/libRenderCore_MI355X.so"; [ "$v" != new ] && lib="$ROOT/gpuab/$v/libRenderCore_MI355X.so"
    LH2_CORE_LIB="$lib" timeout -k 10 300 python3 tools/bench_configs.py --configs ${CONFIGS:-5,3} > "$OUT/c_${v}_$r.json" 2> "$OUT/c_${v}_$r.err"
    echo "$v round $r: $(python3 -c "
import json
for l in open('$OUT/c_${v}_$r.json'):
    if l.startswith('{'):
        d=json.loads(l); print(d.get('config'), d.get('ms_per_frame'), d.get('traceTime0_ms'), d.get('traceTime1_ms'), end='; ')")"
  done
done
if [ -n "${FULL:-}" ]; then
  timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -v --timeout 300 --timeout-method thread -k config5 > "$OUT/full5.log" 2>&1
  tail -1 "$OUT/full5.log"
fi
echo "r06 si done"
