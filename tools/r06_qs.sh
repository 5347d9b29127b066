#!/bin/bash
# Round 6: the quantized nodes' grid steps as f32 (LH2_QSCALE) and the node step's packed offset / exit-pad FMAs, through
# gpurun: the GPU suite on the in-tree build, then the bounce kernel alone and the config-2 bench against gpuab/base (the
# previous commit) and gpuab/qs (the f32 steps only), and configs 3 and 5 against base.  -> gpurun_out/r06qs/
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/r06qs"
mkdir -p "$OUT"
cd "$ROOT"
export LH2_BLUENOISE="$ROOT/lighthouse2_amd/data/bluenoise.bin"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
tail -1 "$OUT/gpu_tests.log"
bash tools/ab_kernel_libs.sh base qs > "$OUT/kernel.txt"
cat "$OUT/kernel.txt"
bash tools/ab_bench_libs.sh base qs > "$OUT/bench.txt"
cat "$OUT/bench.txt"
for r in 1 2; do
  for v in new base; do
    lib="$ROOT/lighthouse2_amd/libRenderCore_MI355X.so"; [ "$v" = base ] && lib="$ROOT/gpuab/base/libRenderCore_MI355X.so"
    LH2_CORE_LIB="$lib" timeout -k 10 300 python3 tools/bench_configs.py --configs 3,5 > "$OUT/c35_${v}_$r.json" 2> "$OUT/c35_${v}_$r.err"
    echo "$v round $r: $(python3 -c "
import json
for l in open('$OUT/c35_${v}_$r.json'):
    if l.startswith('{'):
        d=json.loads(l); print(d.get('config'), d.get('ms_per_frame'), end='; ')")"
  done
done
echo "r06 qs done"
