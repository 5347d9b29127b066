#!/bin/bash
# Round 6: node-step variants, through gpurun (every variant staged under gpuab/, the in-tree build = "new"):
#   base  the previous commit;  qs  the quantized nodes' grid steps as f32 (LH2_QSCALE);
#   qspk  qs + the node offsets and exit pads as packed FMAs;  qspke  qspk + the early node loads in every lane;
#   new   qs + the early node loads in every lane.
# The GPU suite on new, the bounce kernel alone and the config-2 bench for all, configs 3 and 5 for new / qs / base.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/r06qs2"
mkdir -p "$OUT"
cd "$ROOT"
export LH2_BLUENOISE="$ROOT/lighthouse2_amd/data/bluenoise.bin"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
tail -1 "$OUT/gpu_tests.log"
bash tools/ab_kernel_libs.sh base qs qspk qspke > "$OUT/kernel.txt"
cat "$OUT/kernel.txt"
bash tools/ab_bench_libs.sh base qs qspk qspke > "$OUT/bench.txt"
cat "$OUT/bench.txt"
for r in 1 2; do
  for v in new qs base; do
    lib="$ROOT/lighthouse2_amd/libRenderCore_MI355X.so"; [ "$v" != new ] && lib="$ROOT/gpuab/$v/libRenderCore_MI355X.so"
    LH2_CORE_LIB="$lib" timeout -k 10 300 python3 tools/bench_configs.py --configs 3,5 > "$OUT/c35_${v}_$r.json" 2> "$OUT/c35_${v}_$r.err"
    echo "$v round $r: $(python3 -c "
import json
for l in open('$OUT/c35_${v}_$r.json'):
    if l.startswith('{'):
        d=json.loads(l); print(d.get('config'), d.get('ms_per_frame'), end='; ')")"
  done
done
echo "r06 qs2 done"
