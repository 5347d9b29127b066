#!/bin/bash
# shadow split (setting shadowSplit 0 / 1 / 2 / 3): parity, config-3 frames
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/split"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "shadow_split or room_depth4 or render_frame_parity or path_groups" > "$OUT/tests.log" 2>&1 || { echo TESTFAIL; tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
for rep in 1 2; do for sp in 0 1 2 3; do
timeout -k 10 300 python3 tools/bench_configs.py --configs 3 --frames 10 --setting shadowSplit=$sp > "$OUT/c3_$sp.jsonl" 2>"$OUT/c3_$sp.log" || exit 1
python3 -c "
import json
for l in open('$OUT/c3_$sp.jsonl'):
    d=json.loads(l); print('split $sp', d['config'], d['ms_per_frame'], d['Mrays_s'], 'trace', d['traceTime0_ms'], d['traceTime1_ms'], d['traceTimeX_ms'], 'shadow', d['shadowTraceTime_ms'], 'shade', d['shadeTime_ms'])"; done; done
