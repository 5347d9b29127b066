#!/bin/bash
# A/B of the per-ray traversal loops (traceVersion 4 / 5 / 6): parity of the traversal variants, bounce
# microbenchmark, traversal statistics, config-2 frame, configs 3 and 5
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/abv"
mkdir -p "$OUT"
cd "$ROOT"
V="${VERSIONS:-4 5 6}"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "variants or deep_stack or single_instance or traversal_versions or render_frame_parity or room_depth4" > "$OUT/tests.log" 2>&1 || { echo TESTFAIL; tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
for rep in 1 2; do for v in $V; do timeout -k 10 120 python3 tools/trace_kernel_bench.py --set bounce --iters 20 --setting traceVersion=$v > "$OUT/tkb_$v.log" 2>&1 || exit 1; echo "v$v $(tail -1 "$OUT/tkb_$v.log" | cut -c1-80)"; done; done
VERSIONS="$V" bash tools/stats_ab.sh || exit 1
for v in $V; do timeout -k 10 200 python3 bench.py --steps 20 --no-cpu-baseline --no-config4 --setting traceVersion=$v > "$OUT/bench_$v.json" 2> "$OUT/bench_$v.log" || { tail "$OUT/bench_$v.log"; exit 1; }; python3 -c "import json;d=json.load(open('$OUT/bench_$v.json'));print('bench v$v',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['detail']['traceTime0_ms'],d['detail']['traceTime1_ms'])"; done
for v in $V; do timeout -k 10 300 python3 tools/bench_configs.py --configs 3,5 --frames 5 --setting traceVersion=$v > "$OUT/configs_v$v.jsonl" 2>"$OUT/configs_v$v.log" || exit 1
python3 -c "
import json
for l in open('$OUT/configs_v$v.jsonl'):
    d=json.loads(l); print('v$v', d['config'], d['ms_per_frame'], d['Mrays_s'], 'trace', d['traceTime0_ms'], d['traceTime1_ms'], d['traceTimeX_ms'], 'shadow', d['shadowTraceTime_ms'], 'shade', d['shadeTime_ms'])"; done
