#!/bin/bash
# traceVersion 7 (leaf slot + batched leaf tests) vs 6: parity, bounce launch per leafBatch, stats, frame, configs
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/abslot"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "variants or deep_stack or single_instance or traversal_versions" > "$OUT/tests.log" 2>&1 || { echo TESTFAIL; tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
for rep in 1 2; do
timeout -k 10 120 python3 tools/trace_kernel_bench.py --set bounce --iters 20 --setting traceVersion=6 > "$OUT/v6.log" 2>&1 || exit 1; echo "v6 $(tail -1 "$OUT/v6.log" | cut -c1-80)"
for b in 4 8 16 24 32 48; do timeout -k 10 120 python3 tools/trace_kernel_bench.py --set bounce --iters 20 --setting traceVersion=7 --leaf-batch $b > "$OUT/v7_$b.log" 2>&1 || exit 1; echo "v7 batch $b $(tail -1 "$OUT/v7_$b.log" | cut -c1-80)"; done
done
VERSIONS="6 7" bash tools/stats_ab.sh || exit 1
for v in 6 7; do timeout -k 10 300 python3 tools/bench_configs.py --configs 3,5 --frames 5 --setting traceVersion=$v > "$OUT/configs_v$v.jsonl" 2>"$OUT/configs_v$v.log" || exit 1
python3 -c "
import json
for l in open('$OUT/configs_v$v.jsonl'):
    d=json.loads(l); print('v$v', d['config'], d['ms_per_frame'], d['Mrays_s'], 'trace', d['traceTime0_ms'], d['traceTime1_ms'], d['traceTimeX_ms'], 'shadow', d['shadowTraceTime_ms'], 'shade', d['shadeTime_ms'])"; done
