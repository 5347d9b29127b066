set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pool
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "tail_pool or traversal_variants or deep_stack or render_frame_parity" > gpurun_out/pool/tests.log 2>&1 || { tail -30 gpurun_out/pool/tests.log; exit 1; }
tail -3 gpurun_out/pool/tests.log
NAME=tailPool VALUES="0 4 8 16 24 32 64" EXTRA_ARGS="--set bounce" bash tools/sweep_setting.sh > gpurun_out/pool/sweep.txt 2>&1 || { cat gpurun_out/pool/sweep.txt; exit 1; }
cat gpurun_out/pool/sweep.txt
for v in 0 16 32; do timeout -k 10 180 python bench.py --no-cpu-baseline --setting tailPool=$v 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print('pool=$v', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])" || exit 1; done | tee gpurun_out/pool/bench.txt
