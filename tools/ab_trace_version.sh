set -e
mkdir -p gpurun_out/ab
export LH2_TRACE_VERSION=2
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/tests_v2.log 2>&1
for v in 1 2 1 2; do
  LH2_TRACE_VERSION=$v timeout -k 10 120 python tools/trace_kernel_bench.py --iters 20 > gpurun_out/ab/kb_v$v.json 2>/dev/null
  cat gpurun_out/ab/kb_v$v.json >> gpurun_out/ab/kb_all.txt; echo " v$v" >> gpurun_out/ab/kb_all.txt
done
for v in 1 2; do
  LH2_TRACE_VERSION=$v timeout -k 10 200 python bench.py --steps 20 --no-cpu-baseline > gpurun_out/ab/bench_v$v.json 2>/dev/null
done
echo ok
