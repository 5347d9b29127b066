set -uo pipefail
mkdir -p gpurun_out
for b in 7 6 5 4 3; do
  timeout -k 10 120 python3 tools/trace_kernel_bench.py --set both --setting traceBlocksPerCU=$b > gpurun_out/blk_$b.json 2>/dev/null || exit 1
done
