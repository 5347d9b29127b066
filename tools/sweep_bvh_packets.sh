set -e
mkdir -p gpurun_out/sbvh
for ml in 2 4; do for tc in 1 1.5 2 3; do
  r=$(timeout -k 10 120 python tools/trace_kernel_bench.py --set both --refill 32 --pre-setting bvhMaxLeaf=$ml --pre-setting bvhTraversalCost=$tc --setting unitCoherent=1 2>/dev/null)
  b=$(timeout -k 10 120 python tools/trace_kernel_bench.py --set bounce --refill 32 --pre-setting bvhMaxLeaf=$ml --pre-setting bvhTraversalCost=$tc 2>/dev/null)
  echo "{\"maxLeaf\": $ml, \"tc\": $tc, \"packet\": $r, \"perray\": $b}" >> gpurun_out/sbvh/sweep.jsonl
done; done
