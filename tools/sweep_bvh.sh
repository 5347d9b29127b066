#!/bin/bash
# BVH build parameter sweep on the closest-hit microbenchmark (GPU box): gpurun_out/sweep_bvh.jsonl
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p "$ROOT/gpurun_out"
for leaf in ${LEAVES:-2 4 8}; do
  for ct in ${COSTS:-0.5 1 2 3}; do
    out=$(timeout -k 10 120 python3 "$ROOT/tools/trace_kernel_bench.py" --pre-setting bvhMaxLeaf=$leaf --pre-setting bvhTraversalCost=$ct) || exit 1
    echo "{\"leaf\": $leaf, \"cost\": $ct, \"res\": $out}" | tee -a "$ROOT/gpurun_out/sweep_bvh.jsonl"
  done
done
