#!/bin/bash
# BVH builder: exact SAH sweep below n triangles per node (setting bvhSweep) vs binned only
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/sweep"
mkdir -p "$OUT"
cd "$ROOT"
for rep in 1 2; do for sw in 0 64 512 4096; do
  timeout -k 10 200 python3 tools/trace_kernel_bench.py --set both --iters 20 --pre-setting bvhSweep=$sw > "$OUT/s$sw.log" 2>&1 || exit 1
  echo "sweep $sw $(tail -1 "$OUT/s$sw.log" | cut -c1-160)"
done; done
for sw in 0 512; do timeout -k 10 300 python3 tools/bench_configs.py --configs 3 --frames 10 --setting bvhSweep=$sw > "$OUT/c3_$sw.jsonl" 2>&1 || exit 1; echo "c3 sweep $sw $(cut -c1-60 "$OUT/c3_$sw.jsonl")"; done
