#!/bin/bash
# Whole-frame A/B: bench.py (no CPU baseline) for every built variant in gpuvar/ -> gpurun_out/ab_bench.jsonl
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export LH2_BLUENOISE="$ROOT/lighthouse2_amd/data/bluenoise.bin"
vs=("$@"); [ ${#vs[@]} -eq 0 ] && vs=($(ls "$ROOT/gpuvar"))
for v in "${vs[@]}"; do
  out=$(LH2_CORE_LIB="$ROOT/gpuvar/$v/libRenderCore_MI355X.so" timeout -k 10 200 python3 "$ROOT/bench.py" --no-cpu-baseline --steps 30) || exit 1
  echo "{\"variant\": \"$v\", \"res\": $out}" | tee -a "$ROOT/gpurun_out/ab_bench.jsonl"
done
