#!/bin/bash
# Time the closest-hit microbenchmark for every built variant in gpuvar/ (tools/build_variants.sh).
# usage (on the GPU box): bash tools/ab_variants.sh [variant ...]   -> gpurun_out/ab.jsonl
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export LH2_BLUENOISE="$ROOT/lighthouse2_amd/data/bluenoise.bin"
mkdir -p "$ROOT/gpurun_out"
vs=("$@"); [ ${#vs[@]} -eq 0 ] && vs=($(ls "$ROOT/gpuvar"))
for v in "${vs[@]}"; do
  for rep in 1 2; do
    out=$(LH2_CORE_LIB="$ROOT/gpuvar/$v/libRenderCore_MI355X.so" timeout -k 10 120 python3 "$ROOT/tools/trace_kernel_bench.py" ${TKB_ARGS:-} 2>/dev/null)
    rc=$?
    echo "{\"variant\": \"$v\", \"rep\": $rep, \"rc\": $rc, \"res\": ${out:-null}}" | tee -a "$ROOT/gpurun_out/ab.jsonl"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
