#!/bin/bash
# A/B of built variants (gpuvar/<name>, tools/build_variants.sh / build_rev.sh), interleaved, 2 rounds:
# the closest-hit microbenchmark (primary + bounce rays) and bench.py's frame.  -> gpurun_out/ab_bench.jsonl
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p "$ROOT/gpurun_out"
export LH2_BLUENOISE="$ROOT/lighthouse2_amd/data/bluenoise.bin"   # variants live outside the package
vs=("$@"); [ ${#vs[@]} -eq 0 ] && vs=($(ls "$ROOT/gpuvar"))
for rep in 1 2; do
  for v in "${vs[@]}"; do
    lib="$ROOT/gpuvar/$v/libRenderCore_MI355X.so"
    k=$(LH2_CORE_LIB="$lib" timeout -k 10 120 python3 "$ROOT/tools/trace_kernel_bench.py" --set both 2>>"$ROOT/gpurun_out/ab_bench.err"); rc=$?
    [ $rc -ne 0 ] && { echo "{\"variant\": \"$v\", \"rc\": $rc}" >> "$ROOT/gpurun_out/ab_bench.jsonl"; exit $rc; }
    b=$(LH2_CORE_LIB="$lib" timeout -k 10 180 python3 "$ROOT/bench.py" --no-cpu-baseline 2>>"$ROOT/gpurun_out/ab_bench.err" | tail -1); rc=$?
    [ $rc -ne 0 ] && { echo "{\"variant\": \"$v\", \"rc\": $rc}" >> "$ROOT/gpurun_out/ab_bench.jsonl"; exit $rc; }
    echo "{\"variant\": \"$v\", \"rep\": $rep, \"kernel\": $k, \"bench\": $b}" | tee -a "$ROOT/gpurun_out/ab_bench.jsonl"
  done
done
exit 0
