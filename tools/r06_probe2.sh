#!/bin/bash
# Round 6: the candidate node-step instruction classes (tools/valu_rate's second batch) at 8 waves per SIMD, through
# gpurun; tools/valu_rate built on the CPU.  -> gpurun_out/r06probe2/valu_rate.jsonl
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/r06probe2"
mkdir -p "$OUT"
: > "$OUT/valu_rate.jsonl"
for m in add fma cvtb max maxi minu max3 max3i orsdwa sub pkadd pkmul pkfma shr bfe perm med3 cmp32 cmpi minf; do
  timeout -k 10 60 "$ROOT/tools/valu_rate" --mode "$m" --waves 8 >> "$OUT/valu_rate.jsonl"
done
echo "probe2 done"
