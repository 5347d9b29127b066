#!/bin/bash
# configs 3 and 5 (tools/bench_configs.py) for each variant in gpuvar/ with optional extra settings
# usage: bash tools/ab_configs.sh "variant[:setting=value,...]" ...   -> gpurun_out/ab_configs.jsonl
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export LH2_BLUENOISE="$ROOT/lighthouse2_amd/data/bluenoise.bin"
for spec in "$@"; do
  v="${spec%%:*}"; st=""; [ "$spec" != "$v" ] && for kv in $(echo "${spec#*:}" | tr ',' ' '); do st="$st --setting $kv"; done
  LH2_CORE_LIB="$ROOT/${VARDIR:-gpuvar}/$v/libRenderCore_MI355X.so" timeout -k 10 300 python3 "$ROOT/tools/bench_configs.py" --configs ${CONFIGS:-3,5} --frames 6 $st > /tmp/abc.jsonl || exit 1
  while read -r l; do echo "{\"spec\": \"$spec\", \"res\": $l}" >> "$ROOT/gpurun_out/ab_configs.jsonl"; done < /tmp/abc.jsonl
done
