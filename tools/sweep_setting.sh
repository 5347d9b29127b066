#!/bin/bash
# Sweep one runtime setting on the closest-hit microbenchmark: NAME=leafBatch VALUES="1 8 16" bash tools/sweep_setting.sh
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
for v in $VALUES; do
  out=$(timeout -k 10 120 python3 "$ROOT/tools/trace_kernel_bench.py" --setting $NAME=$v $EXTRA_ARGS) || exit 1
  echo "$NAME=$v $out"
done
