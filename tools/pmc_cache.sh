#!/bin/bash
# Cache behaviour of the closest-hit microbenchmark (SET, default bounce): vL1D hit rate and L2 read latency
# (TCP pass), L2 hit rate and memory-side read latency (TCC pass); summarise with tools/pmc_latency.py DIR KERNEL.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/cache"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
SET="${SET:-bounce}"
run() { timeout -s KILL 120 rocprofv3 --pmc "$@" -f csv -d "$OUT/$P" -o run -- python3 "$ROOT/tools/trace_kernel_bench.py" --set "$SET" --iters 3 > "$OUT/$P.log" 2>&1; }
P=p1 run TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_UTCL1_TRANSLATION_MISS_sum &&
P=p2 run TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum
echo cache passes done
