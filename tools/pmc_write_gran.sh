#!/bin/bash
# WRITE_SIZE calibration for scattered 16-B record stores (tools/write_gran.hip) and the same counters on the
# bounce traversal (tools/trace_kernel_bench.py --set bounce): one rocprofv3 --pmc pass per counter group.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/pmc_wg"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export LH2_BLUENOISE="$ROOT/lighthouse2_amd/data/bluenoise.bin"
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/wg1" -o run --output-format csv -- "$ROOT/tools/write_gran" > "$OUT/wg1.log" 2>&1
timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --kernel-trace -d "$OUT/wg2" -o run --output-format csv -- "$ROOT/tools/write_gran" > "$OUT/wg2.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/tr1" -o run --output-format csv -- python3 "$ROOT/tools/trace_kernel_bench.py" --set bounce --iters 3 > "$OUT/tr1.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --kernel-trace -d "$OUT/tr2" -o run --output-format csv -- python3 "$ROOT/tools/trace_kernel_bench.py" --set bounce --iters 3 > "$OUT/tr2.log" 2>&1
echo "pmc write gran done"
