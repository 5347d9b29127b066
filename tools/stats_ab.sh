#!/bin/bash
# traversal statistics (LH2_TRACE_STATS build in gpustats/) of the bounce-ray launch, per traceVersion
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p "$ROOT/gpurun_out/stats"
for v in ${VERSIONS:-4 5}; do
  LH2_CORE_LIB="$ROOT/gpustats/libRenderCore_MI355X.so" timeout -k 10 120 python3 "$ROOT/tools/trace_kernel_bench.py" --set ${SET:-bounce} --iters 2 --setting traceVersion=$v > "$ROOT/gpurun_out/stats/v$v.log" 2>&1 || exit 1
  echo "v$v: $(grep LH2_TRACE_STATS "$ROOT/gpurun_out/stats/v$v.log" | tail -1)"
done
