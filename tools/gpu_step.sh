#!/bin/bash
# one A/B step through gpurun: GPU suite, then tools/ab_all.sh against the gpuab/ builds named in AB_LIBS, then
# per-kernel times (tools/ab_kstats.sh) -> gpurun_out/$STEP/
set -euo pipefail
STEP="${STEP:-step}"
OUT="$GRAFT_REPO_ROOT/gpurun_out/$STEP"
mkdir -p "$OUT"
if [ "${TESTS:-1}" != "0" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
  tail -2 "$OUT/gpu_tests.log"
fi
bash tools/ab_all.sh ${AB_LIBS:-base} > "$OUT/ab.txt" 2>&1
cat "$OUT/ab.txt"
if [ "${KSTATS:-1}" != "0" ]; then STEP="$STEP" bash tools/ab_kstats.sh ${AB_LIBS:-base}; fi
echo done
