#!/bin/bash
# one A/B step through gpurun: GPU suite, then tools/ab_all.sh against the gpuab/ builds named in AB_LIBS,
# then SQ counters of the bounce launch (in-tree library) -> gpurun_out/$STEP/
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
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE -f csv -d "$OUT/sq1" -o run -- python3 "$GRAFT_REPO_ROOT/tools/trace_kernel_bench.py" --set bounce --iters 5 > "$OUT/sq1.log" 2>&1
echo done
