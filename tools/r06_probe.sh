#!/bin/bash
# Round 6, first GPU call (through gpurun from the repo root): the VALU issue-rate probe per instruction class
# (tools/valu_rate, built on the CPU), the bench at HEAD, and the path tail from bounce 2 against 3 on the small frames
# (the N = 4 / 8 shares of the 4K frame), two interleaved rounds.  Every GPU step has its own limit.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/r06probe"
mkdir -p "$OUT"
cd "$ROOT"
export LH2_BLUENOISE="$ROOT/lighthouse2_amd/data/bluenoise.bin"
timeout -k 10 180 "$ROOT/tools/valu_rate" > "$OUT/valu_rate.jsonl"
echo "valu done"
if [ -n "${TESTS:-1}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
  tail -1 "$OUT/gpu_tests.log"
fi
timeout -k 10 400 python3 bench.py --cpu-seconds 5 > "$OUT/bench.json" 2> "$OUT/bench.log"
echo "bench done"
for r in 1 2; do
  for v in 3 2; do
    timeout -k 10 200 python3 tools/config4_shares.py --ranks 4,8 --setting "pathTail=$v" > "$OUT/shares_pt${v}_$r.jsonl" 2> "$OUT/shares_pt${v}_$r.err"
    echo "pathTail=$v round $r: $(tr '\n' ' ' < "$OUT/shares_pt${v}_$r.jsonl")"
  done
done
echo "r06 probe done"
