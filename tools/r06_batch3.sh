#!/bin/bash
# Round 6, third GPU call (through gpurun from the repo root): the GPU suite on the finish-behind schedule (small lit frames'
# shadow launches and finalize on the side stream, RenderCore::kFinishBehind), then an A/B of the N = 1 / 8 config-4 shares
# and config 3 against gpuab/nobehind (-DLH2_FINISH_BEHIND=0) and gpuab/chainprio (-DLH2_CHAIN_PRIORITY=1), two interleaved
# rounds, gpuab/bfsorder (-DLH2_BVH4_ORDER=0: the breadth-first BVH4 node order), and the N = 8 share's kernel timeline.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/r06c"
mkdir -p "$OUT"
cd "$ROOT"
export LH2_BLUENOISE="$ROOT/lighthouse2_amd/data/bluenoise.bin"
if [ -n "${TESTS:-1}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
  tail -1 "$OUT/gpu_tests.log"
fi
for r in 1 2; do
  for v in main nobehind chainprio bfsorder; do
    lib="$ROOT/lighthouse2_amd/libRenderCore_MI355X.so"; [ "$v" != main ] && lib="$ROOT/gpuab/$v/libRenderCore_MI355X.so"
    LH2_CORE_LIB="$lib" timeout -k 10 200 python3 tools/config4_shares.py --ranks 1,8 > "$OUT/shares_${v}_$r.jsonl" 2> "$OUT/shares_${v}_$r.err"
    LH2_CORE_LIB="$lib" timeout -k 10 200 python3 tools/bench_configs.py --configs 3,5 > "$OUT/c3_${v}_$r.json" 2> "$OUT/c3_${v}_$r.err"
    python3 - "$OUT/shares_${v}_$r.jsonl" "$OUT/c3_${v}_$r.json" "$v $r" <<'PY'
import json, sys
sh = [json.loads(l) for l in open(sys.argv[1]) if l.strip()]
cs = [json.loads(l) for l in open(sys.argv[2]) if l.strip().startswith("{")]
c3 = [c for c in cs if c.get("config") == "config3"][-1]
c5 = [c for c in cs if c.get("config") == "config5"][-1]
print(sys.argv[3], "shares", [s["ms_per_frame"] for s in sh], "ratio", round(sh[0]["ms_per_frame"] / sh[-1]["ms_per_frame"], 3),
      "| c3", c3["ms_per_frame"], {k: c3[k] for k in ("traceTime0_ms", "traceTime1_ms", "traceTimeX_ms", "shadowTraceTime_ms", "shadeTime_ms")}, "| c5", c5["ms_per_frame"], flush=True)
PY
  done
done
bash tools/share_timeline.sh 8 > "$OUT/share8.txt" 2>&1
cp gpurun_out/share8/timeline.txt "$OUT/share8_timeline.txt"
tail -3 "$OUT/share8_timeline.txt"
echo "r06 batch3 done"
