#!/bin/bash
# Round 6 library A/B through gpurun: the in-tree library ("new") against variant builds gpuab/<name>/ (tools/build_variant.sh).
# Optionally the GPU suite on "new" first (SUITE=1).  Then REPS interleaved rounds of, per library: config 3 and (C5=1)
# config 5 (tools/bench_configs.py), the config-4 rank shares N = 1 and 8 (tools/config4_shares.py) and config 2
# (bench.py, no CPU baseline / config 4 / other configs).  One line per library and round.
# usage: SUITE=1 REPS=2 bash tools/r06_ablib.sh name[:setting=value]...   (new = the in-tree library)
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-r06ab}"
mkdir -p "$OUT"
cd "$ROOT"
export LH2_BLUENOISE="$ROOT/lighthouse2_amd/data/bluenoise.bin"
if [ -n "${SUITE:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${SUITE_K:+-k "$SUITE_K"} > "$OUT/gpu_tests.log" 2>&1
  tail -1 "$OUT/gpu_tests.log"
fi
cfgs=3; [ -n "${C5:-}" ] && cfgs=3,5
for rep in $(seq 1 "${REPS:-2}"); do
  for v in ${BASE-new} "$@"; do
    lib="${v%%:*}"; sa=(); [ "$lib" != "$v" ] && sa=(--setting "${v#*:}")
    if [ "$lib" = new ]; then unset LH2_CORE_LIB; else export LH2_CORE_LIB="$ROOT/gpuab/$lib/libRenderCore_MI355X.so"; fi
    v="${v//[:=,]/_}"
    timeout -k 10 300 python3 tools/bench_configs.py --configs $cfgs "${sa[@]}" > "$OUT/c_${v}_$rep.json" 2> "$OUT/c_${v}_$rep.err"
    timeout -k 10 200 python3 tools/config4_shares.py --ranks 1,8 "${sa[@]}" > "$OUT/sh_${v}_$rep.jsonl" 2> "$OUT/sh_${v}_$rep.err"
    timeout -k 10 180 python3 bench.py --no-cpu-baseline --no-config4 --no-configs --steps 30 "${sa[@]}" > "$OUT/b_${v}_$rep.json" 2> "$OUT/b_${v}_$rep.err"
    python3 - "$OUT" "$v" "$rep" <<'PY'
import json, sys
out, v, rep = sys.argv[1:4]
cs = {}
for l in open(f"{out}/c_{v}_{rep}.json"):
    if l.startswith("{"):
        d = json.loads(l); cs[d["config"]] = d
sh = [json.loads(l) for l in open(f"{out}/sh_{v}_{rep}.jsonl") if l.strip()]
b = [json.loads(l) for l in open(f"{out}/b_{v}_{rep}.json") if l.startswith("{")][-1]
line = f"{v:22s} r{rep} c2 {b['value']:.1f} {b['ms_per_step']:.4f} trace1 {b['detail']['traceTime1_ms']}"
for k, d in cs.items():
    line += f" | {k} {d['ms_per_frame']} shadow {d.get('shadowTraceTime_ms')}"
line += " | shares " + " ".join(f"N{s['ranks']} {s['ms_per_frame']:.4f}" for s in sh) + f" ratio {sh[0]['ms_per_frame'] / sh[-1]['ms_per_frame']:.3f}"
print(line, flush=True)
PY
  done
done
echo "r06 ablib done"
