#!/bin/bash
# VGPR / SGPR / spill / LDS usage of the core's kernels, from the gfx950 code object in build/obj/lh2_kernels.o
# (host tool, no GPU): bash tools/kernel_resources.sh [object]
set -euo pipefail
OBJ="${1:-$(cd "$(dirname "$0")/.." && pwd)/build/obj/lh2_kernels.o}"
B=/opt/rocm/lib/llvm/bin
T="$(mktemp -d)"
$B/llvm-objcopy --dump-section=.hip_fatbin="$T/fat.bin" "$OBJ"
$B/clang-offload-bundler --unbundle --type=o --input="$T/fat.bin" --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output="$T/k.co"
$B/llvm-readelf --notes "$T/k.co" | python3 -c '
import sys, re
cur = {}
rows = []
for line in sys.stdin:
    # a kernel record starts with "- .<first key>" (keys are sorted: .group_segment_fixed_size precedes .name)
    if re.match(r"\s*-\s+\.", line) and cur.get("name"):
        rows.append(cur)
        cur = {}
    m = re.match(r"\s*-?\s*\.(name|vgpr_count|sgpr_count|vgpr_spill_count|sgpr_spill_count|group_segment_fixed_size|private_segment_fixed_size|agpr_count):\s+(.*)", line)
    if not m: continue
    cur[m.group(1)] = m.group(2).strip()
if cur: rows.append(cur)
for r in rows:
    if "vgpr_count" not in r: continue
    g = lambda k: r.get(k, "0")
    print("%4s vgpr %3s agpr %4s sgpr spill v%s/s%s scratch %4s lds %6s  %s" % (g("vgpr_count"), g("agpr_count"), g("sgpr_count"),
          g("vgpr_spill_count"), g("sgpr_spill_count"), g("private_segment_fixed_size"), g("group_segment_fixed_size"), r["name"]))
'
rm -rf "$T"
