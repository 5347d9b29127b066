#!/bin/bash
# Build the working tree's render core with a sed expression applied to one source file, for A/B timing:
#   tools/build_variant.sh <name> <file under lighthouse2_amd/csrc> '<sed expression>'  -> gpuab/<name>/libRenderCore_MI355X.so
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
name="$1"; file="$2"; expr="$3"
tmp="$(mktemp -d /tmp/lh2var.XXXXXX)"
mkdir -p "$tmp/lighthouse2_amd"
cp -r "$ROOT/lighthouse2_amd/csrc" "$tmp/lighthouse2_amd/"
cp -r "$ROOT/include" "$tmp/"
sed -i "$expr" "$tmp/lighthouse2_amd/csrc/$file"
if cmp -s "$ROOT/lighthouse2_amd/csrc/$file" "$tmp/lighthouse2_amd/csrc/$file"; then echo "sed changed nothing" >&2; exit 1; fi
mkdir -p "$ROOT/gpuab/$name"
make -s -C "$tmp/lighthouse2_amd/csrc" OUT="$ROOT/gpuab/$name/libRenderCore_MI355X.so" OBJDIR="$tmp/build" -j8 2>&1 | grep -v "argument unused" || true
rm -rf "$tmp"
echo "$name built"
