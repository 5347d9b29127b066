#!/bin/bash
# Build kernel variants of the render core for A/B timing: gpuvar/<name>/libRenderCore_MI355X.so
# usage: tools/build_variants.sh name1 "EXTRA flags 1" name2 "EXTRA flags 2" ...
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
while [ $# -ge 2 ]; do
  name="$1"; flags="$2"; shift 2
  d="$ROOT/gpuvar/$name"          # git-ignored, but travels to the GPU box (not in .gpurunignore)
  mkdir -p "$d" "$ROOT/build/var/$name"
  make -s -C "$ROOT/lighthouse2_amd/csrc" OUT="$d/libRenderCore_MI355X.so" OBJDIR="$ROOT/build/var/$name" EXTRA="$flags" -j8
  echo "$name: $flags"
done
