#!/bin/bash
# Build the render core of a git revision for A/B timing: gpuvar/<name>/libRenderCore_MI355X.so
# usage: tools/build_rev.sh <name> <rev>   (the revision's csrc/ and include/ from a temporary worktree)
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
name="$1"; rev="$2"
wt="$(mktemp -d /tmp/lh2rev.XXXXXX)"
git -C "$ROOT" worktree add --detach -q "$wt" "$rev"
mkdir -p "$ROOT/gpuvar/$name"
make -s -C "$wt/lighthouse2_amd/csrc" OUT="$ROOT/gpuvar/$name/libRenderCore_MI355X.so" OBJDIR="$wt/build" -j8
git -C "$ROOT" worktree remove --force "$wt"
echo "$name: $(git -C "$ROOT" rev-parse --short "$rev")"
