#!/bin/bash
# Build the product library of a git revision (default HEAD) as lib/libslam2d_<name>.so for same-box A/B
# runs (tools/ab_bench.sh).  usage: tools/build_variant.sh <name> [rev] [EXTRA hipcc flags]
set -e
NAME=$1; REV=${2:-HEAD}; EXTRA=${3:-}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
git -C "$ROOT" archive "$REV" creating-2d-laser-slam-from-scratch_amd/csrc include | tar -x -C "$TMP"
make -s -C "$TMP/creating-2d-laser-slam-from-scratch_amd/csrc" OUT="$ROOT/creating-2d-laser-slam-from-scratch_amd/lib/libslam2d_$NAME.so" EXTRA="$EXTRA"
rm -rf "$TMP"
echo "built lib/libslam2d_$NAME.so from $REV"
