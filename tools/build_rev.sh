#!/bin/bash
# Builds librtamd.so of git revision REV into build_ab/REV/ (A/B against the
# working tree with tools/ab.py --lib2 build_ab/REV/librtamd.so).
set -e
REV=${1:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/build_ab/$REV
TMP=$(mktemp -d)
git -C "$ROOT" archive "$REV" opengl-ray-tracer_amd include | tar -x -C "$TMP"
make -s -C "$TMP/opengl-ray-tracer_amd" lib/librtamd.so
mkdir -p "$OUT"
cp "$TMP/opengl-ray-tracer_amd/lib/librtamd.so" "$OUT/"
rm -rf "$TMP"
echo "$OUT/librtamd.so"
