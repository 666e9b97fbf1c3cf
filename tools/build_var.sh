#!/bin/bash
# Builds librtamd.so of the working tree with extra compiler flags into
# build_ab/NAME/ (A/B with tools/abf.py --lib2 build_ab/NAME/librtamd.so).
# usage: bash tools/build_var.sh NAME "-DFLAG=..."
set -e
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/build_ab/$NAME
mkdir -p "$OUT"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off \
  -fhip-fp32-correctly-rounded-divide-sqrt -w "$@" -o "$OUT/librtamd.so" \
  "$ROOT/opengl-ray-tracer_amd/csrc/rt_kernels.hip" "$ROOT/opengl-ray-tracer_amd/csrc/rt_group.hip" \
  "$ROOT/opengl-ray-tracer_amd/csrc/lbvh.hip" "$ROOT/opengl-ray-tracer_amd/csrc/accel.cpp" -L/opt/rocm/lib -lrccl
echo "$OUT/librtamd.so"
