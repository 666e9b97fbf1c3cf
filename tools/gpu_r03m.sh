#!/bin/bash
# Round 3: MT micro-optimisations (empty slots skipped, D*m1 shared; "current") against the
# r03l build (build_ab/mthead), full frames and camera-only frames (maxBounces 1).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for b in 0 1; do
  for f in 2 1; do
    echo -n "mt config 3 bounces $b inflight $f: "
    timeout -k 10 240 python tools/abf.py --mt --lib2 build_ab/mthead/librtamd.so --bounces $b --config 3 --inflight $f --frames 20 --rounds 2 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
  done
done
