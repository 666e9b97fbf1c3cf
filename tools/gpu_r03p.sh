#!/bin/bash
# Round 3: where the car frame's time goes by bounce (maxBounces 1/2/3, abf.py, the same build
# as both arms), and the MT car with 3 frames in flight.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for b in 1 2 3; do
  for f in 2 1; do
    echo -n "car bounces $b inflight $f: "
    timeout -k 10 150 python tools/abf.py --lib2 build_ab/cur/librtamd.so --bounces $b --config 3 --inflight $f --frames 200 --rounds 2 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
  done
done
for f in 3 4; do
  echo -n "mt car inflight $f: "
  timeout -k 10 240 python tools/abf.py --mt --lib2 build_ab/cur/librtamd.so --config 3 --inflight $f --frames 20 --rounds 2 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
done
