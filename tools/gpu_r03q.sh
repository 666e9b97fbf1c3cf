#!/bin/bash
# Round 3: MT per-ray padding with Z at the centre of the bulk triangles (the road quad no
# longer drags it 23 units off the car; "current") against the r03l build (build_ab/cur).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_frames.py tests/test_gpu_parity.py -m gpu -q --timeout 200 --timeout-method thread -k "mt or moller" > gpurun_out/pytest_r03q_mt.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 gpurun_out/pytest_r03q_mt.log
[ $rc -eq 0 ] || exit $rc
for c in 3 5 2; do
  for f in 2 1; do
    fr=20; [ $c = 2 ] && fr=100; [ $c = 5 ] && fr=10
    echo -n "mt config $c inflight $f: "
    timeout -k 10 240 python tools/abf.py --mt --lib2 build_ab/cur/librtamd.so --config $c --inflight $f --frames $fr --rounds 2 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
  done
done
