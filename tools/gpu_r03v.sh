#!/bin/bash
# Round 3: the MT camera bound (accel.h mt_camera_cos; "current") against the r03s build
# (build_ab/cur): MT GPU subset incl. the multi-frame camera test, then MT and barycentric A/B.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_frames.py tests/test_gpu_parity.py -m gpu -q --timeout 200 --timeout-method thread -k "mt or moller or camera_bound" > gpurun_out/pytest_r03v_mt.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 gpurun_out/pytest_r03v_mt.log
[ $rc -eq 0 ] || exit $rc
for f in 2 1; do
  echo -n "mt config 3 inflight $f: "
  timeout -k 10 240 python tools/abf.py --mt --lib2 build_ab/cur/librtamd.so --config 3 --inflight $f --frames 30 --rounds 2 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
done
echo -n "mt config 2 inflight 2: "
timeout -k 10 240 python tools/abf.py --mt --lib2 build_ab/cur/librtamd.so --config 2 --inflight 2 --frames 100 --rounds 2 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
echo -n "bary config 3 inflight 2: "
timeout -k 10 150 python tools/abf.py --lib2 build_ab/cur/librtamd.so --config 3 --inflight 2 --frames 200 --rounds 2 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
