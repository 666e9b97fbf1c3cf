#!/bin/bash
# Round 3: per-ray Moller-Trumbore padding (accel_bound.h / accel_math.h mt_pad, mt_slab).
# MT parity subset, then MT frames A/B against HEAD's build (build_ab/head) on configs 3 and 2,
# then the production (barycentric) frame A/B on config 3 to show it did not move.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_frames.py tests/test_gpu_parity.py -m gpu -v -rf --timeout 200 --timeout-method thread -k "mt or moller" > gpurun_out/pytest_r03i_mt.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|ERROR" gpurun_out/pytest_r03i_mt.log | tail -8
[ $rc -eq 0 ] || exit $rc
for c in 3 2; do
  for f in 2 1; do
    fr=20; [ $c = 2 ] && fr=100
    echo -n "mt config $c inflight $f: "
    timeout -k 10 240 python tools/abf.py --mt --lib2 build_ab/head/librtamd.so --config $c --inflight $f --frames $fr --rounds 2 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
  done
done
echo -n "bary config 3 inflight 2: "
timeout -k 10 150 python tools/abf.py --lib2 build_ab/head/librtamd.so --config 3 --inflight 2 --frames 200 --rounds 3 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
