#!/bin/bash
# Round 3: MT frame variants against the working tree (per-ray padding, r03i): unrolled child
# loops, local leaf sizes, and the walk policy (rt_set_walk via --set2 on a copy of the build).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in mtu2 mtu4 mtleaf1 mtleaf4; do
  for f in 2 1; do
    echo -n "$v mt config 3 inflight $f: "
    timeout -k 10 240 python tools/abf.py --mt --lib2 build_ab/$v/librtamd.so --config 3 --inflight $f --frames 20 --rounds 2 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
  done
done
for w in 0 1 2; do
  for f in 2 1; do
    echo -n "walk=$w mt config 3 inflight $f: "
    timeout -k 10 240 python tools/abf.py --mt --lib2 build_ab/cur/librtamd.so --set2 walk=$w --config 3 --inflight $f --frames 20 --rounds 2 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
  done
done
