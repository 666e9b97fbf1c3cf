#!/bin/bash
# Round 3: the barycentric car under the other walk policies (rt_set_walk: per lane from bounce
# N; 3 = all packets) against the auto policy, in flight and serially.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for w in 0 2 3; do
  for f in 2 1; do
    echo -n "walk=$w car inflight $f: "
    timeout -k 10 150 python tools/abf.py --lib2 build_ab/cur/librtamd.so --set2 walk=$w --config 3 --inflight $f --frames 200 --rounds 2 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
  done
done
