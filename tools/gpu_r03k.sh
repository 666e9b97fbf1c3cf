#!/bin/bash
# Round 3: MT per-ray padding with v_rcp_f32 in place of IEEE divisions (current) against
# the unrolled-division build (build_ab/mtu4); configs 3 and 2, images compared.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in 3 2; do
  for f in 2 1; do
    fr=20; [ $c = 2 ] && fr=100
    echo -n "mt config $c inflight $f: "
    timeout -k 10 240 python tools/abf.py --mt --lib2 build_ab/mtu4/librtamd.so --config $c --inflight $f --frames $fr --rounds 2 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
  done
done
