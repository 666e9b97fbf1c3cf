#!/bin/bash
# A/B of experiment builds in latency mode (rt_set_latency_mode on both arms), serial frames.
set -o pipefail
for n in $1; do
  for c in ${2:-3}; do
    echo -n "$n config $c latency mode serial: "
    timeout -k 10 150 python tools/abf.py --lib2 build_ab/$n/librtamd.so --config $c --inflight 1 --frames 200 --rounds 3 --set latency=1 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
  done
done
