#!/bin/bash
# Round 4: waves per workgroup (rt_set_launch) under the wall-time order, car in flight.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=6
ab() {  # name, args
  local n=$1; shift
  timeout -k 10 300 python tools/abf.py --lib2 opengl-ray-tracer_amd/lib/librtamd.so --rounds 3 --frames 400 "$@" > gpurun_out/abf_r04zz16_$n.json 2> gpurun_out/abf_r04zz16_$n.err || { echo "$n failed"; tail -3 gpurun_out/abf_r04zz16_$n.err; exit 1; }
  echo "$n $(cat gpurun_out/abf_r04zz16_$n.json)"
}
ab launch2 --inflight 3 --set2 launch=2
ab launch1 --inflight 3 --set2 launch=1
