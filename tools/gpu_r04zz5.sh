#!/bin/bash
# Round 4: config 5 compaction knobs under the wall-time cost order (in flight).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=6
ab() {  # name, args
  local n=$1; shift
  timeout -k 10 300 python tools/abf.py --lib2 opengl-ray-tracer_amd/lib/librtamd.so --config 5 --rounds 3 --frames 40 "$@" > gpurun_out/abf_r04zz5_$n.json 2> gpurun_out/abf_r04zz5_$n.err || { echo "$n failed"; tail -3 gpurun_out/abf_r04zz5_$n.err; exit 1; }
  echo "$n $(cat gpurun_out/abf_r04zz5_$n.json)"
}
ab tail1 --inflight 3 --set2 tail=1
ab tlanes16 --inflight 3 --set2 tlanes=16
ab tlanes48 --inflight 3 --set2 tlanes=48
ab period64 --inflight 3 --set2 period=64
