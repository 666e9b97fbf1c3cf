#!/bin/bash
# Round 4, step y: in-flight knobs under the wall-time cost order (heavy-tile splits, latency mode, F = 4).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
ab() {  # name, args
  local n=$1; shift
  timeout -k 10 300 python tools/abf.py --lib2 opengl-ray-tracer_amd/lib/librtamd.so --rounds 3 --frames 300 "$@" > gpurun_out/abf_r04y_$n.json 2> gpurun_out/abf_r04y_$n.err || { echo "$n failed"; tail -3 gpurun_out/abf_r04y_$n.err; exit 1; }
  echo "$n $(cat gpurun_out/abf_r04y_$n.json)"
}
ab h63x2 --inflight 3 --set2 heavy=6302
ab h127x2 --inflight 3 --set2 heavy=12702
ab h255x2 --inflight 3 --set2 heavy=25502
ab h63x4 --inflight 3 --set2 heavy=6304
ab latency --inflight 3 --set2 latency=1
ab f4 --inflight 4
ab period16 --inflight 3 --set2 period=16
ab period4 --inflight 3 --set2 period=4
