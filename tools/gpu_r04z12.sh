#!/bin/bash
# Round 4: the heaviest slots' camera rays (and shadows) per lane under the wall-time order --
# in flight (abf) and waited (latency sweep).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python tools/latency_sweep.py --frames 300 --blocks 3 > gpurun_out/lat_r04z12.json 2> gpurun_out/lat_r04z12.err || exit 1
export GPU_MAX_HW_QUEUES=6
ab() {  # name, args
  local n=$1; shift
  timeout -k 10 300 python tools/abf.py --lib2 opengl-ray-tracer_amd/lib/librtamd.so --rounds 3 --frames 300 "$@" > gpurun_out/abf_r04z12_$n.json 2> gpurun_out/abf_r04z12_$n.err || { echo "$n failed"; tail -3 gpurun_out/abf_r04z12_$n.err; exit 1; }
  echo "$n $(cat gpurun_out/abf_r04z12_$n.json)"
}
ab lanek128m3 --inflight 3 --set2 lanek=1283
ab lanek648m3 --inflight 3 --set2 lanek=6483
ab lanek648m1 --inflight 3 --set2 lanek=6481
ab lanek0 --inflight 3 --set2 lanek=0
