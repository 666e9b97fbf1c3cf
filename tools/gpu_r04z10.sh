#!/bin/bash
# Round 4: MT car in flight -- the cost measure, heavy-tile splits and F.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
ab() {  # name, args
  local n=$1; shift
  timeout -k 10 300 python tools/abf.py --lib2 opengl-ray-tracer_amd/lib/librtamd.so --mt --rounds 3 --frames 60 "$@" > gpurun_out/abf_r04z10_$n.json 2> gpurun_out/abf_r04z10_$n.err || { echo "$n failed"; tail -3 gpurun_out/abf_r04z10_$n.err; exit 1; }
  echo "$n $(cat gpurun_out/abf_r04z10_$n.json)"
}
ab work --inflight 3 --set2 costtime=0
ab h63x4 --inflight 3 --set2 heavy=6304
ab h127x2 --inflight 3 --set2 heavy=12702
ab latency --inflight 3 --set2 latency=1
ab f2 --inflight 2
