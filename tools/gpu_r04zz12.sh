#!/bin/bash
# Round 4: the all-packet frames' heavy split (auto: heaviest 1/256 as 8 waves) around its default under the
# wall-time order -- MT car and config 2, in flight.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
ab() {  # name, args
  local n=$1; shift
  timeout -k 10 300 python tools/abf.py --lib2 opengl-ray-tracer_amd/lib/librtamd.so --rounds 3 "$@" > gpurun_out/abf_r04zz12_$n.json 2> gpurun_out/abf_r04zz12_$n.err || { echo "$n failed"; tail -3 gpurun_out/abf_r04zz12_$n.err; exit 1; }
  echo "$n $(cat gpurun_out/abf_r04zz12_$n.json)"
}
ab mt_h63x8 --mt --inflight 3 --frames 60 --set2 heavy=6308
ab mt_h255x8 --mt --inflight 3 --frames 60 --set2 heavy=25508
ab mt_h511x8 --mt --inflight 3 --frames 60 --set2 heavy=51108
ab c2_h63x8 --config 2 --inflight 4 --frames 400 --set2 heavy=6308
ab c2_h255x8 --config 2 --inflight 4 --frames 400 --set2 heavy=25508
