#!/bin/bash
# Round 4: the all-packet frames' heavy split (auto: heaviest 1/256 as 8 waves) around its default under the
# wall-time order -- MT car and config 2, in flight.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
ab() {  # name, args
  local n=$1; shift
  timeout -k 10 300 python tools/abf.py --lib2 opengl-ray-tracer_amd/lib/librtamd.so --rounds 3 "$@" > gpurun_out/abf_r04zz13_$n.json 2> gpurun_out/abf_r04zz13_$n.err || { echo "$n failed"; tail -3 gpurun_out/abf_r04zz13_$n.err; exit 1; }
  echo "$n $(cat gpurun_out/abf_r04zz13_$n.json)"
}
ab mt_off --mt --inflight 3 --frames 60 --set2 heavy=1
ab c2_off --config 2 --inflight 4 --frames 400 --set2 heavy=1
ab mt_h127x4 --mt --inflight 3 --frames 60 --set2 heavy=12704
