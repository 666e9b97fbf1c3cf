#!/bin/bash
# MT frames: walk policies A/B (same build; lib2 runs with rt_set_walk / rt_debug_shadow_walk overrides).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
L=opengl-ray-tracer_amd/lib/librtamd.so
for s in ${SETS:-walk=0 shwalk=0 walk=2}; do
  timeout -k 10 300 python tools/abf.py --mt --lib2 $L --set2 $s --config 3 --inflight 2 --rounds 2 --frames 20 > gpurun_out/abf_mt_$s.json 2> gpurun_out/abf_mt_$s.err || { echo "abf $s failed"; tail -5 gpurun_out/abf_mt_$s.err; exit 1; }
  echo $s; cat gpurun_out/abf_mt_$s.json
done
