#!/bin/bash
# Round 4, step g: config 5 sensitivity: cones off, XCD-banded schedule (current build).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
L=opengl-ray-tracer_amd/lib/librtamd.so
for v in cone=0 schedule=2 tail=0; do
  GPU_MAX_HW_QUEUES=8 timeout -k 10 400 python tools/abf.py --lib2 $L --set2 $v --config 5 --inflight 3 --rounds 3 --frames 60 > gpurun_out/abf_r04g_$v.json 2> gpurun_out/abf_r04g_$v.err; rc=$?
  echo "$v rc=$rc"; cat gpurun_out/abf_r04g_$v.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/abf_r04g_$v.err; exit $rc; }
done
