#!/bin/bash
# Round 4, step v: wall-time cost order -- latency sweep 2 and in-flight A/Bs (configs 3, 5, 2).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python tools/latency_sweep.py --frames 300 --blocks 3 > gpurun_out/lat_r04v.json 2> gpurun_out/lat_r04v.err && \
timeout -k 10 300 python tools/abf.py --lib2 opengl-ray-tracer_amd/lib/librtamd.so --set2 costtime=1 --inflight 3 --rounds 3 --frames 300 --config 3 > gpurun_out/abf_r04v_c3.json 2> gpurun_out/abf_r04v_c3.err && \
timeout -k 10 300 python tools/abf.py --lib2 opengl-ray-tracer_amd/lib/librtamd.so --set2 costtime=1 --inflight 3 --rounds 3 --frames 60 --config 5 > gpurun_out/abf_r04v_c5.json 2> gpurun_out/abf_r04v_c5.err && \
timeout -k 10 300 python tools/abf.py --lib2 opengl-ray-tracer_amd/lib/librtamd.so --set2 costtime=1 --inflight 3 --rounds 3 --frames 300 --config 2 > gpurun_out/abf_r04v_c2.json 2> gpurun_out/abf_r04v_c2.err
