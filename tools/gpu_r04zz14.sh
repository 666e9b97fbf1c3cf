#!/bin/bash
# Round 4: tile / part / slot forced into SGPRs in every k_accel instance (RT_UNIFORM_TILE=1 build), in flight.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=6
timeout -k 10 300 python tools/abf.py --lib2 build_ab/utile/librtamd.so --inflight 3 --rounds 4 --frames 400 > gpurun_out/abf_r04zz14_c3.json 2> gpurun_out/abf_r04zz14_c3.err && \
timeout -k 10 300 python tools/abf.py --lib2 build_ab/utile/librtamd.so --config 2 --inflight 3 --rounds 3 --frames 400 > gpurun_out/abf_r04zz14_c2.json 2> gpurun_out/abf_r04zz14_c2.err
rc=$?; cat gpurun_out/abf_r04zz14_*.json; exit $rc
