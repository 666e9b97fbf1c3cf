#!/bin/bash
# Round 4: MT child test with mt_pad's 1/lf bound instead of a reciprocal (RT_MT_ILF=1 build) -- A/B in flight and serially.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
timeout -k 10 400 python tools/abf.py --lib2 build_ab/mtilf/librtamd.so --mt --inflight 3 --rounds 4 --frames 60 > gpurun_out/abf_r04zz9_mt3.json 2> gpurun_out/abf_r04zz9_mt3.err && \
timeout -k 10 400 python tools/abf.py --lib2 build_ab/mtilf/librtamd.so --mt --inflight 1 --rounds 3 --frames 40 > gpurun_out/abf_r04zz9_mt1.json 2> gpurun_out/abf_r04zz9_mt1.err && \
timeout -k 10 400 python tools/abf.py --lib2 build_ab/mtilf/librtamd.so --mt --config 2 --inflight 3 --rounds 3 --frames 300 > gpurun_out/abf_r04zz9_mt_c2.json 2> gpurun_out/abf_r04zz9_mt_c2.err
rc=$?; cat gpurun_out/abf_r04zz9_*.json; exit $rc
