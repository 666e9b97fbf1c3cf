#!/bin/bash
# Round 4, step e: latency knob sweep (car, waited frames) and the octant-sorted tail A/B (config 5).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python tools/latency_sweep.py --blocks 4 > gpurun_out/latency_sweep_r04e.json 2> gpurun_out/latency_sweep_r04e.err; rc=$?
echo "sweep rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/latency_sweep_r04e.err; exit $rc; }
python -c "import json; d=json.load(open('gpurun_out/latency_sweep_r04e.json')); print(sorted(((round(v,4),k) for k,v in d['waited_ms'].items()))); print('images equal', all(d['image_equal'].values()))"
GPU_MAX_HW_QUEUES=6 timeout -k 10 400 python tools/abf.py --lib2 build_ab/tailsort/librtamd.so --config 5 --inflight 3 --rounds 3 --frames 60 > gpurun_out/abf_r04e_tailsort.json 2> gpurun_out/abf_r04e_tailsort.err; rc=$?
echo "abf tailsort rc=$rc"; cat gpurun_out/abf_r04e_tailsort.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/abf_r04e_tailsort.err; exit $rc; }
GPU_MAX_HW_QUEUES=6 timeout -k 10 400 python tools/abf.py --lib2 build_ab/tailsort/librtamd.so --config 5 --inflight 1 --rounds 3 --frames 40 > gpurun_out/abf_r04e_tailsort1.json 2> gpurun_out/abf_r04e_tailsort1.err; rc=$?
echo "abf tailsort serial rc=$rc"; cat gpurun_out/abf_r04e_tailsort1.json
