#!/bin/bash
# Round 4, step h: timeline of the animated car frame (rt_animate's upload + refit kernels +
# the render), one frame in flight: kernel and memory-copy traces.
set -o pipefail
mkdir -p gpurun_out/prof_r04h_anim
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/prof_r04h_anim -o run -- \
  python3 bench.py --config 3 --animate --no-cpu --inflight 1 --steps 20 --warmup 3 > gpurun_out/prof_r04h_anim/bench.json 2> gpurun_out/prof_r04h_anim/bench.err; rc=$?
echo "rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/prof_r04h_anim/bench.err; exit $rc; }
find gpurun_out/prof_r04h_anim -name "*.csv" | head
