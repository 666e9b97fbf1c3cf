#!/bin/bash
# Round 4: latency mode on big frames (config 4 at 4K, config 5) against the default mode.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python tools/latency_sweep.py --config 4 --frames 100 --blocks 3 > gpurun_out/lat_r04zz2_c4.json 2> gpurun_out/lat_r04zz2_c4.err && \
timeout -k 10 500 python tools/latency_sweep.py --config 5 --frames 40 --blocks 3 > gpurun_out/lat_r04zz2_c5.json 2> gpurun_out/lat_r04zz2_c5.err
timeout -k 10 400 python tools/latency_sweep.py --config 2 --frames 300 --blocks 3 > gpurun_out/lat_r04zz2_c2.json 2> gpurun_out/lat_r04zz2_c2.err
