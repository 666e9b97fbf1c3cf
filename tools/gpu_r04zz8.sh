#!/bin/bash
# Round 4: split walks under the wall-time order (latency sweep, car).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python tools/latency_sweep.py --config 3 --frames 300 --blocks 3 > gpurun_out/lat_r04zz8_c3.json 2> gpurun_out/lat_r04zz8_c3.err
