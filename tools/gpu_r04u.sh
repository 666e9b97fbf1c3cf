#!/bin/bash
# Round 4, step u: the cost order by wave wall time (latency mode sweep).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python tools/latency_sweep.py --frames 300 --blocks 3 > gpurun_out/lat_r04u.json 2> gpurun_out/lat_r04u.err
