#!/bin/bash
# Round 4: whole-tile cost frames -- latency-mode split-set sizes (tools/latency_sweep.py).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python tools/latency_sweep.py --frames 300 --blocks 3 > gpurun_out/lat_r04z7.json 2> gpurun_out/lat_r04z7.err
