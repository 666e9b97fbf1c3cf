#!/bin/bash
# Round 4, step q: per-tile timeline of the latency-mode car frame (busy waves over time).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python tools/tile_profile.py --config 3 --latency > gpurun_out/tiles_r04q_lat.json 2> gpurun_out/tiles_r04q_lat.err && \
timeout -k 10 240 python tools/tile_profile.py --config 3 > gpurun_out/tiles_r04q_def.json 2> gpurun_out/tiles_r04q_def.err && \
timeout -k 10 1200 bash tools/gpu_prof.sh r04q_c3
