#!/bin/bash
# Round 4, step t: latency-mode car frame timeline with the split heavy tiles' parts stamped.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python tools/tile_profile.py --config 3 --latency > gpurun_out/tiles_r04t_lat.json 2> gpurun_out/tiles_r04t_lat.err
