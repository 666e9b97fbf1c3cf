#!/bin/bash
# Round 4, step s: waited car frame over host-made dispatch orders (tools/order_probe.py).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python tools/order_probe.py --frames 300 --blocks 3 > gpurun_out/order_r04s.json 2> gpurun_out/order_r04s.err
