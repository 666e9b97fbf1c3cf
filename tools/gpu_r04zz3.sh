#!/bin/bash
# Round 4: latency mode limited to 16 tiles per wave slot -- config 4 check and the latency GPU tests.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python tools/latency_sweep.py --config 4 --frames 100 --blocks 3 > gpurun_out/lat_r04zz3_c4.json 2> gpurun_out/lat_r04zz3_c4.err && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "latency or heavy or cost or steady" > gpurun_out/pytest_r04zz3.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r04zz3.log; exit $rc
