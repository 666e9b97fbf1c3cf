#!/bin/bash
# Round 4: latency mode's exactness test including the 3840x2160 case over its frame-size limit.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "latency_mode_exact" > gpurun_out/pytest_r04zz17.log 2>&1; rc=$?
tail -8 gpurun_out/pytest_r04zz17.log; exit $rc
