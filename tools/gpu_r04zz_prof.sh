#!/bin/bash
# Round 4 close-out profiles: rocprofv3 passes (kernel trace, FETCH/WRITE, SQ, TCC) of the solo
# bench command for the car, config 5, the MT car and config 2 on the final build.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 bash tools/gpu_prof.sh r04zz_c3 && \
timeout -k 10 1200 bash tools/gpu_prof.sh r04zz_c5 --config 5 && \
timeout -k 10 1200 bash tools/gpu_prof.sh r04zz_mt --mt && \
timeout -k 10 900 bash tools/gpu_prof.sh r04zz_c2 --config 2
