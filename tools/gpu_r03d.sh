#!/bin/bash
# Round 3: bench line + solo roofline profile of the current build (config 3).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > gpurun_out/bench_r03d.json 2> gpurun_out/bench_r03d.err; rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_r03d.json
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_prof.sh r03d_c3 || exit $?
bash tools/gpu_prof.sh r03d_c5 --config 5 || exit $?
