#!/bin/bash
# Round 3: GPU suite + bench line + solo profiles of the current build.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_r03f.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r03f.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_r03f.json 2> gpurun_out/bench_r03f.err; rc=$?; echo "bench rc=$rc"; head -c 700 gpurun_out/bench_r03f.json
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_prof.sh r03f_c3 || exit $?
bash tools/gpu_prof.sh r03f_c5 --config 5 || exit $?
