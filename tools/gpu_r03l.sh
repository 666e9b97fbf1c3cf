#!/bin/bash
# Round 3: GPU suite, bench lines (config 3 default; MT car; config 5) and solo profiles
# (configs 3 and 5, MT car) of the current build.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_r03l.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r03l.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_r03l.json 2> gpurun_out/bench_r03l.err; rc=$?; echo "bench rc=$rc"; head -c 600 gpurun_out/bench_r03l.json; echo
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --mt --steps 20 --warmup 3 > gpurun_out/bench_r03l_mt.json 2> gpurun_out/bench_r03l_mt.err; rc=$?; echo "bench mt rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config 5 --steps 20 --warmup 3 > gpurun_out/bench_r03l_c5.json 2> gpurun_out/bench_r03l_c5.err; rc=$?; echo "bench c5 rc=$rc"
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_prof.sh r03l_c3 || exit $?
bash tools/gpu_prof.sh r03l_c5 --config 5 || exit $?
bash tools/gpu_prof.sh r03l_c3mt --mt || exit $?
