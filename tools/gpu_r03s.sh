#!/bin/bash
# Round 3 close: GPU suite, bench lines (config 3 default; MT car; config 5) and solo profiles
# (config 3, MT car) of the final build.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_r03s.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r03s.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_r03s.json 2> gpurun_out/bench_r03s.err; rc=$?; echo "bench rc=$rc"; head -c 400 gpurun_out/bench_r03s.json; echo
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --mt --steps 40 --warmup 4 > gpurun_out/bench_r03s_mt.json 2> gpurun_out/bench_r03s_mt.err; rc=$?; echo "bench mt rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config 5 --steps 20 --warmup 3 > gpurun_out/bench_r03s_c5.json 2> gpurun_out/bench_r03s_c5.err; rc=$?; echo "bench c5 rc=$rc"
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_prof.sh r03s_c3 || exit $?
bash tools/gpu_prof.sh r03s_c3mt --mt || exit $?
