#!/bin/bash
# Round 3, first GPU call: smoke, the GPU suite, the default bench line, and the
# brute-force MT walk-policy A/B on config 5.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/smoke.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rf --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|ERROR" gpurun_out/pytest_gpu.log | tail -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_r03a.json 2> gpurun_out/bench_r03a.err; rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_r03a.json
[ $rc -eq 0 ] || exit $rc
for w in -1 1 3; do
  timeout -k 10 200 python bench.py --config 5 --brute --mt --no-cpu --steps 20 --warmup 3 --walk $w > gpurun_out/bench_r03a_c5_brute_mt_walk$w.json 2>> gpurun_out/bench_r03a.err || exit $?
done
grep -ho '"ms_per_step": [0-9.]*\|"walk": [-0-9]*' gpurun_out/bench_r03a_c5_brute_mt_walk*.json
bash tools/gpu_prof.sh r03a_c3 || exit $?
