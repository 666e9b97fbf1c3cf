#!/bin/bash
# MT auto walk policy (walk_from: 2 for MT frames): MT parity tests, walk=3 / walk=1 A/B against auto, bench --mt.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_frames.py tests/test_gpu_parity.py -m gpu -v -rf --timeout 200 --timeout-method thread -k "mt or moller or walk" > gpurun_out/pytest_mtwalk.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|ERROR" gpurun_out/pytest_mtwalk.log | tail -5
[ $rc -eq 0 ] || exit $rc
SETS="walk=3 walk=1" bash tools/gpu_mt_walk.sh || exit 1
timeout -k 10 240 python bench.py --no-cpu --mt --steps 20 --warmup 3 > gpurun_out/bench_mtwalk.json 2> gpurun_out/bench_mtwalk.err || { tail -5 gpurun_out/bench_mtwalk.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_mtwalk.json')); print('mt', round(d['ms_per_step'],4), 'serial', round(d['serial_ms_per_step'],4))"
