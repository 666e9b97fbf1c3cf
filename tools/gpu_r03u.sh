#!/bin/bash
# Round 3: the default bench line with 3 frames in flight at 1080p (plan_inflight), and the
# GPU tests that drive bench.py.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_bench_cli.py tests/test_gpu_frames.py -m gpu -q --timeout 240 --timeout-method thread -k "bench or steady" > gpurun_out/pytest_r03u.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/pytest_r03u.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_r03u.json 2> gpurun_out/bench_r03u.err; rc=$?; echo "bench rc=$rc"
[ $rc -eq 0 ] || exit $rc
python -c "import json; d=json.load(open('gpurun_out/bench_r03u.json')); print('F', d['frames_in_flight'], 'q', d['hw_queues'], 'ms', round(d['ms_per_step'],4), 'serial', round(d['serial_ms_per_step'],4), 'lat', round(d['serial_ms_per_step_latency_mode'],4), 'parity', d['parity'])"
