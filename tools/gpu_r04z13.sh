#!/bin/bash
# Round 4: latency mode's instance without the compaction queue's code (11 -> 4 spilled VGPRs).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "latency or heavy or cost or steady" > gpurun_out/pytest_r04z13.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r04z13.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench_r04z13_$i.json 2> gpurun_out/bench_r04z13_$i.err || { tail -3 gpurun_out/bench_r04z13_$i.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_r04z13_$i.json')); print(d['ms_per_step'], d['serial_ms_per_step_latency_mode'], d['serial_frame_ms_median'], d['serial_frame_ms_median_python'], (d.get('parity') or {}).get('ok'))"
done
