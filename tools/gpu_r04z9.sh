#!/bin/bash
# Round 4, whole-tile cost frames, record-only instances, period 16, latency split 1/200 x 4 -- full GPU suite and bench lines.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_r04z9.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r04z9.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 300 python bench.py --no-cpu --steps 20 --warmup 5 > gpurun_out/bench_r04z9_$i.json 2> gpurun_out/bench_r04z9_$i.err; rc=$?
echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_r04z9_$i.err; exit $rc; }
python -c "import json; d=json.load(open('gpurun_out/bench_r04z9_$i.json')); print({k: d.get(k) for k in ('ms_per_step','serial_ms_per_step','serial_ms_per_step_latency_mode','serial_frame_ms_median','serial_frame_ms_median_python')}, d.get('parity', {}).get('ok'))"
done
timeout -k 10 300 python bench.py --mode strong --no-cpu > gpurun_out/bench_r04z9_strong1.json 2> gpurun_out/bench_r04z9_strong1.err; rc=$?
echo "bench strong rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_r04z9_strong1.err; exit $rc; }
python -c "import json; d=json.load(open('gpurun_out/bench_r04z9_strong1.json')); print({k: d.get(k) for k in ('ms_per_step','serial_ms_per_step','serial_frame_ms_median')})"
