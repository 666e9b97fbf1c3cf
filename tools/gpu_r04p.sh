#!/bin/bash
# Round 4, step p: group waits marking only dirty streams; group tests and the 1-rank strong line.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "group or rccl or native or bench" > gpurun_out/pytest_r04p.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r04p.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 300 python bench.py --mode strong --no-cpu > gpurun_out/bench_r04p_strong1_$i.json 2> gpurun_out/bench_r04p_strong1_$i.err; rc=$?
echo "bench strong rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_r04p_strong1_$i.err; exit $rc; }
python -c "import json; d=json.load(open('gpurun_out/bench_r04p_strong1_$i.json')); print({k: d.get(k) for k in ('ms_per_step','serial_ms_per_step','serial_frame_ms_median')})"
timeout -k 10 300 python bench.py --no-cpu --steps 20 --warmup 5 > gpurun_out/bench_r04p_$i.json 2> gpurun_out/bench_r04p_$i.err; rc=$?
echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_r04p_$i.err; exit $rc; }
python -c "import json; d=json.load(open('gpurun_out/bench_r04p_$i.json')); print({k: d.get(k) for k in ('ms_per_step','serial_ms_per_step_latency_mode','serial_frame_ms_median','serial_frame_ms_median_python')})"
done
