#!/bin/bash
# Round 4, step o: event-polled waits. Group / host-loop tests, the latency probe, waited frames
# and the driver's bench command.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "group or rccl or native or host_render or bench or latency" > gpurun_out/pytest_r04o.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r04o.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 100 ./tools/native/build/latency_probe; rc=$?; [ $rc -eq 0 ] || exit $rc
timeout -k 10 100 python tools/waited_trace.py; rc=$?; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r04o.json 2> gpurun_out/bench_r04o.err; rc=$?
echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_r04o.err; exit $rc; }
python -c "import json; d=json.load(open('gpurun_out/bench_r04o.json')); print({k: d.get(k) for k in ('ms_per_step','serial_ms_per_step_latency_mode','serial_frame_ms_median','serial_frame_ms_median_python')})"
timeout -k 10 300 python bench.py --mode strong --no-cpu > gpurun_out/bench_r04o_strong1.json 2> gpurun_out/bench_r04o_strong1.err; rc=$?
echo "bench strong rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_r04o_strong1.err; exit $rc; }
python -c "import json; d=json.load(open('gpurun_out/bench_r04o_strong1.json')); print({k: d.get(k) for k in ('ms_per_step','serial_ms_per_step','serial_frame_ms_median')})"
for v in w3 w2; do
  GPU_MAX_HW_QUEUES=6 timeout -k 10 300 python tools/abf.py --lib2 build_ab/$v/librtamd.so --config 3 --inflight 1 --set latency=1 --rounds 3 --frames 100 > gpurun_out/abf_r04o_$v.json 2> gpurun_out/abf_r04o_$v.err; rc=$?
  echo "abf latency $v rc=$rc"; cat gpurun_out/abf_r04o_$v.json; [ $rc -eq 0 ] || { tail -3 gpurun_out/abf_r04o_$v.err; exit $rc; }
done
