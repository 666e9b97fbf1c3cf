#!/bin/bash
# Round 4: the record-only k_accel instances (wall-time costs without walk counters) -- cost-order
# periods in flight, the latency sweep's default, and the schedule/cost GPU tests.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "schedule or heavy or latency or steady or cost or lane_k or mt" > gpurun_out/pytest_r04z4.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r04z4.log; [ $rc -eq 0 ] || exit $rc
ab() {  # name, args
  local n=$1; shift
  timeout -k 10 300 python tools/abf.py --lib2 opengl-ray-tracer_amd/lib/librtamd.so --rounds 4 --frames 400 "$@" > gpurun_out/abf_r04z4_$n.json 2> gpurun_out/abf_r04z4_$n.err || { echo "$n failed"; tail -3 gpurun_out/abf_r04z4_$n.err; exit 1; }
  echo "$n $(cat gpurun_out/abf_r04z4_$n.json)"
}
export GPU_MAX_HW_QUEUES=6
ab period4 --inflight 3 --set2 period=4
ab period2 --inflight 3 --set2 period=2
ab period64 --inflight 3 --set2 period=64
for i in 1 2; do
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench_r04z4_$i.json 2> gpurun_out/bench_r04z4_$i.err || { tail -3 gpurun_out/bench_r04z4_$i.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_r04z4_$i.json')); print(d['ms_per_step'], d['serial_frame_ms_median'], d['serial_frame_ms_median_python'], (d.get('parity') or {}).get('ok'))"
done
