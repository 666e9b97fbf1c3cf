#!/bin/bash
# Round 4: bench-level F = 3 vs F = 4 (alternated), and the cost-order period (16, 32) in flight.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
for f in 3 4; do
timeout -k 10 300 python bench.py --no-cpu --inflight $f > gpurun_out/bench_r04z2_f${f}_$i.json 2> gpurun_out/bench_r04z2_f${f}_$i.err || { tail -3 gpurun_out/bench_r04z2_f${f}_$i.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_r04z2_f${f}_$i.json')); print('F', d['frames_in_flight'], d['ms_per_step'], d['hw_queues'], d['serial_frame_ms_median'])"
done
done
ab() {  # name, args
  local n=$1; shift
  timeout -k 10 300 python tools/abf.py --lib2 opengl-ray-tracer_amd/lib/librtamd.so --rounds 4 --frames 400 "$@" > gpurun_out/abf_r04z2_$n.json 2> gpurun_out/abf_r04z2_$n.err || { echo "$n failed"; tail -3 gpurun_out/abf_r04z2_$n.err; exit 1; }
  echo "$n $(cat gpurun_out/abf_r04z2_$n.json)"
}
export GPU_MAX_HW_QUEUES=6
ab period16 --inflight 3 --set2 period=16
ab period32 --inflight 3 --set2 period=32
