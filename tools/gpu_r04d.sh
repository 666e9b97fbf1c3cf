#!/bin/bash
# Round 4, step d: own hardware queues for rt_group's slots (default now), and whether frames
# mode gains from them too (tools/group_cost.py variants); then both bench lines.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python tools/group_cost.py > gpurun_out/group_cost_r04d2.json 2> gpurun_out/group_cost_r04d2.err; rc=$?
echo "group_cost rc=$rc"; cat gpurun_out/group_cost_r04d2.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/group_cost_r04d2.err; exit $rc; }
for m in frames strong; do
  timeout -k 10 300 python bench.py --mode $m --no-cpu > gpurun_out/bench_r04d_$m.json 2> gpurun_out/bench_r04d_$m.err; rc=$?
  echo "bench $m rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_r04d_$m.err; exit $rc; }
  python -c "import json; d=json.load(open('gpurun_out/bench_r04d_$m.json')); print('  ', {k: d.get(k) for k in ('ms_per_step','serial_ms_per_step','serial_ms_per_step_latency_mode','serial_frame_ms_median','group_phases_ms')})"
done
