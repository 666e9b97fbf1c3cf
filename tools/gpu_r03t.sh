#!/bin/bash
# Round 3: frames in flight 2/3/4 on the car (abf.py, the same build as both arms), and
# configs 2 and 4 bench lines of the final build.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for f in 2 3 4; do
  echo -n "car inflight $f: "
  timeout -k 10 150 python tools/abf.py --lib2 build_ab/cur/librtamd.so --config 3 --inflight $f --frames 300 --rounds 2 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
done
timeout -k 10 300 python bench.py --no-cpu --config 2 --steps 100 --warmup 10 > gpurun_out/bench_r03t_c2.json 2> gpurun_out/bench_r03t_c2.err || exit 1
timeout -k 10 300 python bench.py --no-cpu --config 4 --steps 50 --warmup 5 > gpurun_out/bench_r03t_c4.json 2> gpurun_out/bench_r03t_c4.err || exit 1
for c in c2 c4; do python -c "import json; d=json.load(open('gpurun_out/bench_r03t_$c.json')); print('$c', round(d['ms_per_step'],4), 'serial', round(d['serial_ms_per_step'],4), 'F', d['frames_in_flight'])"; done
