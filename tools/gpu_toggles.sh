#!/bin/bash
# Bench lines for the reference's runtime toggles (useBVH=0, MT, Fresnel) on config 3.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r02}
for t in brute mt fresnel; do
  timeout -k 10 240 python bench.py --no-cpu --$t --steps ${STEPS:-30} --warmup 3 > gpurun_out/bench_${TAG}_$t.json 2> gpurun_out/bench_${TAG}_$t.err || { echo "bench --$t failed"; tail -5 gpurun_out/bench_${TAG}_$t.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/bench_${TAG}_$t.json')); print('$t', round(d['ms_per_step'],4), 'serial', round(d['serial_ms_per_step'],4), d['roofline']['kernel'])"
done
