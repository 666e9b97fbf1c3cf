#!/bin/bash
# Round 3: Moller-Trumbore bench lines beyond the car: config 5 (100k triangles), the
# brute-force branch on configs 3 and 5 (one-leaf tree under the MT accelerator), monkey.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { # tag args...
  local tag=$1; shift
  timeout -k 10 300 python bench.py --no-cpu "$@" > gpurun_out/bench_r03o_$tag.json 2> gpurun_out/bench_r03o_$tag.err || { echo "bench $tag failed"; tail -5 gpurun_out/bench_r03o_$tag.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_r03o_$tag.json')); print('$tag', round(d['ms_per_step'],4), 'serial', round(d['serial_ms_per_step'],4), 'parity', d.get('parity',{}).get('ok'))"
}
run c5mt --mt --config 5 --steps 20 --warmup 3 || exit 1
run c3mtbrute --mt --brute --steps 20 --warmup 3 || exit 1
run c5mtbrute --mt --brute --config 5 --steps 5 --warmup 1 || exit 1
run c2mt --mt --config 2 --steps 50 --warmup 5 || exit 1
