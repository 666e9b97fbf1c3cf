#!/bin/bash
# Round 4: bench after the bounded waited warm-up -- default command and config 5.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --no-cpu > gpurun_out/bench_r04zz15.json 2> gpurun_out/bench_r04zz15.err || { tail -5 gpurun_out/bench_r04zz15.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_r04zz15.json')); print(d['ms_per_step'], d['serial_frame_ms_median'], (d.get('parity') or {}).get('ok'))"
timeout -k 10 600 python bench.py --config 5 --no-cpu --steps 30 --warmup 5 > gpurun_out/bench_r04zz15_c5.json 2> gpurun_out/bench_r04zz15_c5.err || { tail -5 gpurun_out/bench_r04zz15_c5.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_r04zz15_c5.json')); print(d['ms_per_step'], d['serial_frame_ms_median'], (d.get('parity') or {}).get('ok'))"
