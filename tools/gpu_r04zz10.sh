#!/bin/bash
# Round 4: MT with the 1/lf bound by default -- the MT / accelerator GPU tests and the MT bench line.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "mt or MT or moller or accel or brute" > gpurun_out/pytest_r04zz10.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r04zz10.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --mt --no-cpu --steps 40 --warmup 5 > gpurun_out/bench_r04zz10_mt.json 2> gpurun_out/bench_r04zz10_mt.err || { tail -3 gpurun_out/bench_r04zz10_mt.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_r04zz10_mt.json')); print(d['ms_per_step'], d['serial_frame_ms_median'], (d.get('parity') or {}).get('ok'))"
