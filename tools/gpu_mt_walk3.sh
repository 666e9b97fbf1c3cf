#!/bin/bash
# MT auto walk = all packets: MT parity tests, config 5 and 3 A/B against walk=1 (the old default), bench --mt c3.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_frames.py tests/test_gpu_parity.py -m gpu -v -rf --timeout 200 --timeout-method thread -k "mt or moller or walk" > gpurun_out/pytest_mtwalk3.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|ERROR" gpurun_out/pytest_mtwalk3.log | tail -5
[ $rc -eq 0 ] || exit $rc
L=opengl-ray-tracer_amd/lib/librtamd.so
for c in 5 2; do
  timeout -k 10 300 python tools/abf.py --mt --lib2 $L --set2 walk=1 --config $c --inflight 2 --rounds 2 --frames 20 > gpurun_out/abf_mt_c${c}_walk1.json 2> gpurun_out/abf_mt_c${c}_walk1.err || { tail -5 gpurun_out/abf_mt_c${c}_walk1.err; exit 1; }
  echo c$c; cat gpurun_out/abf_mt_c${c}_walk1.json
done
timeout -k 10 240 python bench.py --no-cpu --mt --steps 20 --warmup 3 > gpurun_out/bench_mtwalk3.json 2> gpurun_out/bench_mtwalk3.err || { tail -5 gpurun_out/bench_mtwalk3.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_mtwalk3.json')); print('mt', round(d['ms_per_step'],4), 'serial', round(d['serial_ms_per_step'],4))"
