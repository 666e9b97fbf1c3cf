#!/bin/bash
# MT accelerator: GPU parity (accelerated == literal k_packet MT frame, oracle bands and cameras),
# then bench --mt on configs 3 and 2.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-mt}
timeout -k 10 500 python -u -m pytest tests/test_gpu_frames.py tests/test_gpu_parity.py -m gpu -v -rf --timeout 200 --timeout-method thread -k "mt or moller" > gpurun_out/pytest_$TAG.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|ERROR" gpurun_out/pytest_$TAG.log | tail -20
[ $rc -eq 0 ] || exit $rc
for c in 3 2; do
  timeout -k 10 240 python bench.py --no-cpu --mt --config $c --steps ${STEPS:-20} --warmup 3 > gpurun_out/bench_${TAG}_c$c.json 2> gpurun_out/bench_${TAG}_c$c.err || { echo "bench --mt c$c failed"; tail -5 gpurun_out/bench_${TAG}_c$c.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/bench_${TAG}_c$c.json')); print('mt c$c', round(d['ms_per_step'],4), 'serial', round(d['serial_ms_per_step'],4), d['roofline']['kernel'])"
done
# MT local leaf size A/B (build_ab/mtleaf{1,2}: tools/build_var.sh NAME -DRTA_MT_LEAF=N; current = 4)
for v in mtleaf2 mtleaf1; do
  if [ -f build_ab/$v/librtamd.so ]; then
    timeout -k 10 300 python tools/abf.py --mt --lib2 build_ab/$v/librtamd.so --config 3 --inflight 2 --rounds 2 --frames 20 > gpurun_out/abf_$v.json 2> gpurun_out/abf_$v.err || { echo "abf $v failed"; tail -5 gpurun_out/abf_$v.err; exit 1; }
    echo $v; cat gpurun_out/abf_$v.json
  fi
done
