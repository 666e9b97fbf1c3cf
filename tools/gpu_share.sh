#!/bin/bash
# Root-share group tests + config 3/5 bench lines (regression check of the row mapping).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_frames.py tests/test_bench_cli.py -m gpu -v -rf --timeout 120 --timeout-method thread -k "group or rccl or strong or native" > gpurun_out/pytest_share.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|ERROR" gpurun_out/pytest_share.log | tail -30
[ $rc -eq 0 ] || exit $rc
for c in 3 5; do
  timeout -k 10 200 python bench.py --config $c --steps 40 --warmup 5 --no-cpu > gpurun_out/share_c$c.json 2> gpurun_out/share_c$c.err || { echo "config $c failed"; tail -5 gpurun_out/share_c$c.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/share_c$c.json'));print($c, round(d['ms_per_step'],4), 'ms serial', round(d['serial_ms_per_step'],4), round(d['value']), d['unit'])"
done
