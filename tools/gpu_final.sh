#!/bin/bash
# Final check of a snapshot: smoke, the whole GPU suite, the default bench line, MT bench lines (configs 3, 5).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-final}
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 200 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|ERROR" gpurun_out/pytest_$TAG.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -5 gpurun_out/bench_$TAG.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_$TAG.json')); print('default', round(d['ms_per_step'],4), 'serial', round(d['serial_ms_per_step'],4), round(d['value']))"
for c in 3 5; do
  timeout -k 10 240 python bench.py --no-cpu --mt --config $c --steps 20 --warmup 3 > gpurun_out/bench_${TAG}_mt_c$c.json 2> gpurun_out/bench_${TAG}_mt_c$c.err || { tail -5 gpurun_out/bench_${TAG}_mt_c$c.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_${TAG}_mt_c$c.json')); print('mt c$c', round(d['ms_per_step'],4), 'serial', round(d['serial_ms_per_step'],4))"
done
