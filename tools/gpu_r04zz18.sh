#!/bin/bash
# Round 4 final (after the atom allocation change): the full GPU suite and the driver's default bench command on the final build.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_r04zz18.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r04zz18.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 600 python bench.py > gpurun_out/bench_r04zz18.json 2> gpurun_out/bench_r04zz18.err || { tail -5 gpurun_out/bench_r04zz18.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_r04zz18.json')); print({k: d.get(k) for k in ('ms_per_step','serial_frame_ms_median','value','steps','warmup')}, (d.get('parity') or {}).get('ok'), d['roofline']['bound'], round(d['roofline']['frac'],4))"
