#!/bin/bash
# Round 4, step m: split heavy tiles record their parts' summed cost; exactness tests of the
# schedule / heavy / latency paths, then the lane_k latency sweep again (bimodality check).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "heavy or latency or schedule or cost or steady" > gpurun_out/pytest_r04m.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r04m.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python tools/latency_sweep.py --blocks 5 > gpurun_out/latency_sweep_r04m.json 2> gpurun_out/latency_sweep_r04m.err; rc=$?
echo "sweep rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/latency_sweep_r04m.err; exit $rc; }
python -c "
import json; d=json.load(open('gpurun_out/latency_sweep_r04m.json'))
for k,v in d['per_block'].items(): print(k, [round(x,4) for x in v])
print('images equal', all(d['image_equal'].values()))"
