#!/bin/bash
# Round 3 close: the strong-mode path the driver's N > 1 runs take (rt_group over RCCL, frame
# slots on one communicator, self-check against the single-GPU frame), here with one rank.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --mode strong --no-cpu --steps 50 --warmup 5 > gpurun_out/bench_r03w_strong1.json 2> gpurun_out/bench_r03w_strong1.err; rc=$?; echo "bench strong rc=$rc"
[ $rc -eq 0 ] || { tail -5 gpurun_out/bench_r03w_strong1.err; exit $rc; }
python -c "import json; d=json.load(open('gpurun_out/bench_r03w_strong1.json')); print({k: d.get(k) for k in ('ms_per_step','frames_in_flight','scaling','gather','group_phases_ms','self_check')})"
