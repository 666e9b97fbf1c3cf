#!/bin/bash
# Round 4, step i: rt_animate as two launches (k_animate reading the pinned host buffer, then
# k_anim_refit with write-through): animation GPU tests, animated bench lines, timeline.
set -o pipefail
mkdir -p gpurun_out/prof_r04i_anim
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "anim or refit or update_bvh or lbvh" > gpurun_out/pytest_r04i.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r04i.log; [ $rc -eq 0 ] || exit $rc
for c in 2 3; do
  timeout -k 10 300 python bench.py --config $c --animate --no-cpu > gpurun_out/bench_r04i_anim_c$c.json 2> gpurun_out/bench_r04i_anim_c$c.err; rc=$?
  echo "bench animate c$c rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_r04i_anim_c$c.err; exit $rc; }
  python -c "import json; d=json.load(open('gpurun_out/bench_r04i_anim_c$c.json')); print({k: d.get(k) for k in ('ms_per_step','serial_ms_per_step','serial_frame_ms_median')}, d['parity']['ok'], d['parity']['max_abs'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/prof_r04i_anim -o run -- \
  python3 bench.py --config 3 --animate --no-cpu --inflight 1 --steps 20 --warmup 3 > gpurun_out/prof_r04i_anim/bench.json 2> gpurun_out/prof_r04i_anim/bench.err; rc=$?
echo "trace rc=$rc"
