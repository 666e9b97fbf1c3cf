#!/bin/bash
# Round 4, step j: host loops (plain and animated) tests, animated bench lines on the C++ loop.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "host_render_loop or anim" > gpurun_out/pytest_r04j.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r04j.log; [ $rc -eq 0 ] || exit $rc
for c in 2 3; do
  timeout -k 10 300 python bench.py --config $c --animate --no-cpu > gpurun_out/bench_r04j_anim_c$c.json 2> gpurun_out/bench_r04j_anim_c$c.err; rc=$?
  echo "bench animate c$c rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_r04j_anim_c$c.err; exit $rc; }
  python -c "import json; d=json.load(open('gpurun_out/bench_r04j_anim_c$c.json')); print({k: d.get(k) for k in ('ms_per_step','serial_ms_per_step','serial_frame_ms_median','serial_frame_ms_median_python')}, d['parity']['ok'], d['parity']['animation_frames_applied'])"
done
