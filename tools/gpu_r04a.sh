#!/bin/bash
# Round 4, step a: the group/wait changes (rank 0 renders into the frame, no unstripe at
# P = 1, spinning bounded waits, F = 3 at one rank) -- the group and frame GPU tests, then
# the frames-mode and 1-rank strong-mode bench lines.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_frames.py -m gpu -x -q --timeout 240 --timeout-method thread \
  -k "group or image_rows or steady_state or rgb_format or native" > gpurun_out/pytest_r04a.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r04a.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu --steps 100 --warmup 10 > gpurun_out/bench_r04a.json 2> gpurun_out/bench_r04a.err; rc=$?
echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_r04a.err; exit $rc; }
timeout -k 10 300 python bench.py --mode strong --no-cpu --steps 100 --warmup 10 > gpurun_out/bench_r04a_strong1.json 2> gpurun_out/bench_r04a_strong1.err; rc=$?
echo "bench strong rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_r04a_strong1.err; exit $rc; }
python - <<'PY'
import json
for f in ("bench_r04a", "bench_r04a_strong1"):
    d = json.load(open(f"gpurun_out/{f}.json"))
    print(f, {k: d.get(k) for k in ("ms_per_step", "frames_in_flight", "serial_ms_per_step", "serial_ms_per_step_latency_mode",
                                     "serial_frame_ms_median", "kernel_ms_mean", "group_phases_ms", "parity")})
    print("   roofline", {k: d["roofline"].get(k) for k in ("bound", "frac", "traffic")})
PY
for c in 2 3; do
  timeout -k 10 300 python bench.py --config $c --animate --no-cpu --steps 100 --warmup 10 > gpurun_out/bench_r04a_anim_c$c.json 2> gpurun_out/bench_r04a_anim_c$c.err; rc=$?
  echo "bench animate c$c rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_r04a_anim_c$c.err; exit $rc; }
  python -c "import json; d=json.load(open('gpurun_out/bench_r04a_anim_c$c.json')); print({k: d.get(k) for k in ('ms_per_step','serial_ms_per_step','serial_frame_ms_median','parity')})"
done
