#!/bin/bash
# Round 6 final: smoke + the GPU suite, the driver's default bench command, and the
# moving-camera / animated lines after rt_sync_frame.
set -o pipefail
mkdir -p gpurun_out/r06q
export TMPDIR=/tmp
bash tools/gpu_tests.sh > gpurun_out/r06q/tests.out 2>&1 || { tail -20 gpurun_out/r06q/tests.out; exit 1; }
cp gpurun_out/pytest_gpu.log gpurun_out/smoke.log gpurun_out/r06q/
timeout -k 10 300 python bench.py > gpurun_out/r06q/bench_default.json 2> gpurun_out/r06q/bench_default.err || exit 1
for cp in orbit dolly; do
  timeout -k 10 300 python bench.py --steps 100 --camera-path $cp > gpurun_out/r06q/bench_$cp.json 2> gpurun_out/r06q/bench_$cp.err || exit 1
done
timeout -k 10 300 python bench.py --steps 100 --animate --camera-path orbit > gpurun_out/r06q/bench_anim_orbit.json 2> gpurun_out/r06q/bench_anim_orbit.err || exit 1
