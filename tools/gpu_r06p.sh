#!/bin/bash
# Round 6: rt_sync_frame (the waited frame ends at the frame event recorded before a
# latency-mode cost frame's order kernels): moving-frame exactness, then the
# moving-camera probe with the frame event off (0) and on (1), alternated.
set -o pipefail
mkdir -p gpurun_out/r06p
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_frames.py -k "moving_camera or loop" > gpurun_out/r06p/pytest.log 2>&1 || exit 1
for path in orbit dolly; do
  for m in 0 1 0 1; do
    timeout -k 10 180 python -u tools/camera_probe.py --path $path --variants m1:1:0 --frame-event $m \
        >> gpurun_out/r06p/probe_${path}.jsonl 2>> gpurun_out/r06p/probe.err || exit 1
  done
done
