#!/bin/bash
# Round 6: the cost order's kernels on an order stream (rt_debug_order_stream): exactness
# of moving frames in each mode, then the moving-camera probe with the order on the
# context's stream (0) and on the order stream in latency mode (1).
set -o pipefail
mkdir -p gpurun_out/r06o
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_frames.py -k "moving_camera" > gpurun_out/r06o/pytest.log 2>&1 || exit 1
for path in orbit dolly; do
  for m in 0 1 0 1; do
    timeout -k 10 180 python -u tools/camera_probe.py --path $path --variants m1:1:0 --order-stream $m \
        >> gpurun_out/r06o/probe_${path}.jsonl 2>> gpurun_out/r06o/probe.err || exit 1
  done
done
