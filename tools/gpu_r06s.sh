#!/bin/bash
# Round 6: moving-frame exactness tests (frame event, order permutation after the wait).
set -o pipefail
mkdir -p gpurun_out/r06s
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_frames.py -k "moving_camera" > gpurun_out/r06s/pytest.log 2>&1
