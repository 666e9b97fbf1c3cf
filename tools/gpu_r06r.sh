#!/bin/bash
# Round 6: moving-camera cost-order policies again now that the order runs behind the waited
# frame's end (rt_sync_frame): period, dilation and split tiles on moving cost frames.
set -o pipefail
mkdir -p gpurun_out/r06r
for path in orbit dolly; do
  for rep in 1 2; do
    timeout -k 10 240 python -u tools/camera_probe.py --path $path --variants m1:1:0,m1:1:1,m2:1:0,m1:2:0,m1:0:0 \
        >> gpurun_out/r06r/probe_${path}.jsonl 2>> gpurun_out/r06r/probe.err || exit 1
  done
done
