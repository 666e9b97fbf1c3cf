#!/bin/bash
# Round 4: whole-tile cost frames -- latency-mode waited-frame states after the bench's in-flight pass (tools/waited_modes.py).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=6
timeout -k 10 500 python tools/waited_modes.py --trials 6 --blocks 10 --per 32 > gpurun_out/modes_r04z6.json 2> gpurun_out/modes_r04z6.err
