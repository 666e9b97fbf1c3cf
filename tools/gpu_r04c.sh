#!/bin/bash
# Round 4, step c: is the 1-rank strong line's gap hardware-queue sharing? The strong bench
# with the default 6 queues, with 16, and with CU-masked (own-queue) streams.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # tag, env..., then bench args after --
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --mode strong --no-cpu > gpurun_out/bench_r04c_$tag.json 2> gpurun_out/bench_r04c_$tag.err; local rc=$?
  echo "$tag rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_r04c_$tag.err; exit $rc; }
  python -c "import json; d=json.load(open('gpurun_out/bench_r04c_$tag.json')); print('  ', {k: d.get(k) for k in ('ms_per_step','serial_ms_per_step','serial_frame_ms_median','hw_queues')})"
}
run q6 GPU_MAX_HW_QUEUES=4
run q16 GPU_MAX_HW_QUEUES=16
run cumask GPU_MAX_HW_QUEUES=4 RT_STREAMS_CUMASK=1
run q6b GPU_MAX_HW_QUEUES=4
