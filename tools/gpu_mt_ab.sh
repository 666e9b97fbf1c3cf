#!/bin/bash
# MT local build A/B: every build_ab/mt*/librtamd.so against the working tree (tools/abf.py --mt, config 3).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for d in build_ab/mt*/; do
  v=$(basename $d)
  timeout -k 10 300 python tools/abf.py --mt --lib2 $d/librtamd.so --config 3 --inflight 2 --rounds 2 --frames 20 > gpurun_out/abf_$v.json 2> gpurun_out/abf_$v.err || { echo "abf $v failed"; tail -5 gpurun_out/abf_$v.err; exit 1; }
  echo $v; cat gpurun_out/abf_$v.json
done
