#!/bin/bash
# GPU tests, then throughput A/B (2 frames in flight) and per-dispatch A/B against build_ab/REV.
set -o pipefail
REV=$1; CFGS=${2:-"3 5"}
bash tools/gpu_tests.sh || exit 1
for c in $CFGS; do
  timeout -k 10 200 python tools/abf.py --lib2 build_ab/$REV/librtamd.so --config $c 2>&1 | grep -v amdgpu.ids || exit 1
done
bash tools/gpu_abrev.sh $REV "$CFGS" default,default@2
