#!/bin/bash
# GPU parity tests, then A/B timing of k_accel variants on configs 3 and 5.
# usage: bash tools/gpu_ab.sh TAG [variants]
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-ab}
VAR=${2:-default,lane_all,packet_all,hybrid_w2}
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q -rf > gpurun_out/pytest_$TAG.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
for c in 3 5; do
  timeout -k 10 300 python tools/ab.py --config $c --rounds 3 --frames 20 --variants $VAR --times > gpurun_out/ab_${TAG}_c$c.txt 2>&1 || exit 1
  grep -v amdgpu.ids gpurun_out/ab_${TAG}_c$c.txt | head -12
done
