#!/bin/bash
# A/B of the current build against a second build (build_ab/*.so) on configs 3 and 5.
# usage: bash tools/gpu_ab2.sh TAG LIB2 VARIANTS [CONFIGS]
set -o pipefail
mkdir -p gpurun_out
TAG=$1; LIB2=$2; VAR=$3; CFGS=${4:-"3 5"}
export TMPDIR=/tmp
for c in $CFGS; do
  timeout -k 10 300 python tools/ab.py --config $c --rounds 4 --frames 20 --variants $VAR --lib2 $LIB2 > gpurun_out/ab2_${TAG}_c$c.txt 2>&1 || { tail -5 gpurun_out/ab2_${TAG}_c$c.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/ab2_${TAG}_c$c.txt
done
