#!/bin/bash
# A/B of variants of the current build on the given configs (no second build).
# usage: bash tools/gpu_ab3.sh TAG VARIANTS [CONFIGS]
set -o pipefail
mkdir -p gpurun_out
TAG=$1; VAR=$2; CFGS=${3:-"3 5"}
export TMPDIR=/tmp
for c in $CFGS; do
  timeout -k 10 300 python tools/ab.py --config $c --rounds 4 --frames 20 --variants $VAR > gpurun_out/ab3_${TAG}_c$c.txt 2>&1 || { tail -5 gpurun_out/ab3_${TAG}_c$c.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/ab3_${TAG}_c$c.txt
done
