#!/bin/bash
# A/B of the working tree against a built revision (tools/build_rev.sh REV).
# usage: bash tools/gpu_abrev.sh REV "CONFIGS" VARIANTS
set -o pipefail
mkdir -p gpurun_out
REV=${1:-HEAD}; CFGS=${2:-"3 5 2"}; VAR=${3:-default,default@2,reftree}
for c in $CFGS; do
  timeout -k 10 240 python tools/ab.py --config $c --rounds 5 --frames 20 --variants $VAR --lib2 build_ab/$REV/librtamd.so > gpurun_out/abrev_c$c.txt 2>&1 || { echo "ab $c failed"; tail -20 gpurun_out/abrev_c$c.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/abrev_c$c.txt
done
