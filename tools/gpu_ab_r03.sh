#!/bin/bash
# Throughput (2 in flight) and serial (1 in flight) A/B of experiment builds against the
# working tree: tools/abf.py alternates the builds in child processes and compares images.
# usage: bash tools/gpu_ab_r03.sh "NAME1 NAME2 ..." "3 5"
set -o pipefail
mkdir -p gpurun_out
NAMES=$1; CFGS=${2:-"3 5"}
for n in $NAMES; do
  for c in $CFGS; do
    for f in 2 1; do
      fr=200; [ $c = 5 ] && fr=30
      echo -n "$n config $c inflight $f: "
      timeout -k 10 150 python tools/abf.py --lib2 build_ab/$n/librtamd.so --config $c --inflight $f --frames $fr --rounds 3 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
    done
  done
done
