#!/bin/bash
# Scene-tree round: GPU tests, then A/B of scene tree vs reference tree.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for c in 2 3 5; do
  timeout -k 10 240 python tools/ab.py --config $c --rounds 4 --frames 20 --variants default,reftree,lane_all,packet_all > gpurun_out/ab_tree_c$c.txt 2>&1 || { echo "ab $c failed"; tail -20 gpurun_out/ab_tree_c$c.txt; exit 1; }
  cat gpurun_out/ab_tree_c$c.txt
done
