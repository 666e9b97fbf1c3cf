#!/bin/bash
# Round 3: 64-byte prim records (PrimRec) — GPU suite, then A/B against HEAD's build.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_r03h.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r03h.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_r03.sh head2 "3 5 2"
