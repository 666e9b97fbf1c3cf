#!/bin/bash
# Round 4, step k: sky-row fan-in: the group tests (copy transport, 2-8 members), the native
# C++ group host, and a gloo rehearsal of the strong bench on one GPU.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "group or rccl or native or bench" > gpurun_out/pytest_r04k.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r04k.log; [ $rc -eq 0 ] || exit $rc
