#!/bin/bash
# One GPU call: smoke, GPU parity tests, bench (N=1), profiles.
# usage: bash tools/gpu_round.sh TAG [pytest selection]
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r02}
SEL=${2:-tests}
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 gpurun_out/smoke.log; exit 1; }
timeout -k 10 900 python -u -m pytest $SEL -m gpu -v -rf --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|ERROR" gpurun_out/pytest_gpu.log | tail -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err; rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_$TAG.json
[ $rc -eq 0 ] || exit $rc
bash tools/profile.sh ${TAG}_c3 --steps 20 --warmup 3
