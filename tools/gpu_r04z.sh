#!/bin/bash
# Round 4 close-out: the GPU suite, the driver's bench command, the 1-rank strong line, the
# animated lines, configs 2 / 4 / 5 and the Moller-Trumbore car on the current build.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r04z}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_$T.log; [ $rc -eq 0 ] || exit $rc
run() {  # name, bench args
  local n=$1; shift
  timeout -k 10 400 python bench.py "$@" > gpurun_out/bench_${T}_$n.json 2> gpurun_out/bench_${T}_$n.err; local rc=$?
  echo "bench $n rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_${T}_$n.err; exit $rc; }
  python -c "import json; d=json.load(open('gpurun_out/bench_${T}_$n.json')); print('  ', {k: (round(d[k],4) if isinstance(d.get(k), float) else d.get(k)) for k in ('ms_per_step','serial_ms_per_step','serial_frame_ms_median','value')}, 'parity', (d.get('parity') or {}).get('ok'))"
}
run main --gpus 1 --steps 20 --warmup 5
run strong1 --mode strong --no-cpu
run anim_c2 --config 2 --animate --no-cpu
run anim_c3 --config 3 --animate --no-cpu
run c2 --config 2 --no-cpu
run c4 --config 4 --no-cpu --steps 50
run c5 --config 5 --no-cpu --steps 30 --warmup 5
run mt --mt --no-cpu --steps 40 --warmup 5
