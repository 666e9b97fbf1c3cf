#!/bin/bash
# Round 4, step x: wall-time cost order -- latency-mode tile timeline, config 2/4/5/MT/animated lines,
# and the rocprofv3 passes of the car for the roofline's PMC entry.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r04x
timeout -k 10 240 python tools/tile_profile.py --config 3 --latency > gpurun_out/tiles_${T}_lat.json 2> gpurun_out/tiles_${T}_lat.err || exit 1
run() {  # name, bench args
  local n=$1; shift
  timeout -k 10 400 python bench.py "$@" > gpurun_out/bench_${T}_$n.json 2> gpurun_out/bench_${T}_$n.err; local rc=$?
  echo "bench $n rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_${T}_$n.err; exit $rc; }
  python -c "import json; d=json.load(open('gpurun_out/bench_${T}_$n.json')); print('  ', {k: (round(d[k],4) if isinstance(d.get(k), float) else d.get(k)) for k in ('ms_per_step','serial_ms_per_step','serial_frame_ms_median','value')}, 'parity', (d.get('parity') or {}).get('ok'))"
}
run anim_c2 --config 2 --animate --no-cpu
run anim_c3 --config 3 --animate --no-cpu
run c2 --config 2 --no-cpu
run c4 --config 4 --no-cpu --steps 50
run c5 --config 5 --no-cpu --steps 30 --warmup 5
run mt --mt --no-cpu --steps 40 --warmup 5
timeout -k 10 1200 bash tools/gpu_prof.sh ${T}_c3
