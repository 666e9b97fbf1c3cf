#!/bin/bash
# Round 3: BASELINE.md's CPU plan (configs 2 and 5 with the oracle + cpuRayTracer,
# the MT car) and solo roofline profiles of configs 2, 5 and the MT car.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in 2 5; do
  timeout -k 10 300 python bench.py --config $c > gpurun_out/bench_r03b_c$c.json 2> gpurun_out/bench_r03b_c$c.err || { echo "bench c$c failed"; tail -5 gpurun_out/bench_r03b_c$c.err; exit 1; }
  echo "c$c done"
done
timeout -k 10 300 python bench.py --mt > gpurun_out/bench_r03b_c3_mt.json 2> gpurun_out/bench_r03b_c3_mt.err || { echo "bench mt failed"; tail -5 gpurun_out/bench_r03b_c3_mt.err; exit 1; }
echo "mt done"
bash tools/gpu_prof.sh r03b_c2 --config 2 || exit $?
bash tools/gpu_prof.sh r03b_c5 --config 5 || exit $?
bash tools/gpu_prof.sh r03b_c3mt --mt --steps 10 || exit $?
