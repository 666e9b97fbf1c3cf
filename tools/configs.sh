#!/bin/bash
# Bench every single-GPU workload (no CPU leg): configs 2, 3, 4 (1 GPU), 5.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-cfg}
for c in 2 3 4 5; do
  timeout -k 10 180 python bench.py --config $c --steps 30 --warmup 5 --no-cpu > gpurun_out/${TAG}_c$c.json 2> gpurun_out/${TAG}_c$c.err || { echo "config $c failed"; tail -5 gpurun_out/${TAG}_c$c.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_c$c.json'));print($c, round(d['ms_per_step'],4), 'ms', round(d['kernel_ms_mean'],4), 'kernel ms', round(d['value']), d['unit'])"
done
