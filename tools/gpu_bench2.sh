#!/bin/bash
# bench.py default (2 frames in flight) + serial + a 2-rank gloo rehearsal on one GPU.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-b2}
timeout -k 10 300 python bench.py --cpu-seconds 8 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
timeout -k 10 300 python bench.py --no-cpu --inflight 1 > gpurun_out/${TAG}_bench_f1.json 2> gpurun_out/${TAG}_bench_f1.err || { tail -20 gpurun_out/${TAG}_bench_f1.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench_f1.json'));print('F=1', d['ms_per_step'], d['value'])"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --backend gloo --no-cpu --steps 50 > gpurun_out/${TAG}_bench_gloo2.json 2> gpurun_out/${TAG}_bench_gloo2.err || { tail -20 gpurun_out/${TAG}_bench_gloo2.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench_gloo2.json'));print('gloo2', d['ms_per_step'], d['value'], d['n_gpus'], d['frames_in_flight'])"
