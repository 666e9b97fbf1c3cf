#!/bin/bash
# bench.py at N=1, then the N=2 paths rehearsed on one GPU with gloo (weak and strong).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu > gpurun_out/bm_n1.json 2> gpurun_out/bm_n1.err || exit 1
cat gpurun_out/bm_n1.json
for m in weak strong; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
     bench.py --gpus 2 --steps 30 --warmup 3 --backend gloo --mode $m --no-cpu > gpurun_out/bm_g2_$m.json 2> gpurun_out/bm_g2_$m.err || { tail -20 gpurun_out/bm_g2_$m.err; exit 1; }
  cat gpurun_out/bm_g2_$m.json
done
