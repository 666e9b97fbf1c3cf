#!/bin/bash
# Per-tile timing / concurrency analysis of the default kernel on configs 3 and 5.
set -o pipefail
mkdir -p gpurun_out
for c in 3 5 4; do
  timeout -k 10 240 python tools/ab.py --config $c --rounds 2 --frames 10 --variants default,w3_all --times > gpurun_out/times_c$c.txt 2>&1 || exit 1
done
