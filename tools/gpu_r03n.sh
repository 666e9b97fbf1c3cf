#!/bin/bash
# Round 3: with the 121-VGPR production instance, the two register-bound experiments of round 2
# again: the software-pipelined leaf loop (RT_LEAF_PREFETCH) and split walks everywhere
# (RT_SPLIT_ALL), each against the working tree on configs 3 and 5.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_ab_r03.sh "lpf splitall" "3 5"
