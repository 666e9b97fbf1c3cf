#!/bin/bash
# Round 3 close: solo profile of config 2 with the final build (pmc_summary config2_n1_auto).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_prof.sh r03x_c2 --config 2 || exit $?
