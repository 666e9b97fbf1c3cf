#!/bin/bash
# Roofline evidence for one workload, every pass its own rocprofv3 run of the solo
# bench command (--inflight 1: one frame in flight, so each launch runs alone):
#   trace   --kernel-trace --stats          (kernel durations)
#   fetch   --pmc FETCH_SIZE                (one TCC group per pass)
#   write   --pmc WRITE_SIZE
#   sq1/sq2 --pmc SQ_*/GRBM_GUI_ACTIVE      (issue side)
#   tcc     --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum
# usage: bash tools/gpu_prof.sh TAG [bench args...]
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--no-cpu --inflight 1 --steps 20 --warmup 3 $*"
run() {  # name rocprof-args...
  local name=$1; shift
  timeout -k 10 240 rocprofv3 "$@" --output-format csv -d $OUT/$name -o run -- python3 bench.py $ARGS \
      > $OUT/bench_$name.json 2> $OUT/$name.err || { echo "$TAG pass $name failed"; tail -20 $OUT/$name.err; exit 1; }
}
run trace --kernel-trace --stats
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
run sq1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY
run sq2 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_INSTS_VMEM SQ_INSTS_LDS GRBM_GUI_ACTIVE
run tcc --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum
echo "$TAG passes done"
