#!/bin/bash
# Profile bench.py on the GPU box: kernel trace + stats, then FETCH_SIZE and
# WRITE_SIZE in separate --pmc passes (MI355X_MICROARCH.md: one TCC counter
# group per pass; never combined with runtime/sys tracing).
# usage: bash tools/profile.sh TAG [bench args...]
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 bench.py --no-cpu "$@" > $OUT/bench_trace.json 2> $OUT/trace.err || { echo "trace pass failed"; tail -20 $OUT/trace.err; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- \
    python3 bench.py --no-cpu "$@" > $OUT/bench_fetch.json 2> $OUT/fetch.err || { echo "fetch pass failed"; tail -20 $OUT/fetch.err; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- \
    python3 bench.py --no-cpu "$@" > $OUT/bench_write.json 2> $OUT/write.err || { echo "write pass failed"; tail -20 $OUT/write.err; exit 1; }
find $OUT -name "*.csv" | head -20
