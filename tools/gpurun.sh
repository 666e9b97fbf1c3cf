#!/bin/bash
# Rebuild every in-tree native piece (the box runs the .so files as shipped),
# then send the command to the GPU box.   usage: bash tools/gpurun.sh TIMEOUT 'command'
set -e
cd "$(dirname "$0")/.."
make -s -j8 -C opengl-ray-tracer_amd
make -s -C oracle build/liboracle.so
make -s -C tests/native
exec /usr/local/graft/bin/gpurun --timeout "$1" -- "$2"
