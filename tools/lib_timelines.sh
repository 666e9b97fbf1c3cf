#!/bin/bash
# Kernel timelines of tools/anim_probe.py (rocprofv3 --kernel-trace) with each of several
# librtamd.so builds swapped in (build_ab/NAME/librtamd.so, tools/build_var.sh), then the
# tree's own build put back. Timing probes only: the variants may render wrong images.
#   bash tools/lib_timelines.sh TAG NAME [NAME ...]      (inside gpurun, from the repo root)
set -e -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; shift
L=opengl-ray-tracer_amd/lib
cp $L/librtamd.so /tmp/librtamd_tree.so
for v in base "$@"; do
    if [ "$v" = base ]; then cp /tmp/librtamd_tree.so $L/librtamd.so; else cp build_ab/$v/librtamd.so $L/librtamd.so; fi
    timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_$v -o run -- \
        python tools/anim_probe.py --frames 40 ${PROBE_ARGS} > gpurun_out/${TAG}_$v.log 2>&1
    echo "$v done"
done
cp /tmp/librtamd_tree.so $L/librtamd.so
