#!/bin/bash
# Round 4, step f: the full GPU suite, the default bench line (as the driver runs it) and the
# 1-rank strong line on the current build.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_r04f.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r04f.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r04f.json 2> gpurun_out/bench_r04f.err; rc=$?
echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_r04f.err; exit $rc; }
timeout -k 10 300 python bench.py --mode strong --no-cpu > gpurun_out/bench_r04f_strong1.json 2> gpurun_out/bench_r04f_strong1.err; rc=$?
echo "bench strong rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_r04f_strong1.err; exit $rc; }
python - <<'PY'
import json
for f in ("bench_r04f", "bench_r04f_strong1"):
    d = json.load(open(f"gpurun_out/{f}.json"))
    print(f, {k: d.get(k) for k in ("ms_per_step", "frames_in_flight", "serial_ms_per_step", "serial_ms_per_step_latency_mode",
                                     "serial_frame_ms_median", "serial_frame_ms_median_python", "kernel_ms_mean")})
    print("   parity", (d.get("parity") or {}).get("ok"), "cpu", (d.get("cpu_baseline") or {}).get("value"))
PY
