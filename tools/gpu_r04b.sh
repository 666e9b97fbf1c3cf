#!/bin/bash
# Round 4, step b: group fixed cost per variant (tools/group_cost.py), then the frames and
# 1-rank strong bench lines with the timing-event passes split off.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python tools/group_cost.py > gpurun_out/group_cost_r04f.json 2> gpurun_out/group_cost_r04f.err; rc=$?
echo "group_cost rc=$rc"; cat gpurun_out/group_cost_r04f.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/group_cost_r04f.err; exit $rc; }
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench_r04b.json 2> gpurun_out/bench_r04b.err; rc=$?
echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_r04b.err; exit $rc; }
timeout -k 10 300 python bench.py --mode strong --no-cpu > gpurun_out/bench_r04b_strong1.json 2> gpurun_out/bench_r04b_strong1.err; rc=$?
echo "bench strong rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_r04b_strong1.err; exit $rc; }
python - <<'PY'
import json
for f in ("bench_r04b", "bench_r04b_strong1"):
    d = json.load(open(f"gpurun_out/{f}.json"))
    print(f, {k: d.get(k) for k in ("ms_per_step", "frames_in_flight", "serial_ms_per_step", "serial_ms_per_step_latency_mode",
                                     "serial_frame_ms_median", "kernel_ms_mean", "kernel_ms_mean_inflight", "group_phases_ms")})
    print("   roofline", {k: d["roofline"].get(k) for k in ("bound", "frac", "traffic")}, "parity", (d.get("parity") or {}).get("ok"))
PY
timeout -k 10 400 python tools/latency_sweep.py > gpurun_out/latency_sweep_r04b.json 2> gpurun_out/latency_sweep_r04b.err; rc=$?
echo "latency sweep rc=$rc"; cat gpurun_out/latency_sweep_r04b.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/latency_sweep_r04b.err; exit $rc; }
