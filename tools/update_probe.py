#!/usr/bin/env python3
"""Waited frames of a host that rewrites a different 1 % of the scene's shapes every frame
through the reference's per-record upload (rt_update_shapes, src/main.cpp:981-992): the
pattern whose refit set rt_ctx bounds (compact_refit_set). Each frame: the records' calls,
then dispatch + rt_sync; the calls, the dispatch and the wait are timed apart (the refit
set's maps are rebuilt on the host, prepare_animation, whenever new shapes join it).

    python tools/update_probe.py [--config 5] [--frames 40] [--fraction 0.01]
Prints one JSON line: medians of the three parts (ms) and of the whole frame.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "opengl-ray-tracer_amd"), ROOT]
import bench  # noqa: E402
import rtamd  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", type=int, default=5)
ap.add_argument("--frames", type=int, default=40)
ap.add_argument("--fraction", type=float, default=0.01)
a = ap.parse_args()
cfg, W, H, mb, _, _ = bench.WORKLOADS[a.config]
fs = rtamd.generate(cfg, 0, W, H)
S = len(fs.shapes)
rng = np.random.default_rng(5)
order = rng.permutation(S)
per = max(1, int(S * a.fraction))
c = rtamd.ComputeShader(0)
c.upload(fs)
c.set_params(W, H, mb, True)
c.set_kernel_timing(False)
c.set_latency_mode(1)
buf = torch.empty((H, W, 4), dtype=torch.float32, device="cuda")
shapes = fs.shapes.copy()
parts = []
for k in range(a.frames):
    ids = np.sort(order[(k * per) % S:(k * per) % S + per])
    for f in ("triP1", "triP2", "triP3", "sphereCenter", "wallStart"):
        shapes[f][ids] += np.float32(0.001 * (k + 1))
    t0 = time.perf_counter()
    for i in ids:
        c.update_shapes(int(i), shapes[i:i + 1])
    t1 = time.perf_counter()
    c.dispatch_rows(W, H, 0, 1, 1, H, buf.data_ptr(), W * 16)
    t2 = time.perf_counter()
    c.sync()
    t3 = time.perf_counter()
    parts.append(((t1 - t0) * 1e3, (t2 - t1) * 1e3, (t3 - t2) * 1e3, (t3 - t0) * 1e3))
st = c.debug_refit_stats()
c.close()
p = np.array(parts[4:])
print(json.dumps({"config": a.config, "W": W, "H": H, "frames": a.frames, "per_frame_shapes": per,
                  "median_ms": {"update_calls": float(np.median(p[:, 0])), "dispatch": float(np.median(p[:, 1])),
                                "sync": float(np.median(p[:, 2])), "frame": float(np.median(p[:, 3]))},
                  "max_frame_ms": float(p[:, 3].max()), "refit_stats": {k: int(v) for k, v in st.items()}}))
