#!/usr/bin/env python3
"""Waited animated frames around accelerator rebuilds, with the rebuild on a host thread
(rt_debug_async_rebuild 1, the default) and in the flush that asks for it (0).

A shape whose kind of bound changes (an animated triangle squeezed to 1/1000 of its
height at frame 10, back at frame 30) makes the refit ask for a rebuild. Synchronously the frame
that asks waits for the whole host build (the car 4.1 ms, config 5 ~42 ms on the GPU
box); asynchronously the frames go on, exact (the refit enters every box above the
changed shape), and the rebuilt accelerator lands a few frames later.

    python tools/rebuild_stall.py [--config 3|5] [--frames 60]
Prints one JSON line: per mode the median and max waited frame (ms) and the frames that
took longer than 4x the median; and the scene swap itself, rt_upload_scene of the
config's scene into a context that holds it already (host build + device upload, ms).
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "opengl-ray-tracer_amd"))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import rtamd  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", type=int, default=3)
ap.add_argument("--frames", type=int, default=60)
ap.add_argument("--kernel-times", action="store_true", help="also each frame's render-kernel device ms (HIP events)")
a = ap.parse_args()
cfg, W, H, mb, _, _ = bench.WORKLOADS[a.config]
fs = rtamd.generate(cfg, 0, W, H)
if a.config in (3, 4):
    ids, frames = bench.wheel_frames(fs, a.frames)
else:  # 200 triangles drift (config 5 has no published animation)
    rng = np.random.default_rng(3)
    ids = np.sort(rng.choice(np.where(fs.shapes["type"] == 3)[0], 200, replace=False)).astype(np.int32)
    base = fs.shapes[ids].copy()
    frames = []
    for k in range(a.frames):
        r = base.copy()
        for f in ("triP1", "triP2", "triP3"):
            r[f] = (r[f] + np.float32(0.01 * k)).astype(np.float32)
        frames.append(r)
out = {"config": a.config, "W": W, "H": H, "modes": {}}
c = rtamd.ComputeShader(0)
up = []
for _ in range(5):
    t0 = time.perf_counter()
    c.upload(fs)
    up.append((time.perf_counter() - t0) * 1e3)
c.close()
out["upload_ms"] = {"median": float(np.median(up)), "min": float(np.min(up)), "runs": len(up)}
for asy in (0, 1):
    c = rtamd.ComputeShader(0)
    c.upload(fs)
    c.set_params(W, H, mb, True)
    c.set_kernel_timing(a.kernel_times)
    c.set_latency_mode(1)
    fn = c._lib.rt_debug_async_rebuild
    fn.argtypes = [C.c_void_p, C.c_int]
    fn(c._h, asy)
    c.set_animated(ids)
    buf = torch.empty((H, W, 4), dtype=torch.float32, device="cuda")
    ms, parts = [], []  # parts: animate, dispatch, sync (ms)
    for k in range(a.frames):
        recs = frames[k].copy()
        if 10 <= k < 30:  # squeezed towards its first edge: too thin to bound, still a triangle
            mid = recs["triP1"][7] + (recs["triP2"][7] - recs["triP1"][7]) * np.float32(0.5)
            recs["triP3"][7] = (mid + (recs["triP3"][7] - mid) * np.float32(1e-3)).astype(np.float32)
        t0 = time.perf_counter()
        c.set_camera(fs.camera)
        c.set_light(fs.light)
        c.animate(recs)
        t1 = time.perf_counter()
        c.dispatch_rows(W, H, 0, 1, 1, H, buf.data_ptr(), W * 16)
        t2 = time.perf_counter()
        c.sync()
        t3 = time.perf_counter()
        ms.append((t3 - t0) * 1e3)
        parts.append((round((t1 - t0) * 1e3, 3), round((t2 - t1) * 1e3, 3), round((t3 - t2) * 1e3, 3))
                     + ((round(float(c.last_kernel_ms()), 3),) if a.kernel_times else ()))
    st = np.zeros(4, np.int32)
    g = c._lib.rt_debug_rebuild_state
    g.argtypes = [C.c_void_p, C.c_void_p]
    g(c._h, st.ctypes.data)
    med = float(np.median(ms))
    out["modes"]["async" if asy else "sync"] = {
        "median_ms": med, "max_ms": float(np.max(ms)),
        "slow_frames": {int(i): round(float(v), 3) for i, v in enumerate(ms) if v > 4 * med},
        "slow_frame_parts_animate_dispatch_sync_kernel": {int(i): parts[i] for i, v in enumerate(ms) if v > 4 * med},
        "median_parts": [float(np.median([p[j] for p in parts])) for j in range(len(parts[0]))],
        "frames_parts": parts if a.kernel_times else None,
        "rebuilds_started": int(st[1]), "swapped": int(st[2])}
    c.close()
print(json.dumps(out))
