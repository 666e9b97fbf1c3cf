"""Throughput of one rank's share of a strong-scaled frame (the 8-GPU plan's
stripe set of rank 0: rows {y : (y/8) mod P == 0}) with F frames in flight,
each on its own context and stream. Run with different GPU_MAX_HW_QUEUES to
see whether the hardware queues cap the frames that actually overlap.

    GPU_MAX_HW_QUEUES=8 python tools/inflight_share.py [--parts 8] [--inflight 2,4,8]
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "opengl-ray-tracer_amd"))
import rtamd  # noqa: E402
import tiling  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--parts", type=int, default=8)
ap.add_argument("--inflight", default="1,2,4,8,12")
ap.add_argument("--frames", type=int, default=240)
a = ap.parse_args()
W, H = 1920, 1080
fs = rtamd.generate(3, 0, W, H)
plan = tiling.StripePlan(H, a.parts, 8)
rows = plan.rows(0)
res = {"GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES", "default"), "parts": a.parts, "rows": rows}
for F in [int(x) for x in a.inflight.split(",")]:
    ctxs, bufs = [], []
    for _ in range(F):
        s = torch.cuda.Stream()
        c = rtamd.ComputeShader(0)
        c.set_stream(s.cuda_stream)
        c.upload(fs)
        c.set_params(W, H, 3, True)
        ctxs.append(c)
        bufs.append(torch.empty((rows, W, 3), dtype=torch.float32, device="cuda"))
    torch.cuda.synchronize()
    for i in range(16 * F):
        ctxs[i % F].dispatch_rows_rgb(W, H, 0, 8, a.parts, rows, bufs[i % F].data_ptr(), W * 12)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.frames):
        ctxs[i % F].dispatch_rows_rgb(W, H, 0, 8, a.parts, rows, bufs[i % F].data_ptr(), W * 12)
    torch.cuda.synchronize()
    res[f"F{F}_us_per_frame"] = (time.perf_counter() - t0) / a.frames * 1e6
    for c in ctxs:
        c.close()
print(json.dumps(res))
