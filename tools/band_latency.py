"""Kernel time of single tile rows (the GPU nearly idle) vs the full frame:
how long the slowest tiles take by themselves (latency floor of the critical path)."""
import os, sys, json
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "opengl-ray-tracer_amd"))
import rtamd  # noqa: E402

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 3
W, H = 1920, 1080
fs = rtamd.generate(cfg, 0, W, H)
ctx = rtamd.ComputeShader(0)
ctx.upload(fs)
ctx.set_params(W, H, 3, True)
out = torch.empty((H, W, 4), dtype=torch.float32, device="cuda")
res = {}
for y0 in (520, 600, 672, 736):
    for _ in range(3):
        ctx.dispatch_rows(W, H, y0, 8, 1, 8, out.data_ptr(), W * 16)
    ctx.sync()
    ctx.kernel_times()
    for _ in range(10):
        ctx.dispatch_rows(W, H, y0, 8, 1, 8, out.data_ptr(), W * 16)
    res[f"row{y0}"] = float(np.median(ctx.kernel_times()))
    ctx.debug_tile_times(240)
    ctx.dispatch_rows(W, H, y0, 8, 1, 8, out.data_ptr(), W * 16)
    t = ctx.tile_times(240).astype(np.int64)
    ctx.debug_tile_times(0)
    d = (t[:, 1] - t[:, 0]) / 100.0
    res[f"row{y0}_max_tile_us"] = float(d.max())
    res[f"row{y0}_max_lane_nodes"] = int(t[:, 4].max())
for _ in range(3):
    ctx.dispatch_rows(W, H, 0, 1, 1, H, out.data_ptr(), W * 16)
ctx.sync()
ctx.kernel_times()
for _ in range(10):
    ctx.dispatch_rows(W, H, 0, 1, 1, H, out.data_ptr(), W * 16)
res["full"] = float(np.median(ctx.kernel_times()))
print(json.dumps(res))
