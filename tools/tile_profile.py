"""Per-tile anatomy of one frame (diagnostics; run on the GPU box).

    python tools/tile_profile.py [--config 3] [--out gpurun_out/tiles_c3.npz]

Renders the config's frame once with the timed k_accel instance (per-tile
start/end wall clock, per-walk clock ticks and node steps: kTileRec in
rt_kernels.hip) after warm-up frames that derive the cost order, then, for the
64 slowest tiles, renders them ALONE (a one-tile dispatch order through
rt_debug_tile_order with every other tile after them would still run them, so
instead single-row bands around each) to get their latency on an idle GPU.
Saves the records and prints a summary.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "opengl-ray-tracer_amd"))
import rtamd  # noqa: E402

WL = {2: (2, 800, 600, 1), 3: (3, 1920, 1080, 3), 4: (3, 3840, 2160, 3), 5: (5, 1920, 1080, 3)}
ap = argparse.ArgumentParser()
ap.add_argument("--config", type=int, default=3)
ap.add_argument("--out", default=None)
a = ap.parse_args()
cfg, W, H, mb = WL[a.config]
fs = rtamd.generate(cfg, 0, W, H)
ctx = rtamd.ComputeShader(0)
ctx.upload(fs)
ctx.set_params(W, H, mb, True)
out = torch.empty((H, W, 4), dtype=torch.float32, device="cuda")
torch.cuda.synchronize()
tiles_x, tiles_y = (W + 7) // 8, (H + 7) // 8
n = tiles_x * tiles_y
for _ in range(10):
    ctx.dispatch_rows(W, H, 0, 1, 1, H, out.data_ptr(), W * 16)
ctx.sync()
kt = ctx.kernel_times()
ctx.debug_tile_times(n)
ctx.dispatch_rows(W, H, 0, 1, 1, H, out.data_ptr(), W * 16)
rec = ctx.tile_times(n).astype(np.int64)
ctx.debug_tile_times(0)
t0 = rec[:, 0].min()
start = (rec[:, 0] - t0) / 100.0  # us (100 MHz)
dur = (rec[:, 1] - rec[:, 0]) / 100.0
frame_us = (rec[:, 1].max() - t0) / 100.0
order = np.argsort(-dur)
res = {"config": a.config, "frame_us_timed": frame_us, "kernel_ms_untimed_median": float(np.median(kt)),
       "tiles": n, "dur_us_pcts": {p: float(np.percentile(dur, p)) for p in (50, 90, 99, 99.9, 100)}}
# concurrency over time: busy waves per 5 us bucket
edges = np.arange(0, frame_us + 5, 5.0)
busy = [int(((start <= e) & (start + dur > e)).sum()) for e in edges]
res["busy_waves_every_5us"] = busy
slow = order[:64]
res["slowest"] = []
for t in slow[:16]:
    r = rec[t]
    res["slowest"].append({
        "tile": int(t), "tx": int(t % tiles_x), "ty": int(t // tiles_x), "start_us": float(start[t]),
        "dur_us": float(dur[t]), "lane_nodes_sum": int(r[2]), "tests_sum": int(r[3]), "lane_nodes_max": int(r[4]),
        "tests_max": int(r[5]), "walk_ticks": [int(x) for x in r[6:14]], "walk_nodes": [int(x) for x in r[14:22]],
        "wave_leaf_iters": int(r[22]), "wave_node_iters": int(r[23])})
# the slowest tiles' rows rendered alone (8-row bands: one tile row each), idle GPU
alone = {}
for t in slow[:8]:
    ty = int(t // tiles_x)
    if ty in alone:
        continue
    for _ in range(3):
        ctx.dispatch_rows(W, H, ty * 8, 8, 1, 8, out.data_ptr(), W * 16)
    ctx.sync()
    ctx.kernel_times()
    for _ in range(10):
        ctx.dispatch_rows(W, H, ty * 8, 8, 1, 8, out.data_ptr(), W * 16)
    alone[ty] = float(np.median(ctx.kernel_times()) * 1e3)
res["tile_row_alone_us"] = alone
print(json.dumps(res))
if a.out:
    np.savez_compressed(a.out, rec=rec)
ctx.close()
