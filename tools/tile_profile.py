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
ap.add_argument("--latency", action="store_true", help="rt_set_latency_mode on (the waited-frame dispatch)")
a = ap.parse_args()
cfg, W, H, mb = WL[a.config]
fs = rtamd.generate(cfg, 0, W, H)
ctx = rtamd.ComputeShader(0)
ctx.upload(fs)
ctx.set_params(W, H, mb, True)
if a.latency:
    ctx.set_latency_mode(True)
out = torch.empty((H, W, 4), dtype=torch.float32, device="cuda")
torch.cuda.synchronize()
tiles_x, tiles_y = (W + 7) // 8, (H + 7) // 8
n = tiles_x * tiles_y
for _ in range(10):
    ctx.dispatch_rows(W, H, 0, 1, 1, H, out.data_ptr(), W * 16)
ctx.sync()
kt = ctx.kernel_times()
# records: one per tile, then (latency mode's split heavy tiles) one per part slot
cap = n + (4096 if a.latency else 0)
ctx.debug_tile_times(cap)
ctx.dispatch_rows(W, H, 0, 1, 1, H, out.data_ptr(), W * 16)
rec_all = ctx.tile_times(cap).astype(np.int64)
ctx.debug_tile_times(0)
parts = rec_all[n:][rec_all[n:, 1] > 0]  # part slots that ran (end stamp set)
rec = rec_all[:n].copy()
if len(parts):
    # a split tile's own record is unused (zero): duration 0 here, its parts reported below
    rec[rec[:, 1] == 0, 0:2] = rec_all[:n][rec_all[:n, 1] > 0, 0].min()
rec_ev = np.concatenate([rec_all[:n][rec_all[:n, 1] > 0], parts])
t0 = rec_ev[:, 0].min()
start = (rec[:, 0] - t0) / 100.0  # us (100 MHz)
dur = (rec[:, 1] - rec[:, 0]) / 100.0
frame_us = (rec_ev[:, 1].max() - t0) / 100.0
order = np.argsort(-dur)
res = {"config": a.config, "latency_mode": a.latency, "frame_us_timed": frame_us, "kernel_ms_untimed_median": float(np.median(kt)),
       "tiles": n, "dur_us_pcts": {p: float(np.percentile(dur, p)) for p in (50, 90, 99, 99.9, 100)}}
# concurrency over time: busy waves per 5 us bucket
edges = np.arange(0, frame_us + 5, 5.0)
ev_s, ev_e = (rec_ev[:, 0] - t0) / 100.0, (rec_ev[:, 1] - t0) / 100.0
busy = [int(((ev_s <= e) & (ev_e > e)).sum()) for e in edges]
res["busy_waves_every_5us"] = busy
if len(parts):
    ps, pd = (parts[:, 0] - t0) / 100.0, (parts[:, 1] - parts[:, 0]) / 100.0
    po = np.argsort(-pd)
    res["split_parts"] = {"n": int(len(parts)), "dur_us_pcts": {p: float(np.percentile(pd, p)) for p in (50, 90, 100)},
                          "slowest": [{"start_us": float(ps[i]), "dur_us": float(pd[i]), "walk_ticks":
                                       [int(x) for x in parts[i, 6:12]]} for i in po[:12]]}
    # whole tiles (not split) that end last
    we = (rec_all[:n, 1] - t0) / 100.0
    last = np.argsort(-we)[:12]
    res["last_whole_tiles"] = [{"tile": int(t), "start_us": float(start[t]), "end_us": float(we[t]),
                                "walk_ticks": [int(x) for x in rec_all[t, 6:12]]} for t in last]
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
