#!/usr/bin/env python3
"""Waited car frame over host-made dispatch orders (diagnostics; run on the GPU box).

    python tools/order_probe.py [--frames 300] [--blocks 3]

Question: a waited frame keeps the chip full for ~235 us (tools/tile_profile.py
--latency) although three frames in flight take 183 us each. Does the cost
order's phase structure (every heavy tile at once, then the light ones) cost
throughput, and does an order that mixes heavy and light tiles while still
ending on light ones do better?

Per-tile work (lane node steps + tests, the cost order's measure) comes from one
timed frame. Orders (rt_debug_tile_order; a host order turns latency mode's
heavy-tile split off, so "desc" is the like-for-like base):
  rows     identity
  desc     cost descending (the device cost order without splits)
  mixH     the H heaviest descending, then the rest's heavier and lighter halves
           interleaved one to one (each resident set holds both; the order ends
           on the lightest)
  shufH    the H heaviest descending, the middle shuffled, the lightest 8192 last
Plus "sched": the device's own cost order with latency mode (the product path).
Every order's image is compared with the first's. One JSON line.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "opengl-ray-tracer_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import bench  # noqa: E402
import rtamd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=300)
    ap.add_argument("--blocks", type=int, default=3)
    ap.add_argument("--config", type=int, default=3)
    a = ap.parse_args()
    cfg, W, H, mb, _, _ = bench.WORKLOADS[a.config]
    fs = rtamd.generate(cfg, 0, W, H)
    torch.cuda.set_device(0)
    c = rtamd.ComputeShader(0)
    c.upload(fs)
    c.set_params(W, H, mb)
    c.set_kernel_timing(False)
    c.set_latency_mode(1)
    out = torch.empty((H, W, 4), dtype=torch.float32, device="cuda")
    n = ((W + 7) // 8) * ((H + 7) // 8)

    def frame():
        c.set_camera(fs.camera)
        c.set_light(fs.light)
        c.dispatch_rows(W, H, 0, 1, 1, H, out.data_ptr(), W * 16)
        c.sync()

    for _ in range(10):
        frame()
    c.debug_tile_times(n)
    frame()
    rec = c.tile_times(n).astype(np.int64)
    c.debug_tile_times(0)
    cost = rec[:, 2] + rec[:, 3]
    desc = np.argsort(-cost, kind="stable").astype(np.int32)
    rng = np.random.default_rng(7)

    def mix(h):
        rest = desc[h:]
        half = (len(rest) + 1) // 2
        A, B = rest[:half], rest[half:]
        m = np.empty(len(rest), np.int32)
        m[0:2 * len(B):2] = A[:len(B)]
        m[1:2 * len(B):2] = B
        m[2 * len(B):] = A[len(B):]
        return np.concatenate([desc[:h], m])

    def shuf(h):
        mid = desc[h:n - 8192].copy()
        rng.shuffle(mid)
        return np.concatenate([desc[:h], mid, desc[n - 8192:]])

    orders = {"sched": None, "rows": np.arange(n, dtype=np.int32), "desc": desc}
    for h in (0, 1024, 4096):
        orders[f"mix{h}"] = mix(h)
    for h in (1024, 4096):
        orders[f"shuf{h}"] = shuf(h)
    for k, o in orders.items():
        assert o is None or np.array_equal(np.sort(o), np.arange(n)), k
    res, same, ref = {k: [] for k in orders}, {}, None
    for _ in range(a.blocks):
        for k, o in orders.items():
            c.debug_tile_order(o)
            for _ in range(20):
                frame()
            w = []
            for _ in range(a.frames):
                t0 = time.perf_counter()
                frame()
                w.append(time.perf_counter() - t0)
            res[k].append(float(np.median(w)) * 1e3)
            img = out.cpu().numpy()
            if ref is None:
                ref = img
            same[k] = same.get(k, True) and bool(np.array_equal(img, ref))
    c.debug_tile_order(None)
    print(json.dumps({"config": a.config, "frames": a.frames, "blocks": a.blocks,
                      "cost_pcts": {p: float(np.percentile(cost, p)) for p in (50, 90, 99, 100)},
                      "waited_ms": {k: float(np.median(v)) for k, v in res.items()}, "per_block": res,
                      "image_equal": same}))
    c.close()


if __name__ == "__main__":
    main()
