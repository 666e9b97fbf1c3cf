#!/usr/bin/env python3
"""Waited frames along a moving camera against the same cameras held still (VERDICT r4
item 4): is a moving camera slower because its views cost more, or because the
cost-ordered dispatch ranks tiles by an older view?

    python tools/camera_probe.py [--path orbit|dolly] [--samples 8] [--variants 16:0:-1,4:0:-1,1:0:-1]
                                 [--order-stream 0|1|2] [--frame-event 0|1]

From the C++ host loop (librthost.so rth_render_loop, latency mode on, as bench.py's
serial frames):
  * still: for `samples` cameras spread along the path, each held for 160 frames
    (median of the last 120: the cost order converged on that view);
  * moving: the whole path once per variant PERIOD:DILATE:COST (rt_debug_sched_period,
    rt_debug_cost_dilate, rt_debug_cost_time) or mP:DILATE:SPLIT (rt_debug_moving),
    per-frame times; reported as the median over +-window frames around each sampled
    camera, and over the whole path.
Prints one JSON object.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "opengl-ray-tracer_amd"), ROOT]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--path", default="orbit", choices=["orbit", "dolly"])
    ap.add_argument("--samples", type=int, default=8)
    ap.add_argument("--variants", default="16:0:-1,4:0:-1,1:0:-1")
    ap.add_argument("--window", type=int, default=12)
    ap.add_argument("--latency", type=int, default=1)
    ap.add_argument("--order-stream", type=int, default=None,
                    help="rt_debug_order_stream mode for every context (default: the library's)")
    ap.add_argument("--frame-event", type=int, default=None,
                    help="rt_debug_frame_event for every context (default: the library's)")
    a = ap.parse_args()
    import torch
    import bench
    import rtamd
    cfg, W, H, mb, _, target = bench.WORKLOADS[a.config]
    sc = rtamd.Scene().generate(cfg, 0, W / H)
    fs = sc.serializeScene()
    cams = bench.camera_path(rtamd, sc, fs, a.path, target)
    n = len(cams)
    buf = torch.empty((H, W, 4), dtype=torch.float32, device="cuda")

    def fresh(period=None, dilate=0, cost=-1, moving=None):
        ctx = rtamd.ComputeShader(0)
        ctx.upload(fs)
        ctx.set_params(W, H, mb, True)
        ctx.set_kernel_timing(0)
        ctx.set_latency_mode(a.latency)
        if period is not None:
            ctx.debug_sched_period(period)
        ctx.debug_cost_dilate(dilate)
        ctx.debug_cost_time(cost)
        if moving is not None:
            ctx.debug_moving(*moving)
        if a.order_stream is not None:
            ctx.debug_order_stream(a.order_stream)
        if a.frame_event is not None:
            ctx.debug_frame_event(a.frame_event)
        return ctx

    idx = [int(round(k * n / a.samples)) % n for k in range(a.samples)]
    out = {"config": a.config, "path": a.path, "frames": n, "latency_mode": a.latency, "samples": idx,
           "order_stream": a.order_stream, "frame_event": a.frame_event}
    ctx = fresh()
    still = []
    for i in idx:
        ms = rtamd.render_loop(ctx, cams[i:i + 1], fs.light, W, H, buf.data_ptr(), W * 16, 160, True)
        still.append(float(np.median(ms[40:])))
        print(json.dumps({"still": i, "ms": still[-1]}), file=sys.stderr, flush=True)
    ctx.close()
    out["still_ms"] = still
    out["still_median_ms"] = float(np.median(still))
    for v in a.variants.split(","):
        if v.startswith("m"):
            ctx = fresh(moving=[int(x) for x in v[1:].split(":")])
        else:
            p, dil, cost = (int(x) for x in v.split(":"))
            ctx = fresh(p, dil, cost)
        rtamd.render_loop(ctx, cams[:1], fs.light, W, H, buf.data_ptr(), W * 16, 48, True)  # warm: order for cam 0
        ms = np.asarray(rtamd.render_loop(ctx, cams, fs.light, W, H, buf.data_ptr(), W * 16, n, True))
        ctx.close()
        win = []
        for i in idx:
            sel = [(i + d) % n for d in range(-a.window, a.window + 1)]
            win.append(float(np.median(ms[sel])))
        rec = {"moving_ms_at_samples": win, "moving_median_ms": float(np.median(ms)),
               "moving_over_still": float(np.median(np.asarray(win) / np.asarray(still)))}
        out[v] = rec
        print(json.dumps({"variant": v, **rec}), file=sys.stderr, flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
