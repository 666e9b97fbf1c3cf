#!/usr/bin/env python3
"""Waited animated frames from the C++ host loop, for timelines of the per-frame
prelude (run it under `rocprofv3 --kernel-trace`, then tools/kernel_timeline.py).

    python tools/anim_probe.py [--config 3] [--upload device|reference|static] [--frames 200]

device: rt_animate per frame (rth_render_loop_anim); reference: the reference's own
upload calls (rth_render_loop_ref); static: no animation (rth_render_loop).
Prints one JSON line: median / p10 / p90 of the waited frames (ms), latency mode on.
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
    ap.add_argument("--upload", default="device", choices=["device", "reference", "static"])
    ap.add_argument("--frames", type=int, default=200)
    ap.add_argument("--latency", type=int, default=1)
    ap.add_argument("--refit", type=int, default=-1, help="rt_debug_refit mode (-1: default)")
    a = ap.parse_args()
    import torch
    import bench
    import rtamd
    cfg, W, H, mb, _, _ = bench.WORKLOADS[a.config]
    fs = rtamd.generate(cfg, 0, W, H)
    ctx = rtamd.ComputeShader(0)
    ctx.upload(fs)
    ctx.set_params(W, H, mb, True)
    ctx.set_kernel_timing(0)
    ctx.set_latency_mode(a.latency)
    if a.refit >= 0:
        ctx.debug_refit(a.refit)
    out = torch.empty((H, W, 4), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    anim, ref = None, None
    if a.upload != "static":
        ids, frames = bench.sphere_frames(fs, 512) if a.config == 2 else bench.wheel_frames(fs, 64)
        anim = frames
        if a.upload == "device":
            ctx.set_animated(ids)
        else:
            ref = rtamd.ReferenceUpload(fs, ids)
    warm = rtamd.render_loop(ctx, fs.camera, fs.light, W, H, out.data_ptr(), W * 16, 64, True, anim=anim, ref=ref)
    ms = rtamd.render_loop(ctx, fs.camera, fs.light, W, H, out.data_ptr(), W * 16, a.frames, True, anim=anim, ref=ref)
    print(json.dumps({"config": a.config, "upload": a.upload, "frames": a.frames, "latency_mode": a.latency, "refit_mode": a.refit,
                      "median_ms": float(np.median(ms)), "p10_ms": float(np.percentile(ms, 10)),
                      "p90_ms": float(np.percentile(ms, 90)), "warm_median_ms": float(np.median(warm)),
                      "rebuilds": ctx.debug_anim_rebuilds(), "refits": ctx.debug_refits(),
                      **ctx.debug_refit_stats()}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
