#!/usr/bin/env python3
"""Latency mode's split constants off the tuned view: for cameras
spread along bench.py's orbit path, each held still, the waited frame (C++ host loop,
latency mode) with the default split rule and with the heaviest k tiles as `parts`
waves over a grid of k and parts (rt_debug_heavy).

    python tools/view_sweep.py [--samples 4] [--div 400,200,100,50] [--parts 2,4,8]
Prints one JSON object: per camera the default, the best setting and its time.
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
    ap.add_argument("--samples", type=int, default=4)
    ap.add_argument("--div", default="400,200,100,50")
    ap.add_argument("--parts", default="2,4,8")
    ap.add_argument("--frames", type=int, default=120)
    ap.add_argument("--mt", action="store_true", help="useMollerTrumbore = 1")
    a = ap.parse_args()
    import torch
    import bench
    import rtamd
    cfg, W, H, mb, _, target = bench.WORKLOADS[a.config]
    sc = rtamd.Scene().generate(cfg, 0, W / H)
    fs = sc.serializeScene()
    cams = bench.camera_path(rtamd, sc, fs, "orbit", target)
    buf = torch.empty((H, W, 4), dtype=torch.float32, device="cuda")
    ctx = rtamd.ComputeShader(0)
    ctx.upload(fs)
    ctx.set_params(W, H, mb, True, False, a.mt)
    ctx.set_kernel_timing(0)
    ctx.set_latency_mode(1)
    tiles = ((W + 7) // 8) * ((H + 7) // 8)

    def waited(cam):
        rtamd.render_loop(ctx, cam, fs.light, W, H, buf.data_ptr(), W * 16, 48, True)  # the order settles
        return float(np.median(rtamd.render_loop(ctx, cam, fs.light, W, H, buf.data_ptr(), W * 16, a.frames, True)))

    out = {"config": a.config, "mt": a.mt, "tiles": tiles, "views": []}
    for k in range(a.samples):
        i = int(round(k * len(cams) / a.samples)) % len(cams)
        cam = cams[i:i + 1]
        ctx.debug_heavy(-1, 1)
        rec = {"orbit_frame": i, "default_ms": waited(cam), "grid_ms": {}}
        for d in [int(x) for x in a.div.split(",")]:
            for p in [int(x) for x in a.parts.split(",")]:
                ctx.debug_heavy(max(16, tiles // d), p)
                rec["grid_ms"][f"1/{d}x{p}"] = waited(cam)
        ctx.debug_heavy(-1, 1)
        best = min(rec["grid_ms"], key=rec["grid_ms"].get)
        rec["best"] = best
        rec["best_ms"] = rec["grid_ms"][best]
        rec["default_over_best"] = rec["default_ms"] / rec["best_ms"]
        out["views"].append(rec)
        print(json.dumps({k2: v for k2, v in rec.items() if k2 != "grid_ms"}), file=sys.stderr, flush=True)
    ctx.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
