"""Device LBVH (rt_build_lbvh) against the reference builder (host scene library).

    python tools/bench_lbvh.py [--configs 2,3,5] [--frames 20]

Per configuration: the reference builder's time on the host (rts_build_bvh,
split/buildBVH restated), the LBVH's device build time (HIP events around its
kernels and radix sort), the whole rt_build_lbvh call (build + read-back +
adoption, including the accelerator build on the host), and the render time of
the frame over each tree (median device ms over --frames dispatches).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "opengl-ray-tracer_amd"))
import rtamd  # noqa: E402

WL = {2: (2, 800, 600, 1, 15), 3: (3, 1920, 1080, 3, 25), 5: (5, 1920, 1080, 3, 25)}

ap = argparse.ArgumentParser()
ap.add_argument("--configs", default="2,3,5")
ap.add_argument("--frames", type=int, default=20)
a = ap.parse_args()
ctx = rtamd.ComputeShader(0)
for cfg in [int(x) for x in a.configs.split(",")]:
    g, W, H, mb, depth = WL[cfg]
    sc = rtamd.Scene().generate(g, 0, W / H)
    host_ms = []
    for _ in range(3):
        t0 = time.perf_counter()
        sc.buildBVH(depth)
        host_ms.append((time.perf_counter() - t0) * 1e3)
    fs = sc.serializeScene()
    out = torch.empty((H, W, 4), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()

    def render():
        ctx.set_params(W, H, mb, True)
        ctx.dispatch_rows(W, H, 0, 1, 1, H, out.data_ptr(), W * 16)
        ctx.sync()
        ctx.kernel_times()
        for _ in range(a.frames):
            ctx.dispatch_rows(W, H, 0, 1, 1, H, out.data_ptr(), W * 16)
        return float(np.median(ctx.kernel_times()))

    ctx.upload(fs)
    ref_ms = render()
    dev_ms, call_ms = [], []
    for _ in range(3):
        ctx.upload(fs)
        t0 = time.perf_counter()
        dev_ms.append(ctx.build_lbvh())
        call_ms.append((time.perf_counter() - t0) * 1e3)
    lbvh_ms = render()
    info = ctx.accel_info()
    S, N, _ = ctx.scene_size()
    print(json.dumps({
        "config": cfg, "shapes": S, "lbvh_nodes": N, "reference_nodes": len(fs.nodes),
        "host_reference_build_ms": round(min(host_ms), 3),
        "lbvh_device_build_ms": round(min(dev_ms), 3),
        "lbvh_device_Mshapes_per_s": round(S / min(dev_ms) / 1e3, 1),
        "rt_build_lbvh_call_ms": round(min(call_ms), 3),
        "render_ms_reference_tree": round(ref_ms, 4), "render_ms_lbvh_tree": round(lbvh_ms, 4),
        "scene_tree": info["scene_tree"]}))
ctx.close()
