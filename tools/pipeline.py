"""Frames in flight: F contexts on F streams render consecutive frames of the
same scene round-robin (frame n on context n % F, its own surface), so one
frame's tail overlaps the next frame's start. Prints frames/s per F.

    python tools/pipeline.py [--config 3] [--frames 200] [--inflight 1,2,3]
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

WL = {2: (2, 800, 600, 1), 3: (3, 1920, 1080, 3), 5: (5, 1920, 1080, 3)}
ap = argparse.ArgumentParser()
ap.add_argument("--config", type=int, default=3)
ap.add_argument("--frames", type=int, default=200)
ap.add_argument("--inflight", default="1,2,3")
a = ap.parse_args()
cfg, W, H, mb = WL[a.config]
fs = rtamd.generate(cfg, 0, W, H)
res = {}
for F in [int(x) for x in a.inflight.split(",")]:
    ctxs, bufs, streams = [], [], []
    for _ in range(F):
        s = torch.cuda.Stream()
        c = rtamd.ComputeShader(0)
        c.set_stream(s.cuda_stream)
        c.upload(fs)
        c.set_params(W, H, mb, True)
        ctxs.append(c)
        streams.append(s)
        bufs.append(torch.empty((H, W, 4), dtype=torch.float32, device="cuda"))
    torch.cuda.synchronize()

    def run(n):
        for i in range(n):
            c = ctxs[i % F]
            c.set_camera(fs.camera)
            c.set_light(fs.light)
            c.dispatch_rows(W, H, 0, 1, 1, H, bufs[i % F].data_ptr(), W * 16)

    run(10 * F)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(a.frames)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    res[F] = {"ms_per_frame": dt / a.frames * 1e3, "fps": a.frames / dt}
    for c in ctxs:
        c.close()
print(json.dumps({"config": a.config, "frames": a.frames, "inflight": res}))
