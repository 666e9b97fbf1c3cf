#!/usr/bin/env python3
"""Host cost of issuing frames: how long the host spends in the calls
that queue one frame, against the frame's device time, for one rank's 1/P share of
the 1080p car (interleaved 8-row stripes) with F frames in flight.

  * issue_us_per_frame: wall time of the issue loop alone (no wait), per frame --
    from Python (one rt_dispatch_rows_ex per frame) and from the C++ host loop
    (rth_render_rows_loop without waits: camera, light, dispatch per frame);
  * ms_per_frame: the same frames including the final wait (the throughput).
If issue_us_per_frame ~ ms_per_frame, the host, not the GPU, bounds the share.

    GPU_MAX_HW_QUEUES=16 python tools/host_cost.py [--parts 8] [--inflight 8]
"""
import argparse
import json
import os
import sys
import time

os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("RT_HW_QUEUES", "16")  # the box exports 4: override before the runtime starts

import numpy as np  # noqa: E402
import torch  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "opengl-ray-tracer_amd"))
import rtamd  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--parts", default="1,8")
ap.add_argument("--inflight", type=int, default=8)
ap.add_argument("--frames", type=int, default=400)
ap.add_argument("--group", type=int, default=1, help="also a copy-transport group of P members on this GPU")
a = ap.parse_args()
W, H = 1920, 1080
fs = rtamd.generate(3, 0, W, H)
out = {"GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES"), "F": a.inflight, "cases": []}
for P in [int(x) for x in a.parts.split(",")]:
    rows = sum(1 for y in range(H) if (y // 8) % P == 0)
    F = a.inflight
    ctxs, bufs = [], []
    for _ in range(F):
        s = torch.cuda.Stream()
        c = rtamd.ComputeShader(0)
        c.set_stream(s.cuda_stream)
        c.upload(fs)
        c.set_params(W, H, 3, True)
        c.set_kernel_timing(0)
        ctxs.append(c)
        bufs.append(torch.empty((rows, W, 3), dtype=torch.float32, device="cuda"))

    def issue(n):
        for i in range(n):
            ctxs[i % F].dispatch_rows_ex(W, H, 0, 8, 8 * P, rows, bufs[i % F].data_ptr(), W * 12,
                                         fmt=rtamd.FORMAT_RGB32F)

    issue(32 * F)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    issue(a.frames)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    rec = {"P": P, "rows": rows, "py_issue_us_per_frame": (t1 - t0) / a.frames * 1e6,
           "py_ms_per_frame": (t2 - t0) / a.frames * 1e3}
    # the C++ host loop on one context (no waits): camera + light + dispatch per frame
    ms = rtamd.render_rows_loop(ctxs[0], fs.camera, fs.light, W, H, 0, 8, 8 * P, rows, bufs[0].data_ptr(), W * 12,
                                a.frames, False)
    rec["cpp_one_ctx_ms_per_frame"] = float(ms[0]) / a.frames
    for c in ctxs:
        c.close()
    if a.group and P > 1:
        g = rtamd.Group([0] * P, rtamd.GATHER_COPY, frames=F)
        g.upload(fs)
        g.set_params(W, H, 3)
        g.set_phase_timing(False)
        for _ in range(32):
            g.dispatch(W, H, 8)
        g.sync()
        t0 = time.perf_counter()
        for _ in range(a.frames // 4):
            g.set_camera(fs.camera)
            g.set_light(fs.light)
            g.dispatch(W, H, 8)
        t1 = time.perf_counter()
        g.sync()
        t2 = time.perf_counter()
        n = a.frames // 4
        rec["group_copy_members"] = P
        rec["group_issue_us_per_frame"] = (t1 - t0) / n * 1e6
        rec["group_ms_per_frame"] = (t2 - t0) / n * 1e3
        g.close()
    out["cases"].append(rec)
    print(json.dumps(rec), file=sys.stderr, flush=True)
print(json.dumps(out), flush=True)
