"""A/B of two librtamd.so builds in the bench's regime: sustained ms per frame
with F frames in flight (F contexts, streams and surfaces). Each build runs in
its own child process (a second build loaded into one process does not overlap
its frames), alternating A, B, A, B ...; the image of every run is compared.

    python tools/abf.py --lib2 build_ab/REV/librtamd.so [--config 3] [--inflight 2] [--rounds 3] [--frames 200]
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

WL = {2: (2, 800, 600, 1), 3: (3, 1920, 1080, 3), 4: (3, 3840, 2160, 3), 5: (5, 1920, 1080, 3)}
ap = argparse.ArgumentParser()
ap.add_argument("--lib2", required=True)
ap.add_argument("--config", type=int, default=3)
ap.add_argument("--inflight", type=int, default=2)
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--frames", type=int, default=200)
ap.add_argument("--walk2", type=int, default=-1, help="walk policy (rt_set_walk) for the lib2 runs")
ap.add_argument("--set2", default="", help="lib2 settings, e.g. schedule=0,launch=2,walk=0")
ap.add_argument("--set", default="", help="settings for both builds, e.g. latency=1")
ap.add_argument("--nocheck", action="store_true", help="timing only: images may differ (experiments)")
ap.add_argument("--bounces", type=int, default=0, help="override maxBounces")
ap.add_argument("--mt", action="store_true", help="useMollerTrumbore = 1 frames")
ap.add_argument("--child", default=None, help=argparse.SUPPRESS)
a = ap.parse_args()

if a.child is None:
    import subprocess
    res = {"current": [], "lib2": []}
    ref = None
    for _ in range(a.rounds):
        for name in ("current", "lib2"):
            out = subprocess.run([sys.executable, __file__, "--lib2", a.lib2, "--config", str(a.config),
                                  "--inflight", str(a.inflight), "--frames", str(a.frames), "--bounces", str(a.bounces)] + (["--mt"] if a.mt else []) + ["--walk2", str(a.walk2), "--set2", a.set2, "--set", a.set, "--child", name],
                                 capture_output=True, text=True, check=True,
                                 # 2F hardware queues, as bench.plan_inflight sets (the box exports 4,
                                 # and F contexts on 4 shared queues run partly in order)
                                 env=dict(os.environ, GPU_MAX_HW_QUEUES=str(max(6, 2 * a.inflight)))
                                 ).stdout.strip().splitlines()[-1]
            r = json.loads(out)
            res[name].append(r["ms"])
            img = np.load(r["img"])
            ref = img if ref is None else ref
            diff = float(np.abs(img - ref).max())  # NaN if a pixel was not written
            assert a.nocheck or diff <= 1e-4, f"{name} renders an image {diff} away"
    print(json.dumps({"config": a.config, "inflight": a.inflight,
                      "ms_per_frame": {n: {"median": float(np.median(v)), "min": float(np.min(v))}
                                       for n, v in res.items()}}))
    sys.exit(0)

cfg, W, H, mb = WL[a.config]
mb = 0 if a.bounces < 0 else (a.bounces or mb)
fs = rtamd.generate(cfg, 0, W, H)
F = a.inflight
path = None if a.child == "current" else a.lib2
ctxs, bufs = [], []
for _ in range(F):
    s = torch.cuda.Stream()
    c = rtamd.ComputeShader(0, lib_path=path)
    c.set_stream(s.cuda_stream)
    c.upload(fs)
    c.set_params(W, H, mb, True, False, a.mt)
    if a.child == "lib2" and a.walk2 >= 0:
        c.set_walk(a.walk2)
    sets = ([a.set] if a.set else []) + ([a.set2] if a.child == "lib2" and a.set2 else [])
    for kv in ",".join(sets).split(",") if sets else []:
        if True:
            k, v = kv.split("=")
            {"schedule": lambda x: c.set_schedule(x), "launch": lambda x: c.set_launch(x, False),
             "persistent": lambda x: c.set_launch(1, bool(x)), "period": lambda x: c.debug_sched_period(x), "tail": lambda x: c.set_tail(x), "tlanes": lambda x: c.debug_tail_lanes(x), "shwalk": lambda x: c.debug_shadow_walk(x),
             "spec": lambda x: c.debug_spec(x), "stack": lambda x: c.debug_lane_stack(x),
             "walk": lambda x: c.set_walk(x), "tree": lambda x: c.set_tree(x),
             "latency": lambda x: c.set_latency_mode(x), "cone": lambda x: c.debug_cone_cull(x),
             "heavy": lambda x: c.debug_heavy(x // 100, x % 100), "costtime": lambda x: c.debug_cost_time(x),
             "lanek": lambda x: c.debug_lane_k(x // 10, x % 10)}[k](int(v))
    ctxs.append((c, s))
    bufs.append(torch.empty((H, W, 4), dtype=torch.float32, device="cuda"))


def run(n):
    for i in range(n):
        c, _ = ctxs[i % F]
        c.set_camera(fs.camera)
        c.set_light(fs.light)
        c.dispatch_rows(W, H, 0, 1, 1, H, bufs[i % F].data_ptr(), W * 16)


run(4 * F)
torch.cuda.synchronize()
t0 = time.perf_counter()
run(a.frames)
torch.cuda.synchronize()
ms = (time.perf_counter() - t0) / a.frames * 1e3
# the compared image: one more frame into a poisoned surface (no pixel may be left over)
bufs[0].fill_(float("nan"))
torch.cuda.synchronize()
run(1)
torch.cuda.synchronize()
imgpath = f"/tmp/abf_{a.child}_{os.getpid()}.npy"
np.save(imgpath, bufs[0].cpu().numpy())
print(json.dumps({"ms": ms, "img": imgpath}))
