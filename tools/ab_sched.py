"""A/B of walk settings in one process: for each config, alternate the modes
over several rounds (so clock drift hits all), with F frames in flight and one
at a time, and check that every mode gives the same image as the first.

    python tools/ab_sched.py [--configs 3,5,2] [--modes 1,2] [--frames 200] [--rounds 4]
        modes: tile schedules (rt_set_schedule)
    python tools/ab_sched.py --split 0:8,16:8,8:8
        modes: split walks, max_rays:group (rt_debug_split; 0 = off)
    python tools/ab_sched.py --heavy 0:1,256:4
        modes: heaviest tiles as several waves, k:parts (rt_debug_heavy)
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

WL = {2: (2, 800, 600, 1), 3: (3, 1920, 1080, 3), 4: (3, 3840, 2160, 3), 5: (5, 1920, 1080, 3)}
ap = argparse.ArgumentParser()
ap.add_argument("--configs", default="3,5,2")
ap.add_argument("--modes", default="1,2")
ap.add_argument("--frames", type=int, default=200)
ap.add_argument("--rounds", type=int, default=4)
ap.add_argument("--inflight", type=int, default=2)
ap.add_argument("--split", default="")
ap.add_argument("--heavy", default="", help="modes k:parts (rt_debug_heavy)")
ap.add_argument("--lanek", default="", help="modes k:mode (rt_debug_lane_k)")
ap.add_argument("--latency", default="", help="modes 0/1 (rt_set_latency_mode)")
ap.add_argument("--with-latency", action="store_true", help="latency mode on under every mode")
ap.add_argument("--bounces", type=int, default=0, help="maxBounces override (0: the config's)")
ap.add_argument("--share", type=int, default=1, help="render rank 0's 8-row stripes of a P-rank frame")
a = ap.parse_args()
alt = a.split or a.heavy or a.lanek or a.latency
modes = alt.split(",") if alt else [int(m) for m in a.modes.split(",")]


def apply(c, m):
    if a.latency:
        c.set_latency_mode(int(m))
    elif a.lanek:
        k, mode = (int(v) for v in m.split(":"))
        c.debug_lane_k(k, mode)
    elif a.heavy:
        k, parts = (int(v) for v in m.split(":"))
        c.debug_heavy(k, parts)
    elif a.split:
        mx, g = (int(v) for v in m.split(":"))
        c.debug_split(mx, g)
    else:
        c.set_schedule(m)

out = {}
for cfg in [int(x) for x in a.configs.split(",")]:
    scene, W, H, mb = WL[cfg]
    mb = a.bounces or mb
    fs = rtamd.generate(scene, 0, W, H)
    P = a.share
    R = H if P == 1 else sum(min(8, max(0, H - y)) for y in range(0, H, 8 * P))  # rank 0's rows
    F = a.inflight
    # one set of F contexts for every mode (modes switch between timed runs), so
    # that no mode gets streams the others lack
    ctxs, bufs = [], []
    for _ in range(F):
        s = torch.cuda.Stream()
        c = rtamd.ComputeShader(0)
        c.set_stream(s.cuda_stream)
        c.upload(fs)
        c.set_params(W, H, mb, True)
        if a.with_latency:
            c.set_latency_mode(1)
        ctxs.append((c, s))
        bufs.append(torch.empty((R, W, 4), dtype=torch.float32, device="cuda"))
    torch.cuda.synchronize()

    def run(n, f):
        for i in range(n):
            c, _ = ctxs[i % f]
            c.set_camera(fs.camera)
            c.set_light(fs.light)
            if P == 1:
                c.dispatch_rows(W, H, 0, 1, 1, H, bufs[i % f].data_ptr(), W * 16)
            else:
                c.dispatch_rows(W, H, 0, 8, P, R, bufs[i % f].data_ptr(), W * 16)
            if f == 1:
                torch.cuda.synchronize()

    res = {m: {"inflight": [], "serial": []} for m in modes}
    img = {}
    for _ in range(a.rounds):
        for m in modes:
            torch.cuda.synchronize()
            for c, _ in ctxs:
                apply(c, m)
            run(10 * F, F)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            run(a.frames, F)
            torch.cuda.synchronize()
            res[m]["inflight"].append((time.perf_counter() - t0) / a.frames * 1e3)
            t0 = time.perf_counter()
            run(a.frames // 2, 1)
            res[m]["serial"].append((time.perf_counter() - t0) / (a.frames // 2) * 1e3)
            img[m] = bufs[0].clone()
    torch.cuda.synchronize()
    same = {m: bool(torch.equal(img[m], img[modes[0]])) for m in modes}
    out[cfg] = {
        m: {
            "ms_inflight_min": min(r["inflight"]),
            "ms_inflight_med": sorted(r["inflight"])[len(r["inflight"]) // 2],
            "ms_serial_min": min(r["serial"]),
            "ms_serial_med": sorted(r["serial"])[len(r["serial"]) // 2],
            "image_equal": same[m],
        }
        for m, r in res.items()
    }
    for c, _ in ctxs:
        c.close()
    print(json.dumps({"config": cfg, "F": F, "share": P, "modes": out[cfg]}), flush=True)
