"""Animated frames on config 3: the four wheels (640 triangles) turn every
frame (updateWheelAnimations, src/main.cpp:1084-1109, stored normals left as
they were), and the tree is refit on the device (rt_animate) before the render.

    python tools/bench_animate.py [--frames 120] [--width 1920 --height 1080]

Reports, per frame: the host time of rt_animate (class checks + one pinned
upload + two kernel launches), the device time of the whole frame
(animate + render, HIP events on the context stream), the render alone on the
static scene, and the host path the reference's own per-frame upload would
take through this library (rt_update_shapes + rt_update_nodes, which rebuild
the accelerator on the host). Also checks that the refit frame equals the
host-path frame at the end.
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

ap = argparse.ArgumentParser()
ap.add_argument("--frames", type=int, default=120)
ap.add_argument("--width", type=int, default=1920)
ap.add_argument("--height", type=int, default=1080)
ap.add_argument("--host-frames", type=int, default=10)
a = ap.parse_args()
W, H = a.width, a.height
fs = rtamd.generate(3, 0, W, H)
WHEELS = [np.arange(3380 + 160 * w, 3380 + 160 * (w + 1)) for w in range(4)]  # gen_car: body, 4 wheels, road
ids = np.concatenate(WHEELS).astype(np.int32)
assert (fs.shapes["type"][ids] == 3).all()


def rot_z(p, c, ang):
    q = p.astype(np.float64) - c
    cs, sn = np.cos(ang), np.sin(ang)
    return (np.stack([q[:, 0] * cs - q[:, 1] * sn, q[:, 0] * sn + q[:, 1] * cs, q[:, 2]], 1) + c).astype(np.float32)


centres = []
for w in WHEELS:
    v = np.concatenate([fs.shapes[f][w] for f in ("triP1", "triP2", "triP3")]).astype(np.float64)
    centres.append(v.mean(0))


def step(rec, dt):
    out = rec.copy()
    for w, c in zip(range(4), centres):
        sl = slice(160 * w, 160 * (w + 1))
        for f in ("triP1", "triP2", "triP3"):
            out[f][sl] = rot_z(rec[f][sl], c, 1.0 * dt)
    return out


frames = []
rec = fs.shapes[ids].copy()
for k in range(a.frames):
    rec = step(rec, 1 / 60)
    frames.append(rec)

ctx = rtamd.ComputeShader(0)
ctx.upload(fs)
ctx.set_params(W, H, 3, True)
ctx.set_animated(ids)
out = torch.empty((H, W, 4), dtype=torch.float32, device="cuda")
torch.cuda.synchronize()
stream = torch.cuda.Stream()
ctx.set_stream(stream.cuda_stream)

# static render alone
for _ in range(5):
    ctx.dispatch_rows(W, H, 0, 1, 1, H, out.data_ptr(), W * 16)
ctx.sync()
ctx.kernel_times()
for _ in range(20):
    ctx.dispatch_rows(W, H, 0, 1, 1, H, out.data_ptr(), W * 16)
ctx.sync()
render_ms = float(np.median(ctx.kernel_times()))

# animated frames: animate + render, device time between events on the context stream
ev0 = torch.cuda.Event(enable_timing=True)
ev1 = torch.cuda.Event(enable_timing=True)
host_ms = []
ctx.sync()
with torch.cuda.stream(stream):
    ev0.record(stream)
    for rec in frames:
        t0 = time.perf_counter()
        ctx.animate(rec)
        host_ms.append((time.perf_counter() - t0) * 1e3)
        ctx.dispatch_rows(W, H, 0, 1, 1, H, out.data_ptr(), W * 16)
    ev1.record(stream)
ctx.sync()
stream.synchronize()
frame_ms = ev0.elapsed_time(ev1) / len(frames)
per_render = np.asarray(ctx.kernel_times(), np.float64)
refit_img = out.cpu().numpy().copy()
nodes = ctx.read_nodes(len(fs.nodes))

# the host path for the same last frame: update_shapes + update_nodes (accelerator rebuilt on the host)
ctx2 = rtamd.ComputeShader(0)
ctx2.upload(fs)
ctx2.set_params(W, H, 3, True)
shapes = fs.shapes.copy()
shapes[ids] = frames[-1]
t_host = []
for _ in range(a.host_frames):
    t0 = time.perf_counter()
    ctx2.update_shapes(int(ids[0]), shapes[ids[0]:ids[-1] + 1])
    ctx2.update_nodes(nodes)
    t_host.append((time.perf_counter() - t0) * 1e3)
host_img = ctx2.render(W, H)
same = bool(np.array_equal(host_img, refit_img))
print(json.dumps({
    "workload": f"config 3 {W}x{H}, 640 wheel triangles animated",
    "frames": len(frames),
    "render_static_ms": round(render_ms, 4),
    "frame_animate_render_ms": round(frame_ms, 4),
    "rt_animate_host_ms_median": round(float(np.median(host_ms)), 4),
    "rt_animate_host_ms_max": round(float(np.max(host_ms)), 3),
    "host_rebuilds": ctx.debug_anim_rebuilds(),
    "render_ms_first10": round(float(per_render[:10].mean()), 4),
    "render_ms_last10": round(float(per_render[-10:].mean()), 4),
    "host_path_update_ms_median": round(float(np.median(t_host)), 3),
    "refit_frame_equals_host_path_frame": same,
}))
ctx.close()
ctx2.close()
