#!/usr/bin/env python3
"""Fixed cost of the rt_group path against frames mode on one GPU.

    python tools/group_cost.py [--frames 200] [--blocks 3]

Variants, each in its own child process (so that no variant's streams share the
hardware queues with another's), alternated over blocks:
  A_frames            frames mode (bench.py frames): F contexts on F streams,
                      frame i on context i mod F, kernel timing events on;
  A_frames_notiming   the same with rt_set_kernel_timing(0);
  A_own_notiming      the contexts on their own rt_create streams (not torch's);
  A_own_cumask_notiming  the same with RT_STREAMS_CUMASK=1 (a hardware queue each);
  B_group             a 1-rank RCCL group with F frame slots (bench.py --mode
                      strong at N = 1), phase and kernel timing on;
  C_group_notiming    the same with rt_group_set_phase_timing(0) and
                      rt_set_kernel_timing(0) on its contexts.
Per variant: host microseconds per frame call, sustained ms per frame with F in
flight, and the median waited frame (latency mode on, each frame waited for by
the renderer's own wait: rt_sync / rt_group_sync). Each child checks its last
frame bit for bit against a single context's frame. One JSON line (medians over
blocks).
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VARIANTS = ("A_frames", "A_frames_notiming", "A_own_notiming", "A_own_cumask_notiming", "B_group", "C_group_notiming")
ENV = {"A_own_cumask_notiming": {"RT_STREAMS_CUMASK": "1"}}


def child(a):
    os.environ.setdefault("GPU_MAX_HW_QUEUES", str(2 * a.inflight))
    sys.path.insert(0, os.path.join(ROOT, "opengl-ray-tracer_amd"))
    import numpy as np
    import torch
    import rtamd
    W, H, F = 1920, 1080, a.inflight
    name = a.variant
    timing = not name.endswith("_notiming")
    fs = rtamd.generate(3, 0, W, H)
    torch.cuda.set_device(0)
    ref_ctx = rtamd.ComputeShader(0)
    ref_ctx.upload(fs)
    ref_ctx.set_params(W, H, 3)
    ref = ref_ctx.render(W, H)
    ref_ctx.close()
    if name.startswith("A_"):
        own = name.startswith("A_own")
        streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(F - 1)]
        cs, bufs = [], []
        for st in streams:
            c = rtamd.ComputeShader(0)
            if not own:  # else the context's own stream (rt_create; RT_STREAMS_CUMASK: own queue)
                c.set_stream(st.cuda_stream)
            c.upload(fs)
            c.set_params(W, H, 3)
            c.set_kernel_timing(timing)
            cs.append(c)
            bufs.append(torch.empty((H, W, 4), dtype=torch.float32, device="cuda"))

        def fr(i):
            c = cs[i % F]
            c.set_camera(fs.camera)
            c.set_light(fs.light)
            c.dispatch_rows(W, H, 0, 1, 1, H, bufs[i % F].data_ptr(), W * 16)

        def sync():
            for c in cs:
                c.sync()

        def last():
            sync()
            return bufs[(n_all - 1) % F].cpu().numpy()
    else:
        g = rtamd.Group(uid=rtamd.group_unique_id(), nranks=1, rank=0, device=0, frames=F)
        g.upload(fs)
        g.set_params(W, H, 3)
        g.set_phase_timing(timing)
        cs = g.contexts
        for c in cs:
            c.set_kernel_timing(timing)

        def fr(i):
            g.set_camera(fs.camera)
            g.set_light(fs.light)
            g.dispatch(W, H, 8)

        sync = g.sync

        def last():
            return g.read_image(W, H)
    n_all = 0
    for i in range(20):
        fr(i)
        n_all += 1
    sync()
    t0 = time.perf_counter()
    host = 0.0
    for i in range(a.frames):
        h0 = time.perf_counter()
        fr(i)
        n_all += 1
        host += time.perf_counter() - h0
    sync()
    el = time.perf_counter() - t0
    for c in cs:
        c.set_latency_mode(1)
    w = []
    for i in range(a.frames):
        t1 = time.perf_counter()
        fr(i)
        n_all += 1
        sync()
        w.append(time.perf_counter() - t1)
    print(json.dumps({"host_us": host / a.frames * 1e6, "inflight_ms": el / a.frames * 1e3,
                      "waited_ms": float(np.median(w)) * 1e3,
                      "image_equal": bool(np.array_equal(last(), ref))}), flush=True)
    os._exit(0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=200)
    ap.add_argument("--blocks", type=int, default=3)
    ap.add_argument("--inflight", type=int, default=3)
    ap.add_argument("--variant", default=None, choices=VARIANTS)
    a = ap.parse_args()
    if a.variant:
        return child(a)
    import statistics
    res = {v: [] for v in VARIANTS}
    for _ in range(a.blocks):
        for v in VARIANTS:
            r = subprocess.run([sys.executable, os.path.abspath(__file__), "--variant", v, "--frames", str(a.frames),
                                "--inflight", str(a.inflight)], capture_output=True, text=True, timeout=240,
                               env=dict(os.environ, **ENV.get(v, {})))
            if r.returncode != 0:
                print(r.stderr[-2000:], file=sys.stderr)
                sys.exit(r.returncode)
            res[v].append(json.loads(r.stdout.strip().splitlines()[-1]))
    out = {v: {k: statistics.median(x[k] for x in rs) for k in ("host_us", "inflight_ms", "waited_ms")}
           for v, rs in res.items()}
    for v, rs in res.items():
        out[v]["image_equal"] = all(x["image_equal"] for x in rs)
        out[v]["blocks"] = [{k: round(x[k], 4) for k in ("inflight_ms", "waited_ms")} for x in rs]
    out["frames"], out["inflight"] = a.frames, a.inflight
    print(json.dumps(out))


if __name__ == "__main__":
    main()
