#!/usr/bin/env python3
"""One rank's share of a strong-scaled car frame on the current build:
the rows rank r renders when P GPUs split the frame into interleaved 8-row stripes
(root share 1: rank r takes {y : (y / 8) mod P == r}), timed

  * waited, one frame at a time from the C++ host loop (librthost.so
    rth_render_rows_loop: camera + light upload, rt_dispatch_rows_ex, rt_sync), with
    and without rt_set_latency_mode -- the per-rank floor of a waited strong frame;
  * with F frames in flight (F contexts on their own streams), the per-rank
    throughput floor;
  * in latency mode, over the heavy-tile split (rt_debug_heavy: the heaviest k tiles
    as `parts` waves), since the auto setting (tiles / 200 as 4 waves) was swept on
    whole frames only.

    [RT_HW_QUEUES=16] python tools/share_sweep.py [--sizes 1080,2160] [--parts 1,2,4,8]
Prints one JSON object.
"""
import argparse
import json
import os
import sys
import time

# before the HIP runtime starts; set, not defaulted: the GPU box exports 4, and with 4
# queues F = 8 contexts share them and run in order (r05's in-flight share figures were
# taken that way: 1/8 share 0.050 ms at F = 8, 0.031 with 8 or 16 queues, r06f)
os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("RT_HW_QUEUES", "16")

import numpy as np  # noqa: E402
import torch  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "opengl-ray-tracer_amd"))
import rtamd  # noqa: E402


def rank_rows(H, P, r, stripe=8):
    return sum(1 for y in range(H) if (y // stripe) % P == r)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1080,2160")
    ap.add_argument("--parts", default="1,2,4,8")
    ap.add_argument("--waited", type=int, default=150)
    ap.add_argument("--inflight", default="1,2,4,8")
    ap.add_argument("--frames", type=int, default=400)
    ap.add_argument("--sweep", type=int, default=1, help="latency-mode heavy-split sweep (1080p)")
    ap.add_argument("--sweep-parts", default="2,4", help="waves per split tile in the sweep")
    ap.add_argument("--sweep-div", default="800,400,200,100,50", help="split k = tiles / each")
    a = ap.parse_args()
    out = {"GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES"), "shares": []}
    for Hs in [int(x) for x in a.sizes.split(",")]:
        H = Hs
        W = H * 16 // 9
        fs = rtamd.generate(3, 0, W, H)
        for P in [int(x) for x in a.parts.split(",")]:
            for r in ([0] if P == 1 else [0, 1]):
                rows = rank_rows(H, P, r)
                tiles = ((W + 7) // 8) * ((rows + 7) // 8)
                rec = {"W": W, "H": H, "P": P, "rank": r, "rows": rows, "tiles": tiles}
                ctx = rtamd.ComputeShader(0)
                ctx.upload(fs)
                ctx.set_params(W, H, 3, True)
                ctx.set_kernel_timing(0)
                buf = torch.empty((rows, W, 3), dtype=torch.float32, device="cuda")
                torch.cuda.synchronize()

                def waited(n=a.waited):
                    rtamd.render_rows_loop(ctx, fs.camera, fs.light, W, H, 8 * r, 8, 8 * P, rows, buf.data_ptr(),
                                           W * 12, 48, True)
                    ms = rtamd.render_rows_loop(ctx, fs.camera, fs.light, W, H, 8 * r, 8, 8 * P, rows,
                                                buf.data_ptr(), W * 12, n, True)
                    return float(np.median(ms))

                rec["waited_ms"] = waited()
                ctx.set_latency_mode(1)
                rec["waited_latency_mode_ms"] = waited()
                if a.sweep and H == 1080:
                    sw = {}
                    for k in sorted({max(16, tiles // int(d)) for d in a.sweep_div.split(",")}):
                        for parts in [int(x) for x in a.sweep_parts.split(",")]:
                            ctx.debug_heavy(k, parts)
                            sw[f"{k}x{parts}"] = waited(100)
                    ctx.debug_heavy(-1, 1)
                    rec["latency_heavy_sweep_ms"] = sw
                ctx.set_latency_mode(0)
                ctx.close()
                # F frames in flight
                for F in [int(x) for x in a.inflight.split(",")]:
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
                    torch.cuda.synchronize()
                    for i in range(32 * F):
                        ctxs[i % F].dispatch_rows_ex(W, H, 8 * r, 8, 8 * P, rows, bufs[i % F].data_ptr(), W * 12,
                                                     fmt=rtamd.FORMAT_RGB32F)
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    for i in range(a.frames):
                        ctxs[i % F].dispatch_rows_ex(W, H, 8 * r, 8, 8 * P, rows, bufs[i % F].data_ptr(), W * 12,
                                                     fmt=rtamd.FORMAT_RGB32F)
                    torch.cuda.synchronize()
                    rec[f"inflight_F{F}_ms"] = (time.perf_counter() - t0) / a.frames * 1e3
                    for c in ctxs:
                        c.close()
                out["shares"].append(rec)
                print(json.dumps(rec), file=sys.stderr, flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
