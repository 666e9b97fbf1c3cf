"""A/B timing of render-kernel variants in one process (interleaved rounds).

    python tools/ab.py [--config 3] [--rounds 5] [--frames 20] [--times]

Prints median device ms per variant (HIP events) and checks that every
variant renders the identical image.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "opengl-ray-tracer_amd"))
import rtamd  # noqa: E402

WL = {2: (2, 800, 600, 1), 3: (3, 1920, 1080, 3), 4: (3, 3840, 2160, 3), 5: (5, 1920, 1080, 3)}
VARIANTS = {
    "default": dict(kernel=0, wpb=1, persistent=False, walk=1),
    "hybrid_w2": dict(kernel=3, wpb=2, persistent=False, walk=1),
    "hybrid_w4": dict(kernel=3, wpb=4, persistent=False, walk=1),
    "lane_all": dict(kernel=3, wpb=1, persistent=False, walk=0),
    "packet_all": dict(kernel=3, wpb=1, persistent=False, walk=99),
    "lane_from2": dict(kernel=3, wpb=1, persistent=False, walk=2),
    "persistent": dict(kernel=3, wpb=1, persistent=True, walk=1),
    "nocone": dict(kernel=3, wpb=1, persistent=False, walk=1, cone=0),
    "packet": dict(kernel=2, wpb=4, persistent=False, walk=1),
    "lpt": dict(kernel=3, wpb=1, persistent=False, walk=1, order="lpt"),
    "mix1": dict(kernel=3, wpb=1, persistent=False, walk=1, order="mix1"),
    "mix3": dict(kernel=3, wpb=1, persistent=False, walk=1, order="mix3"),
    "mix7": dict(kernel=3, wpb=1, persistent=False, walk=1, order="mix7"),
    "rows": dict(kernel=3, wpb=1, persistent=False, walk=1, sched=0),
    "spec_on": dict(kernel=3, wpb=1, persistent=False, walk=1, spec=1),
    "spec_off": dict(kernel=3, wpb=1, persistent=False, walk=1, spec=0),
    "lpt_rows": dict(kernel=3, wpb=1, persistent=False, walk=1, order="rows"),
    "stack20": dict(kernel=3, wpb=1, persistent=False, walk=1, stack=20),
    "stack16": dict(kernel=3, wpb=1, persistent=False, walk=1, stack=16),
    "reftree": dict(kernel=3, wpb=1, persistent=False, walk=1, tree=0),
    "reftree_lane": dict(kernel=3, wpb=1, persistent=False, walk=0, tree=0),
}

ap = argparse.ArgumentParser()
ap.add_argument("--config", type=int, default=3)
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--frames", type=int, default=20)
ap.add_argument("--variants", default="default,lane_all,packet_all,hybrid_w2")
ap.add_argument("--bounces", type=int, default=0, help="override maxBounces")
ap.add_argument("--times", action="store_true", help="per-tile wall-clock distribution")
ap.add_argument("--lib2", default=None, help="second librtamd.so build: variants NAME@2 run on it")
a = ap.parse_args()
cfg, W, H, mb = WL[a.config]
mb = a.bounces or mb
fs = rtamd.generate(cfg, 0, W, H)
ctxs = {}
for key, path in (("", None), ("@2", a.lib2)):
    if key and not path:
        continue
    cx = rtamd.ComputeShader(0, lib_path=path)
    cx.upload(fs)
    cx.set_params(W, H, mb, True)
    ctxs[key] = cx
out = torch.empty((H, W, 4), dtype=torch.float32, device="cuda")
torch.cuda.synchronize()
names = a.variants.split(",")
tiles_n = ((W + 7) // 8) * ((H + 7) // 8)
orders = {}
if any(VARIANTS[n.partition("@")[0]].get("order") for n in names):
    # longest-processing-time-first dispatch from one measured frame (diagnostics:
    # the upper bound of what a cost-ordered dispatch can recover)
    cx = ctxs[""]
    cx.set_kernel(3)
    cx.debug_tile_times(tiles_n)
    cx.dispatch_rows(W, H, 0, 1, 1, H, torch.empty((H, W, 4), dtype=torch.float32, device="cuda").data_ptr(), W * 16)
    tt = cx.tile_times(tiles_n).astype(np.int64)
    cx.debug_tile_times(0)
    d = tt[:, 1] - tt[:, 0]
    orders["lpt"] = np.argsort(-d, kind="stable").astype(np.int32)
    # heaviest tiles interleaved with the lightest, k light per heavy, so that a
    # heavy wave shares its SIMD with short ones rather than with other heavy ones
    for k in (1, 3, 7):
        desc = orders["lpt"]
        nh = len(desc) // (k + 1)
        heavy, light = desc[:nh], desc[nh:][::-1]
        mix = []
        for q in range(nh):
            mix.append(heavy[q])
            mix.extend(light[q * k:(q + 1) * k])
        mix.extend(light[nh * k:])
        orders[f"mix{k}"] = np.array(mix, np.int32)
    rowcost = d.reshape((H + 7) // 8, -1).sum(axis=1)
    orders["rows"] = np.concatenate([np.arange(r * ((W + 7) // 8), (r + 1) * ((W + 7) // 8))
                                     for r in np.argsort(-rowcost, kind="stable")]).astype(np.int32)


def pick(n):
    base, _, tag = n.partition("@")
    return ctxs["@" + tag if tag else ""], VARIANTS[base]


res = {n: [] for n in names}
ref = None
for rnd in range(a.rounds):
    for n in names:
        ctx, v = pick(n)
        ctx.set_kernel(v["kernel"])
        ctx.set_launch(v["wpb"], v["persistent"])
        ctx.set_walk(v["walk"])
        ctx.debug_cone_cull(v.get("cone", 1))
        if hasattr(ctx._lib, "rt_debug_tile_order"):
            ctx.debug_tile_order(orders.get(v.get("order")))
        if hasattr(ctx._lib, "rt_set_schedule"):
            ctx.set_schedule(v.get("sched", 1))
        if hasattr(ctx._lib, "rt_debug_spec"):
            ctx.debug_spec(v.get("spec", 1))
        if hasattr(ctx._lib, "rt_debug_lane_stack"):
            ctx.debug_lane_stack(v.get("stack", 0))
        if hasattr(ctx._lib, "rt_set_tree"):
            ctx.set_tree(v.get("tree", 1))
        ctx.dispatch_rows(W, H, 0, 1, 1, H, out.data_ptr(), W * 16)
        ctx.sync()
        img = out.cpu().numpy()
        if ref is None:
            ref = img
        assert np.array_equal(img, ref) or "stack" in n or float(np.abs(img - ref).max()) <= 1e-4, \
            f"{n} renders a different image"
        ctx.kernel_times()
        for _ in range(a.frames):
            ctx.dispatch_rows(W, H, 0, 1, 1, H, out.data_ptr(), W * 16)
        res[n].extend(ctx.kernel_times().tolist())
summary = {n: {"median_ms": float(np.median(t)), "min_ms": float(np.min(t))} for n, t in res.items()}
print(json.dumps({"config": a.config, "maxBounces": mb, "variants": summary}))
if a.times:
    tiles = ((W + 7) // 8) * ((H + 7) // 8)
    for n in names:
        ctx, v = pick(n)
        ctx.set_kernel(v["kernel"])
        ctx.set_launch(v["wpb"], v["persistent"])
        ctx.set_walk(v["walk"])
        ctx.debug_cone_cull(v.get("cone", 1))
        if hasattr(ctx._lib, "rt_debug_tile_order"):
            ctx.debug_tile_order(orders.get(v.get("order")))
        if hasattr(ctx._lib, "rt_set_schedule"):
            ctx.set_schedule(v.get("sched", 1))
        if hasattr(ctx._lib, "rt_debug_spec"):
            ctx.debug_spec(v.get("spec", 1))
        if hasattr(ctx._lib, "rt_debug_lane_stack"):
            ctx.debug_lane_stack(v.get("stack", 0))
        if hasattr(ctx._lib, "rt_set_tree"):
            ctx.set_tree(v.get("tree", 1))
        ctx.debug_tile_times(tiles)
        ctx.dispatch_rows(W, H, 0, 1, 1, H, out.data_ptr(), W * 16)
        t = ctx.tile_times(tiles).astype(np.int64)
        ctx.debug_tile_times(0)
        dur = (t[:, 1] - t[:, 0]) / 100.0  # us (100 MHz)
        start = (t[:, 0] - t[:, 0].min()) / 100.0
        end = (t[:, 1] - t[:, 0].min()) / 100.0
        q = np.percentile(dur, [50, 90, 99, 100])
        print(json.dumps({"variant": n, "tile_us_p50_p90_p99_max": q.round(1).tolist(), "tile_us_mean": float(dur.mean()),
                          "span_us": float(end.max()), "last_start_us": float(start.max()),
                          "sum_tile_us": float(dur.sum())}))
        rows = (H + 7) // 8
        per_row = dur.reshape(rows, -1).mean(axis=1)
        print("  mean tile us by tile-row (every 10th):", per_row[::10].round(1).tolist())
        tx = (W + 7) // 8
        worst = np.argsort(dur)[::-1][:6]
        print("  slowest tiles (x8, y8, us, nodes sum/max-lane/wave-iters, tests sum/max-lane/wave-iters):",
              [(int(w % tx) * 8, int(w // tx) * 8, round(float(dur[w]), 1), int(t[w, 2]), int(t[w, 4]), int(t[w, 23]),
                int(t[w, 3]), int(t[w, 5]), int(t[w, 22])) for w in worst])
        med = np.argsort(dur)[len(dur) // 2]
        print("  median tile:", (round(float(dur[med]), 1), int(t[med, 2]), int(t[med, 4]), int(t[med, 3]), int(t[med, 5])))
        print("  totals: nodes", int(t[:, 2].sum()), "tests", int(t[:, 3].sum()))
        cyc, nod = t[:, 6:14].sum(axis=0), t[:, 14:22].sum(axis=0)
        tot = cyc.sum()
        for sl in range(min(2 * mb, 8)):
            print(f"  bounce {sl // 2} {'shadow ' if sl % 2 else 'closest'}: wave-Mcycles {cyc[sl] / 1e6:8.1f}"
                  f" ({100.0 * cyc[sl] / max(tot, 1):4.1f}%) lane node steps {nod[sl] / 1e6:7.2f} M")
        slow = np.argsort(dur)[::-1][:32]
        print("  slowest 32 tiles, share of wave cycles per walk:",
              (t[slow, 6:6 + 2 * mb].sum(axis=0) / max(t[slow, 6:6 + 2 * mb].sum(), 1)).round(3).tolist())
        # concurrency profile: tiles in flight over the kernel's span, in 20 slices
        span = float(end.max())
        edges = np.linspace(0.0, span, 21)
        live = [int(((start < b) & (end > a_)).sum()) for a_, b in zip(edges[:-1], edges[1:])]
        print("  tiles in flight per 5% of span:", live)
        busy = np.zeros(400)
        grid = np.linspace(0.0, span, 401)
        for s_, e_ in zip(start, end):
            i0, i1 = np.searchsorted(grid, [s_, e_])
            busy[max(i0 - 1, 0):i1] += 1
        print("  mean tiles resident over span:", round(float(busy.mean()), 1),
              " time with < 1000 / < 250 resident: %.0f%% / %.0f%%" % (100 * (busy < 1000).mean(), 100 * (busy < 250).mean()))
