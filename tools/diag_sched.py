"""Diagnostics: repeat test_cost_schedule_identical_images' loop for several builds and
report, per build and schedule, how many frames differ from the row-major frame and
whether the differing pixels are unwritten (NaN) or different values."""
import sys
import os
import json
import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "opengl-ray-tracer_amd"))
import rtamd  # noqa: E402

libs = [a or None for a in sys.argv[1:]] or [None]
for lib in libs:
    ctx = rtamd.ComputeShader(0, lib_path=lib)
    fs = rtamd.generate(3, 0, 320, 180)
    ctx.upload(fs)
    ctx.set_params(320, 180, 3, True)
    ctx.set_kernel(rtamd.KERNEL_ACCEL)
    out = {}
    for sched in (rtamd.SCHED_COST, rtamd.SCHED_COST_XCD):
        ctx.set_schedule(rtamd.SCHED_ROWS)
        ref = ctx.render(320, 180)
        ctx.set_schedule(sched)
        full = torch.empty((180, 320, 4), dtype=torch.float32, device="cuda")
        bad_frames, nan_px, diff_px, first = 0, 0, 0, None
        for i in range(40):
            full.fill_(float("nan"))
            ctx.dispatch_rows(320, 180, 0, 1, 1, 180, full.data_ptr(), 320 * 16)
            ctx.sync()
            img = full.cpu().numpy()
            if not np.array_equal(img, ref):
                bad_frames += 1
                n = int(np.isnan(img).any(-1).sum())
                d = int(((img != ref) & ~np.isnan(img)).any(-1).sum())
                nan_px += n
                diff_px += d
                if first is None:
                    ys, xs = np.nonzero((img != ref).any(-1))
                    first = {"frame": i, "nan": n, "diff": d, "pixels": [[int(y), int(x)] for y, x in zip(ys[:6], xs[:6])]}
        out[sched] = {"bad_frames": bad_frames, "nan_px": nan_px, "diff_px": diff_px, "first": first}
    print(json.dumps({"lib": lib or "in-tree", "sched": out}), flush=True)
    ctx.close()
