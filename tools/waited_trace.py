#!/usr/bin/env python3
"""Waited car frames through the C++ host loop (librthost.so rth_render_loop), for a
kernel trace: the gap between one frame's kernel end and the next one's start is the
host's turn-around (poll, camera/light upload, launch) plus the launch latency.

    rocprofv3 --kernel-trace --output-format csv -d DIR -o run -- python3 tools/waited_trace.py
"""
import os
import sys

os.environ.setdefault("GPU_MAX_HW_QUEUES", "6")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "opengl-ray-tracer_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import rtamd  # noqa: E402

W, H = 1920, 1080
fs = rtamd.generate(3, 0, W, H)
torch.cuda.set_device(0)
c = rtamd.ComputeShader(0)
c.upload(fs)
c.set_params(W, H, 3)
c.set_kernel_timing(False)
c.set_latency_mode(1)
out = torch.empty((H, W, 4), dtype=torch.float32, device="cuda")
torch.cuda.synchronize()
rtamd.render_loop(c, fs.camera, fs.light, W, H, out.data_ptr(), W * 16, 50, True)
ms = rtamd.render_loop(c, fs.camera, fs.light, W, H, out.data_ptr(), W * 16, 200, True)
print("waited median %.4f ms, p10 %.4f, p90 %.4f" % (np.median(ms), np.percentile(ms, 10), np.percentile(ms, 90)))
c.close()
