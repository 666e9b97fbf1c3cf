#!/usr/bin/env python3
"""Does the latency-mode car frame settle into different states? (diagnostics; GPU box)

    python tools/waited_modes.py [--trials 4] [--blocks 12] [--per 32]

Each trial makes fresh contexts and runs bench.py's sequence: F = 3 contexts with
frames in flight (300 frames, latency mode off), then context 0 alone in latency
mode, waited frames (camera + light upload, dispatch, rt_sync) in blocks. Per
block: the median waited ms and the head of context 0's cost order (its first
63 tiles: the split set), so a slow and a fast state can be told apart by their
orders. One JSON line.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "opengl-ray-tracer_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import bench  # noqa: E402
import rtamd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=4)
    ap.add_argument("--blocks", type=int, default=12)
    ap.add_argument("--per", type=int, default=32)
    ap.add_argument("--head", type=int, default=63)
    a = ap.parse_args()
    cfg, W, H, mb, _, _ = bench.WORKLOADS[3]
    fs = rtamd.generate(cfg, 0, W, H)
    torch.cuda.set_device(0)
    trials = []
    for _ in range(a.trials):
        ctxs, bufs = [], []
        for _ in range(3):
            s = torch.cuda.Stream()
            c = rtamd.ComputeShader(0)
            c.set_stream(s.cuda_stream)
            c.upload(fs)
            c.set_params(W, H, mb)
            c.set_kernel_timing(False)
            ctxs.append((c, s))
            bufs.append(torch.empty((H, W, 4), dtype=torch.float32, device="cuda"))
        for i in range(300):
            c, _ = ctxs[i % 3]
            c.set_camera(fs.camera)
            c.set_light(fs.light)
            c.dispatch_rows(W, H, 0, 1, 1, H, bufs[i % 3].data_ptr(), W * 16)
        torch.cuda.synchronize()
        c = ctxs[0][0]
        c.set_latency_mode(1)
        blocks, heads = [], []
        for b in range(a.blocks):
            w = []
            for _ in range(a.per):
                t0 = time.perf_counter()
                c.set_camera(fs.camera)
                c.set_light(fs.light)
                c.dispatch_rows(W, H, 0, 1, 1, H, bufs[0].data_ptr(), W * 16)
                c.sync()
                w.append(time.perf_counter() - t0)
            blocks.append(round(float(np.median(w)) * 1e3, 4))
            heads.append(sorted(int(x) for x in c.debug_sched_order(a.head)))
        # head changes between blocks (tiles entering / leaving the split set)
        churn = [len(set(heads[k]) ^ set(heads[k - 1])) for k in range(1, len(heads))]
        trials.append({"block_ms": blocks, "head_churn": churn, "heads": heads})
        for c_, _ in ctxs:
            c_.close()
    # tiles in the head of slow blocks but not fast ones
    allb = [(t["block_ms"][k], tuple(t["heads"][k])) for t in trials for k in range(len(t["block_ms"]))]
    ms = np.array([x[0] for x in allb])
    thr = 0.5 * (ms.min() + ms.max())
    slow = [set(h) for m, h in allb if m > thr]
    fast = [set(h) for m, h in allb if m <= thr]
    common_slow = set.intersection(*slow) if slow else set()
    common_fast = set.intersection(*fast) if fast else set()
    print(json.dumps({"trials": [{k: v for k, v in t.items() if k != "heads"} for t in trials],
                      "threshold_ms": float(thr), "n_slow_blocks": len(slow), "n_fast_blocks": len(fast),
                      "only_in_slow_heads": sorted(common_slow - common_fast),
                      "only_in_fast_heads": sorted(common_fast - common_slow)}))


if __name__ == "__main__":
    main()
