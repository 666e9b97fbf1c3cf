#!/usr/bin/env python3
"""Waited-frame latency of the car (bench.py's serial_frame_ms_median setting) over the
latency mode's knobs, one process, one context, modes alternated in blocks.

    python tools/latency_sweep.py [--frames 300] [--blocks 3] [--config 3]

Each frame: camera + light upload, dispatch, wait (rt_sync: the host polls the
stream), rt_set_latency_mode(1), kernel timing events off. Settings: split walks
(rt_debug_split max_rays, group) and the heaviest tiles as several waves
(rt_debug_heavy k, parts). Every setting's frame is compared bit for bit with the
default's. One JSON line: median waited ms per setting (median over blocks).
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

SETTINGS = {
    "default": {},
    # round 4 sweep 1 (latency mode's heavy tiles then 1/512 x 2 waves): profiles/r04e_latency_sweep.json;
    # sweep 3 (raised wave priority for the first k slots, s_setprio): no effect, dropped
    # (profiles/r04r_latency_sweep_prio_negative.json). Sweep 4: the cost order by the
    # tiles' wave wall time (rt_debug_cost_time) instead of their lanes' steps + tests
    # sweep 5 (r04z7): cost frames record whole tiles, so the order no longer depends on
    # the split set it started from; split-set sizes again (profiles/r04z7_latency_sweep.json).
    # Sweep 6 (r04z8): around the new default, 1/256 x 4 (profiles/r04z8_latency_sweep.json).
    # Sweep 7 (r04z12): the heaviest slots' camera rays per lane under the wall-time order
    # (profiles/r04z12_latency_sweep_lanek.json: neutral). Sweep 8 (r04zz2): big frames (config
    # 4 at 3840x2160, config 5), latency mode against the default mode
    # (profiles/r04zz2_latency_sweep_*.json). Sweep 9 (r04zz8): split walks under the new order
    "split16x16": {"split": (16, 16)},
    "split32x8": {"split": (32, 8)},
    "split8x8": {"split": (8, 8)},
    "split16x32": {"split": (16, 32)},
    "split32x16": {"split": (32, 16)},
    "split4x8": {"split": (4, 8)},
    # Sweep 10 (r06): config 2's waited frame (the monkey scene, all-packet: primary + shadow),
    # whose slowest tiles are packet-step chains (profiles/r06h_tile_profile_latency_c2.txt)
    "heavy_off": {"heavy": (0, 1)},
    "heavy300x2": {"heavy": (300, 2)},
    "heavy150x4": {"heavy": (150, 4)},
    "heavy75x8": {"heavy": (75, 8)},
    "heavy40x16": {"heavy": (40, 16)},
    "lanek64x1": {"lane_k": (64, 1)},
    "lanek64x3": {"lane_k": (64, 3)},
    "lanek256x3": {"lane_k": (256, 3)},
    "lanek1024x3": {"lane_k": (1024, 3)},
    "latency0": {"latency": 0},
    "lanek32x3": {"lane_k": (32, 3)},
    "lanek128x3": {"lane_k": (128, 3)},
    "lanek64x3_h40x16": {"lane_k": (64, 3), "heavy": (40, 16)},
    "lanek64x3_h40x8": {"lane_k": (64, 3), "heavy": (40, 8)},
    "lanek128x3_h40x16": {"lane_k": (128, 3), "heavy": (40, 16)},
    "lanek64x3_h20x16": {"lane_k": (64, 3), "heavy": (20, 16)},
    "lanek64x3_h80x16": {"lane_k": (64, 3), "heavy": (80, 16)},
    "h20x16": {"heavy": (20, 16)},
    "h40x32": {"heavy": (40, 32)},
    "h20x32": {"heavy": (20, 32)},
    "h60x32": {"heavy": (60, 32)},
    "h80x32": {"heavy": (80, 32)},
    "h120x32": {"heavy": (120, 32)},
    "h20x64": {"heavy": (20, 64)},
    "h40x64": {"heavy": (40, 64)},
    "h80x64": {"heavy": (80, 64)},
    "h160x16": {"heavy": (160, 16)},
    # the car (config 3): whole-frame rule 162 x 2
    "h162x4": {"heavy": (162, 4)},
    "h162x8": {"heavy": (162, 8)},
    "h162x16": {"heavy": (162, 16)},
    "h162x32": {"heavy": (162, 32)},
    "h81x16": {"heavy": (81, 16)},
    "h81x32": {"heavy": (81, 32)},
    "h324x8": {"heavy": (324, 8)},
    "h324x16": {"heavy": (324, 16)},
    # Sweep 11 (r06): config 5's waited frame with ray compaction (rt_set_tail) off or from
    # another bounce (auto: on from bounce 2 for scenes of >= 8,192 scene-tree items)
    "tail_off": {"tail": 0},
    "tail1": {"tail": 1},
    "tail3": {"tail": 3},
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=300)
    ap.add_argument("--blocks", type=int, default=3)
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    cfg, W, H, mb, _, _ = bench.WORKLOADS[a.config]
    fs = rtamd.generate(cfg, 0, W, H)
    torch.cuda.set_device(0)
    c = rtamd.ComputeShader(0)
    c.upload(fs)
    c.set_params(W, H, mb)
    c.set_kernel_timing(False)
    c.set_latency_mode(1)
    out = torch.empty((H, W, 4), dtype=torch.float32, device="cuda")
    names = [n for n in SETTINGS if not a.only or n in a.only.split(",") or n == "default"]

    def apply(s):
        c.debug_split(*s.get("split", (16, 8)))
        c.debug_heavy(*s.get("heavy", (-1, 2)))
        c.debug_lane_k(*s.get("lane_k", (-1, 2)))
        c.debug_cost_time(s.get("cost_time", -1))
        c.set_latency_mode(s.get("latency", 1))
        c.set_tail(s.get("tail", -1))

    def frame():
        c.set_camera(fs.camera)
        c.set_light(fs.light)
        c.dispatch_rows(W, H, 0, 1, 1, H, out.data_ptr(), W * 16)
        c.sync()

    ref, res, same, pattern = None, {n: [] for n in names}, {}, {}
    for blk in range(a.blocks):
        for n in names:
            apply(SETTINGS[n])
            for _ in range(20):
                frame()
            w = []
            for _ in range(a.frames):
                t0 = time.perf_counter()
                frame()
                w.append(time.perf_counter() - t0)
            res[n].append(float(np.median(w)) * 1e3)
            wa = np.array(w) * 1e3
            slow = wa > 0.5 * (np.percentile(wa, 10) + np.percentile(wa, 90))
            pattern.setdefault(n, []).append({"slow_frac": float(slow.mean()),
                                              "slow_by_phase8": [int(slow[k::8].sum()) for k in range(8)],
                                              "p10": float(np.percentile(wa, 10)), "p90": float(np.percentile(wa, 90)),
                                              "first40": "".join("x" if v else "." for v in slow[:40])})
            img = out.cpu().numpy()
            if ref is None:
                ref = img
            same[n] = same.get(n, True) and bool(np.array_equal(img, ref))
    print(json.dumps({"config": a.config, "frames": a.frames, "blocks": a.blocks,
                      "waited_ms": {n: float(np.median(v)) for n, v in res.items()},
                      "per_block": res, "pattern": pattern, "image_equal": same}))
    c.close()


if __name__ == "__main__":
    main()
