#!/usr/bin/env python3
"""bench.py — frames/s and Mrays/s of the MI355X ray tracer (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 3] [--kernel auto]

A step is one frame of the reference's GPU render loop (src/main.cpp:325-370)
per GPU: per-frame camera + light upload (SSBO 2/1), the render dispatch and
its completion (one process per GPU, launched by torch.distributed.run).
Default workload: config 3, the car scene (4,022 triangles + 100 spheres,
reference BVH with the 2-triangle road), 1920x1080, maxBounces 3, barycentric,
no Fresnel.

Multi-GPU (--mode): frames are independent units, so by default (weak) every
rank renders its own 1920x1080 frame per step -- frame r of a camera orbit
around the car, 1 degree per frame, rank 0 = the config's camera -- with no
collective on the data path: the per-GPU work is fixed as N grows, scaling
"weak". --mode strong instead splits ONE frame per step across the ranks
(interleaved 8-row stripes) and gathers it to rank 0 over RCCL: total work
fixed, scaling "strong" (the frame then ends with its slowest pixel paths,
DESIGN.md §7).

Frames in flight (--inflight F, default auto: 2 at 1920x1080, up to 4 for frames
too small to fill the GPU, e.g. 800x600): frame n of a rank renders on
context n % F, each with its own HIP stream and output surface (double
buffering), so one frame's tail -- its slowest tiles, when most of the GPU is
idle -- overlaps the next frame's start. Every step still renders one whole
frame; ms_per_step is the sustained time per frame. The same K frames are also
timed with one frame in flight (serial_ms_per_step, the single-frame latency
regime), and kernel_ms_mean / kernel_ms_median are the device durations of the
individual dispatches in that one-frame pass (the kernel alone on the GPU: the
roofline's denominator; rocprof's kernel-trace average of `bench.py --inflight 1`
is the matching profile); kernel_ms_mean_inflight is the same events' mean with
frames in flight, where a dispatch's span includes waiting for the other frame.

value = Mrays/s = (closest-hit + shadow rays of the frame, counted on the
reference walk by the counting kernel) x frames / s, summed over the job.
Rank 0 prints one JSON line with the roofline of the render kernel and the CPU
baseline (the oracle, OpenMP on host cores, on a bounded row sample).
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "opengl-ray-tracer_amd"))
import rtamd  # noqa: E402
import tiling  # noqa: E402

METRIC = "Mrays/sec + FPS @1920x1080, car scene (4122 shapes), 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)

# config -> (scene generator config, width, height, maxBounces, description)
WORKLOADS = {
    2: (2, 800, 600, 1, "monkey stand-in (1,240 shapes), 800x600, primary + shadow"),
    3: (3, 1920, 1080, 3, "car stand-in (4,022 triangles + 100 spheres), 1920x1080, reflection depth 3"),
    4: (3, 3840, 2160, 3, "car stand-in, 3840x2160"),
    5: (5, 1920, 1080, 3, "100k random triangles, deep BVH, 1920x1080"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", type=int, default=3, choices=sorted(WORKLOADS))
    ap.add_argument("--variant", type=int, default=0, help="car road: 0 = 2-triangle quad, 1 = 222 strips")
    ap.add_argument("--kernel", default="auto", choices=["auto", "lane", "packet", "accel"])
    ap.add_argument("--stripe", type=int, default=8)
    ap.add_argument("--inflight", type=int, default=0,
                    help="frames in flight per GPU (own context, stream, surface); 0 = auto: 2, or up to 4 "
                         "while a frame has fewer than 16k 8x8 tiles (too few waves to fill the GPU)")
    ap.add_argument("--mode", default="weak", choices=["weak", "strong"],
                    help="N > 1: weak = one frame per GPU (orbit), strong = one frame split over the GPUs + gather")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample time")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = min(16, cores)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo: rehearse the N>1 path with every rank on one GPU")
    return ap.parse_args()


def cpu_baseline(fs, W, H, mb, seconds, threads):
    """The oracle (oracle/rt_oracle.c, the GLSL restated, OpenMP) on a band of
    rows through the middle of the same frame; the band grows until the
    measurement takes roughly `seconds`."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # noqa: E402  (cpu_baseline leg only)
    p = oracle.params(W, H, mb)
    rows = 8
    while True:
        y0 = max(0, H // 2 - rows // 2)
        t0 = time.perf_counter()
        _, st = oracle.render(fs, W, H, p, y0=y0, out_rows=rows, stats=True, threads=threads)
        dt = time.perf_counter() - t0
        if dt >= seconds * 0.5 or rows >= H:
            break
        rows = min(H, max(rows * 2, int(rows * seconds / max(dt, 1e-3) * 0.9)))
    rays = st["closest_rays"] + st["shadow_rays"]
    return {"value": rays / dt / 1e6, "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": f"oracle (GLSL restated, OpenMP) rows [{y0},{y0 + rows}) of the same {W}x{H} frame: "
                      f"{rows * W} pixels, {rays} rays in {dt:.2f} s",
            "ms_per_frame_equiv": dt * 1e3 * H / rows,
            "cpu": platform.processor() or platform.machine()}


def cpu_reference_1core(seconds):
    """BASELINE.md "CPU-ref": the reference's own CPU path, cpuRayTracer
    (src/main.cpp:848-894: brute force over every shape, primary rays only, CPU
    phong) restated in oracle/rt_oracle.c, on ONE core as the reference runs it.
    Config 1 (800x600, 4 spheres + 1 plane) whole frames, and the car scene's
    1920x1080 primary rays on a band of rows (the whole frame would take minutes)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # noqa: E402  (cpu_baseline leg only)
    fs1 = rtamd.generate(1, 0, 800, 600)
    oracle.cpu_raytracer(fs1, 800, 600, threads=1)  # warm-up
    n1, t0 = 0, time.perf_counter()
    while n1 < 3 or time.perf_counter() - t0 < 1.0:
        oracle.cpu_raytracer(fs1, 800, 600, threads=1)
        n1 += 1
    ms1 = (time.perf_counter() - t0) / n1 * 1e3
    fs3 = rtamd.generate(3, 0, 1920, 1080)
    rows, y0 = 2, 539
    while True:
        t0 = time.perf_counter()
        oracle.cpu_raytracer(fs3, 1920, 1080, y0=y0, y1=y0 + rows, threads=1)
        dt = time.perf_counter() - t0
        if dt >= seconds * 0.5 or rows >= 64:
            break
        rows = min(64, max(rows * 2, int(rows * seconds / max(dt, 1e-3) * 0.9)))
    return {"kind": "port", "path": "cpuRayTracer (src/main.cpp:848-894)", "cores": 1,
            "config1_ms_per_frame": ms1, "config1_mrays_primary_per_s": 800 * 600 / ms1 / 1e3,
            "config3_primary_only_mrays_per_s": rows * 1920 / dt / 1e6,
            "config3_primary_only_ms_per_frame_equiv": dt * 1e3 * 1080 / rows,
            "sample": f"cpuRayTracer restated (oracle/rt_oracle.c orc_cpu_raytracer), 1 thread: config 1 {n1} "
                      f"whole 800x600 frames; config 3 rows [{y0},{y0 + rows}) of 1920x1080 in {dt:.2f} s"}


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and a.backend == "gloo":
        torch.cuda.set_device(0)
        dist.init_process_group("gloo")
    elif world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    # One non-default stream shared by torch (RCCL waits on it) and the renderer.
    torch.cuda.set_stream(torch.cuda.Stream())

    cfg, W, H, mb, desc = WORKLOADS[a.config]
    sc = rtamd.Scene().generate(cfg, a.variant, W / H)
    sc_stats = sc.bvh_stats()
    strong = a.mode == "strong" and world > 1
    if not strong and rank > 0:
        # frame `rank` of the orbit: the camera turned about the vertical axis through
        # the look-at point (the origin) by `rank` degrees
        cam0 = sc.serializeScene().camera
        p = cam0["Position"][0].astype(np.float64)
        ang = np.radians(float(rank))
        pos = (p[0] * np.cos(ang) + p[2] * np.sin(ang), p[1], -p[0] * np.sin(ang) + p[2] * np.cos(ang))
        sc.set_camera(pos, float(cam0["fov"][0]), float(cam0["aspectRatio"][0]))
        sc.LookAt((0.0, 0.0, 0.0))
    fs = sc.serializeScene()

    # strong mode gathers one shared buffer per step: one frame in flight there
    tiles = ((W + 7) // 8) * ((H + 7) // 8)
    F = 1 if strong else (a.inflight if a.inflight > 0 else min(4, max(2, -(-16384 // tiles) + 1)))
    main_stream = torch.cuda.current_stream()
    streams = [main_stream] + [torch.cuda.Stream() for _ in range(F - 1)]
    ctxs = []
    for s_ in streams:
        c_ = rtamd.ComputeShader(torch.cuda.current_device())
        c_.set_stream(s_.cuda_stream)
        c_.upload(fs)
        c_.set_params(W, H, mb, True, False, False)
        c_.set_kernel({"auto": 0, "lane": 1, "packet": 2, "accel": 3}[a.kernel])
        ctxs.append(c_)
    ctx = ctxs[0]

    # strong: this rank's interleaved stripes of the one frame; weak: the rank's whole frame
    plan = tiling.StripePlan(H, world if strong else 1, a.stripe)
    prank = rank if strong else 0
    rows = plan.rows(prank)
    bufs = [torch.empty((plan.rows_max, W, 4), dtype=torch.float32, device=dev) for _ in range(F)]

    # Work of this rank's rows on the reference walk (counting kernel, untimed).
    st = ctx.collect_stats(W, H, plan.y0(prank), a.stripe, plan.world, rows)
    mine = torch.tensor([st["closest_rays"], st["shadow_rays"], rtamd.algorithmic_bytes(st, rows * W), st["hits"]],
                        dtype=torch.float64, device=dev)
    total = mine.clone()
    if world > 1:
        total = total.cpu() if a.backend == "gloo" else total
        dist.all_reduce(total)
    rays_step = float(total[0] + total[1])  # all ranks' rays of one step
    b_alg_rank = float(mine[2])

    cam, light = fs.camera, fs.light

    def frame(i, inflight):
        c_ = ctxs[i % inflight]
        c_.set_camera(cam)   # SSBO 2 (src/main.cpp:328-330)
        c_.set_light(light)  # SSBO 1 (:332-334)
        buf = bufs[i % inflight]
        c_.dispatch_rows(W, H, plan.y0(prank), a.stripe, plan.world, rows, buf.data_ptr(), W * 16)
        if strong:
            tiling.gather_to_root(buf, plan)

    def timed(inflight):
        """Wall time of a.steps frames between barriers, max over ranks."""
        for i in range(a.warmup * inflight):
            frame(i, inflight)
        torch.cuda.synchronize()
        for c_ in ctxs:
            c_.kernel_times()  # drop warm-up dispatches
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(a.steps):
            frame(i, inflight)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64,
                          device="cpu" if a.backend == "gloo" else dev)
        if world > 1:
            dist.all_reduce(el, op=dist.ReduceOp.MAX)
        return float(el[0])

    serial = timed(1) if F > 1 else None
    serial_kt = ctx.kernel_times() if F > 1 else None
    elapsed = timed(F)

    kt_if = np.concatenate([c_.kernel_times() for c_ in ctxs]) if F > 1 else ctx.kernel_times()
    # The render kernel's duration is taken where it runs alone (the one-frame-in-flight
    # pass): with frames in flight a dispatch's events also span the time it waits for
    # the other frame's waves to leave the CUs.
    kt = serial_kt if F > 1 else kt_if
    info = ctx.accel_info()
    kname = {1: "k_lane", 2: "k_packet", 3: "k_accel"}.get(info["last_kernel"], "?")
    k_ms = float(np.mean(kt)) if len(kt) else float("nan")
    k_med = float(np.median(kt)) if len(kt) else float("nan")

    if rank == 0:
        frames = a.steps * (1 if strong or world == 1 else world)
        fps = frames / elapsed
        achieved = b_alg_rank / (k_ms * 1e-3) / 1e9
        traffic = None
        pmc_path = os.path.join(ROOT, "profiles", "pmc_summary.json")
        if os.path.exists(pmc_path):
            with open(pmc_path) as f:
                traffic = json.load(f).get(f"config{a.config}_n{world}_{a.kernel}")
        out = {
            "metric": METRIC,
            "value": rays_step * a.steps / elapsed / 1e6,
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": elapsed / a.steps * 1e3,
            "frames_in_flight": F,
            "serial_ms_per_step": (serial if serial is not None else elapsed) / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (procedural stand-in meshes, fixed seed; the reference's .obj assets are absent)",
            "backend": a.backend if world > 1 else None,
            "config": {"workload": f"config {a.config}: {desc}" + (" (222-strip road)" if a.variant else ""),
                       "width": W, "height": H, "maxBounces": mb, "useBVH": 1, "useFresnel": 0,
                       "triangle_test": "barycentric", "shapes": len(fs.shapes), "bvh_nodes": len(fs.nodes),
                       "bvh_max_leaf": sc_stats["max_leaf"], "kernel": a.kernel,
                       "parallelism": (f"row-stripes{a.stripe}x{world}+rccl-gather" if strong else
                                       f"frame-sharded x{world} (one frame per GPU per step, orbit 1 deg/rank)")},
            "fps": fps,
            "mrays_primary_per_s": W * H * fps / 1e6,
            "rays_per_step": rays_step,
            "kernel_ms_mean": k_ms,
            "kernel_ms_median": k_med,
            "kernel_ms_mean_inflight": float(np.mean(kt_if)) if len(kt_if) else float("nan"),
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                # the same bytes over the sustained frame time (frames overlap when F > 1)
                "aggregate_achieved": b_alg_rank * a.steps / elapsed / 1e9,
                "traffic": traffic,
                "algorithmic_bytes_per_launch": b_alg_rank,
                "kernel": kname,
            },
            "accel": info,
            "cpu_baseline": None,
        }
        if world == 1 and not a.no_cpu:
            thr = a.cpu_threads or min(16, os.cpu_count() or 1)
            out["cpu_baseline"] = cpu_baseline(fs, W, H, mb, a.cpu_seconds, thr)
            out["cpu_baseline"]["reference_cpu_path"] = cpu_reference_1core(a.cpu_seconds / 2)
        print(json.dumps(out), flush=True)
    for c_ in ctxs:
        c_.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
