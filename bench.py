#!/usr/bin/env python3
"""bench.py — frames/s and Mrays/s of the MI355X ray tracer (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 3] [--mode auto|frames|strong|weak]

A step is one frame of the reference's GPU render loop (src/main.cpp:325-370):
the per-frame camera + light upload (SSBO 2/1), the render dispatch and its
completion. Default workload: config 3, the car scene (4,022 triangles + 100
spheres, reference BVH with the 2-triangle road), 1920x1080, maxBounces 3,
barycentric, no Fresnel.

--gpus N: one process per GPU. Without torch.distributed.run's environment and
N > 1, bench.py starts `python -m torch.distributed.run --nproc-per-node N` as a
CHILD process (before touching the GPU) and exits with its return code; under
torchrun it checks that WORLD_SIZE == N.

Modes (--mode auto = frames at N = 1, strong at N > 1):
  frames  one GPU renders whole frames (frames in flight: --inflight, auto 3 at
          1080p, 2 at 4K, up to 4 for frames too small to fill the GPU);
  strong  the north star's multi-GPU frame: every step renders ONE
          1920x1080 frame split over the N GPUs by interleaved 8-row stripes and
          gathers it to rank 0 through the C ABI's rt_group (ncclSend/ncclRecv
          over xGMI, then k_unstripe into rank 0's image) — total work fixed,
          scaling "strong". Frames in flight = the group's frame slots
          (rt_group_set_frames): one render stream and buffer set per slot,
          ONE communicator and one fan-in stream per rank. Before timing,
          one gathered frame is compared bit for bit with rank 0's own
          single-GPU frame (exit 5 on a mismatch); every wait on the group
          is bounded (rt_group_sync: exit 4 on a timeout or an RCCL error);
          the JSON line carries each rank's render / fan-in / unstripe times.
          Rank 0 may take 2 stripes per period (--root-share; auto times 1
          and 2 before the measured steps): its rows never cross a link;
  weak    each rank renders its own whole frame per step (frame r of a 1-degree
          camera orbit about the config's look-at point), no collective.

value = Mrays/s = (closest-hit + shadow rays of the frame, counted on the
reference walk by the counting kernel) x frames / s, summed over the job.
Rank 0 prints one JSON line with the render kernel's roofline and the CPU
baseline (N = 1 only: the oracle, OpenMP on the host's cores, on a bounded row
sample of the same frame; plus the reference's 1-core cpuRayTracer).

roofline: the render kernel is bound by dependent-fetch latency, not by HBM
(DESIGN.md §5). `achieved` = HBM bytes per launch measured by rocprofv3
(FETCH_SIZE x2 + WRITE_SIZE, profiles/pmc_summary.json, the same command) /
the kernel's mean device time in THIS run (HIP events on the renderer's
stream, one frame in flight); `frac` = achieved / 8 TB/s. Without a PMC entry
for the workload it falls back to the compulsory bytes (image + the kernel's
device records once). The reference-walk bytes of SURVEY §8(d) are reported
as `reference_equivalent_GBps` (work the accelerator skips; not a bandwidth).
"""
from __future__ import annotations

import argparse
import contextlib
import ctypes
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
METRIC = "Mrays/sec + FPS @1920x1080, car scene (4122 shapes), 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md)

# config -> (scene generator config, width, height, maxBounces, description, camera look-at target)
# The targets are the generators' LookAt points (csrc/scene.cpp: gen_monkey :472, gen_car :549,
# gen_random :570), about which the weak mode's camera orbit turns.
SCHEDULES = {"rows": 0, "cost": 1, "xcd": 2}  # rtamd.SCHED_ROWS / SCHED_COST / SCHED_COST_XCD
WORKLOADS = {
    2: (2, 800, 600, 1, "monkey stand-in (1,240 shapes), 800x600, primary + shadow", (0.0, 10.0, -8.0)),
    3: (3, 1920, 1080, 3, "car stand-in (4,022 triangles + 100 spheres), 1920x1080, reflection depth 3",
        (0.0, 0.0, 0.0)),
    4: (3, 3840, 2160, 3, "car stand-in, 3840x2160", (0.0, 0.0, 0.0)),
    5: (5, 1920, 1080, 3, "100k random triangles, deep BVH, 1920x1080", (0.0, 0.0, 0.0)),
}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", type=int, default=3, choices=sorted(WORKLOADS))
    ap.add_argument("--variant", type=int, default=0, help="car road: 0 = 2-triangle quad, 1 = 222 strips")
    ap.add_argument("--kernel", default="auto", choices=["auto", "lane", "packet", "accel"])
    ap.add_argument("--stripe", type=int, default=8)
    ap.add_argument("--brute", action="store_true", help="useBVH = 0: the brute-force branch (gpu_shader.comp:523-620)")
    ap.add_argument("--mt", action="store_true", help="useMollerTrumbore = 1 (gpu_shader.comp:170-195)")
    ap.add_argument("--fresnel", action="store_true", help="useFresnel = 1 (gpu_shader.comp:500-509)")
    ap.add_argument("--animate", action="store_true",
                    help="the reference's animations, refit on the device (rt_animate) inside the timed step: "
                         "config 2 = scene 1's three bouncing spheres (bounceSphere, src/main.cpp:438-445); "
                         "configs 3/4 = the car's four wheels turning (updateWheelAnimations, :1084-1109)")
    ap.add_argument("--upload", default="device", choices=["device", "reference"],
                    help="--animate's per-frame upload: device = rt_animate (the records, updateBVH on the device); "
                         "reference = the reference's own calls (src/main.cpp:336-346): one rt_update_shapes per "
                         "animated record, updateBVH on the host (rts_update_bvh), one rt_update_nodes "
                         "(librthost.so rth_upload_animated), applied by the renderer as a device refit")
    ap.add_argument("--camera-path", default="static", choices=["static", "orbit", "dolly"],
                    help="the camera per frame: static (the config's camera); orbit = 0.5 deg per frame about "
                         "the look-at point (Camera::LookAt after each step); dolly = Camera::ProcessKeyboard "
                         "FORWARD at the reference's SPEED (15 units/s, 1/60 s per frame), 96 frames in, 96 back "
                         "(src/camera.hpp:75-90, src/main.cpp:509-534)")
    ap.add_argument("--inflight", type=int, default=0,
                    help="frames in flight per GPU; 0 = auto: 3 below 64k 8x8 tiles (1080p), 2 above (4K), up "
                         "to 4 while the GPU's share of a frame has fewer than 16k tiles; strong mode over "
                         "rt_group: at least that, up to 8 for a rank's small share")
    ap.add_argument("--mode", default="auto", choices=["auto", "frames", "strong", "weak"])
    ap.add_argument("--gather", default="auto", choices=["auto", "rt", "torch"],
                    help="strong mode's fan-in: rt = rt_group (RCCL send/recv, C ABI); torch = "
                         "torch.distributed.gather (gloo rehearsals); auto = rt on nccl, torch on gloo")
    ap.add_argument("--root-share", default="auto",
                    help="strong mode over rt_group: rank 0's stripes per period of share + N - 1 "
                         "(rt_group_set_root_share; rank 0's rows never cross a link); auto = the faster of "
                         "1 and 2, timed on every rank before the measured steps")
    ap.add_argument("--schedule", default="cost", choices=["cost", "xcd", "rows"],
                    help="tile dispatch order (rt_set_schedule): cost (default), cost dealt to XCDs as bands, rows")
    ap.add_argument("--refit", type=int, default=-1,
                    help="diagnostics: rt_debug_refit launch shape of the refit (-1: the library's choice)")
    ap.add_argument("--walk", type=int, default=-1,
                    help="walk policy (rt_set_walk): -1 auto, 0 all per lane, >= maxBounces all packets")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample time")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = the host's cores (nproc)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo: rehearse the N>1 path with every rank on one GPU")
    return ap.parse_args(argv)


@contextlib.contextmanager
def quiet_stdout():
    """Route the C-level stdout to stderr while RCCL initialises: it prints a
    version banner there, and rank 0's stdout must hold only the JSON line."""
    libc = ctypes.CDLL(None)
    sys.stdout.flush()
    libc.fflush(None)
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        yield
    finally:
        libc.fflush(None)
        os.dup2(saved, 1)
        os.close(saved)


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(a):
    """--gpus N > 1 outside torchrun: run torchrun as a child and return its exit code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def host_cores():
    """What `nproc` reports: OMP_NUM_THREADS if set, else the CPUs this process may run on."""
    omp = os.environ.get("OMP_NUM_THREADS", "")
    return int(omp) if omp.isdigit() and int(omp) > 0 else len(os.sched_getaffinity(0))


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(rtamd, fs, W, H, mb, seconds, threads, toggles=(True, False, False)):
    """The oracle (oracle/rt_oracle.c, the GLSL restated, OpenMP) on a band of
    rows through the middle of the same frame; the band grows until the
    measurement takes roughly `seconds`."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # noqa: E402  (cpu_baseline leg only)
    p = oracle.params(W, H, mb, *toggles)
    rows = 8
    while True:
        y0 = max(0, H // 2 - rows // 2)
        t0 = time.perf_counter()
        img, st = oracle.render(fs, W, H, p, y0=y0, out_rows=rows, stats=True, threads=threads)
        dt = time.perf_counter() - t0
        if dt >= seconds * 0.5 or rows >= H:
            break
        rows = min(H, max(rows * 2, int(rows * seconds / max(dt, 1e-3) * 0.9)))
    rays = st["closest_rays"] + st["shadow_rays"]
    cpu_baseline.last_image = (y0, img)  # the timed frames are checked against these rows
    return {"value": rays / dt / 1e6, "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": f"oracle (GLSL restated, OpenMP, {threads} threads) rows [{y0},{y0 + rows}) of the same "
                      f"{W}x{H} frame: {rows * W} pixels, {rays} rays in {dt:.2f} s",
            "ms_per_frame_equiv": dt * 1e3 * H / rows,
            "cpu": cpu_model(), "cpus_visible": os.cpu_count(), "cpus_affinity": len(os.sched_getaffinity(0))}


PARITY_TOL = 1e-4  # per channel (BASELINE.json north_star)


def parity_check(frames, ref_y0, ref, what):
    """The frames the timed loop left in its buffers (one per context in flight: each
    holds that context's last timed frame) against the oracle's rows [ref_y0, ref_y0 +
    len(ref)) of the same frame (gpu_shader.comp:433-624 restated, oracle/rt_oracle.c)."""
    import numpy as np
    worst, bad = 0.0, 0
    for f in frames:
        img = f[ref_y0:ref_y0 + len(ref)].astype(np.float64)
        d = np.abs(img - ref.astype(np.float64))
        d[np.isnan(img) & np.isnan(ref)] = 0.0
        d[np.isnan(d)] = np.inf
        worst = max(worst, float(d.max()) if d.size else 0.0)
        bad += int((d > PARITY_TOL).any(axis=-1).sum())
    return {"max_abs": worst, "bad_pixels": bad, "frames_checked": len(frames), "tol": PARITY_TOL,
            "rows_checked": [int(ref_y0), int(ref_y0 + len(ref))], "against": what, "ok": bad == 0}


def cpu_reference_1core(rtamd, seconds, cfg=3, variant=0, W=1920, H=1080):
    """BASELINE.md "CPU-ref": the reference's own CPU path, cpuRayTracer
    (src/main.cpp:848-894: brute force over every shape, primary rays only, CPU
    phong) restated in oracle/rt_oracle.c, on ONE core as the reference runs it.
    Config 1 (800x600, 4 spheres + 1 plane) whole frames, and the run's own scene
    (generator config `cfg`) at W x H, primary rays only, on a band of rows through
    the middle (a whole frame would take minutes)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # noqa: E402  (cpu_baseline leg only)
    fs1 = rtamd.generate(1, 0, 800, 600)
    oracle.cpu_raytracer(fs1, 800, 600, threads=1)  # warm-up
    n1, t0 = 0, time.perf_counter()
    while n1 < 3 or time.perf_counter() - t0 < 1.0:
        oracle.cpu_raytracer(fs1, 800, 600, threads=1)
        n1 += 1
    ms1 = (time.perf_counter() - t0) / n1 * 1e3
    fs3 = rtamd.generate(cfg, variant, W, H)
    rows, y0 = 2, H // 2 - 1
    while True:
        t0 = time.perf_counter()
        oracle.cpu_raytracer(fs3, W, H, y0=y0, y1=y0 + rows, threads=1)
        dt = time.perf_counter() - t0
        if dt >= seconds * 0.5 or rows >= 64:
            break
        rows = min(64, max(rows * 2, int(rows * seconds / max(dt, 1e-3) * 0.9)))
    return {"kind": "port", "path": "cpuRayTracer (src/main.cpp:848-894)", "cores": 1, "cpu": cpu_model(),
            "config1_ms_per_frame": ms1, "config1_mrays_primary_per_s": 800 * 600 / ms1 / 1e3,
            "this_config_primary_only_mrays_per_s": rows * W / dt / 1e6,
            "this_config_primary_only_ms_per_frame_equiv": dt * 1e3 * H / rows,
            "sample": f"cpuRayTracer restated (oracle/rt_oracle.c orc_cpu_raytracer), 1 thread: config 1 {n1} "
                      f"whole 800x600 frames; this run's scene rows [{y0},{y0 + rows}) of {W}x{H} in {dt:.2f} s"}


def wheel_frames(fs, n):
    """Records of the car's 640 wheel triangles for n frames: each wheel turns
    1 rad/s x 1/60 s per frame about its axle (z through its centre), as
    updateWheelAnimations does with deltaTime (src/main.cpp:1084-1109); stored
    normals are left as they were (the reference does not update them)."""
    import numpy as np
    ids = np.arange(3380, 3380 + 640, dtype=np.int32)  # gen_car: body (3,380), 4 wheels x 160, road
    rec = fs.shapes[ids].copy()
    cen = [np.concatenate([rec[f][160 * w:160 * (w + 1)] for f in ("triP1", "triP2", "triP3")]).astype(np.float64)
           .mean(0) for w in range(4)]
    frames = []
    for _ in range(n):
        rec = rec.copy()
        for w in range(4):
            sl = slice(160 * w, 160 * (w + 1))
            for f in ("triP1", "triP2", "triP3"):
                q = rec[f][sl].astype(np.float64) - cen[w]
                c, s = np.cos(1.0 / 60), np.sin(1.0 / 60)
                rec[f][sl] = (np.stack([q[:, 0] * c - q[:, 1] * s, q[:, 0] * s + q[:, 1] * c, q[:, 2]], 1)
                              + cen[w]).astype(np.float32)
        frames.append(rec)
    return ids, frames


# bounceSphere(sphere, currentFrame, amplitude, frequency) on scene 1's first three
# spheres (src/main.cpp:438-445; animatedIndices, :600-616)
BOUNCES = ((10.0, 1.0), (7.0, 0.8), (15.0, 1.5))


def sphere_frames(fs, n):
    """Records of scene 1's three bouncing spheres for n frames 1/60 s apart:
    centre.y = origin.y + amplitude * sin(frequency * t) in float32, as bounceSphere
    sets it (src/main.cpp:1079-1082); the generator's shapes 0-2 are those spheres
    (csrc/scene.cpp scene1_spheres). n = 512 frames spans 8.5 s, a full period of
    the slowest bounce (2 pi / 0.8 s)."""
    import numpy as np
    ids = np.arange(3, dtype=np.int32)
    base = fs.shapes[ids].copy()
    if not (base["type"] == 0).all():
        raise SystemExit("--animate on config 2: shapes 0-2 must be scene 1's spheres")
    frames = []
    for f in range(n):
        t = np.float32(f / 60.0)
        rec = base.copy()
        for k, (amp, fr) in enumerate(BOUNCES):
            rec["sphereCenter"][k][1] = base["sphereCenter"][k][1] + np.float32(amp) * np.sin(np.float32(fr) * t)
        frames.append(rec)
    return ids, frames


def camera_path(rtamd, sc, fs, kind, target):
    """The per-frame cameras of --camera-path (FlatCamera records, dealt as cams[i % n])."""
    import numpy as np
    if kind == "static":
        return np.ascontiguousarray(fs.camera).reshape(1)
    cams = []
    if kind == "orbit":  # 720 frames, 0.5 degrees each: one full turn
        for _ in range(720):
            sc.orbit(target, 0.5)
            cams.append(sc.camera().copy())
        sc.orbit(target, -360.0)
    else:  # Camera::ProcessKeyboard(FORWARD / BACKWARD, 1/60): Position +-= Front * (SPEED * dt), in float
        c = np.ascontiguousarray(fs.camera).reshape(1).copy()
        v = np.float32(15.0) * np.float32(1.0 / 60.0)
        for k in range(192):
            cams.append(c.copy())
            step = c["Front"][0] * v
            c["Position"][0] = c["Position"][0] + step if k < 96 else c["Position"][0] - step
    return np.ascontiguousarray(np.concatenate(cams)).astype(rtamd.CAMERA_DTYPE)


def animated_oracle_scene(fs, ids, frames, applied):
    """The scene one renderer holds after rt_animate was given frames[j] for every j in
    `applied` (in that order): the last frame's records, and the node boxes updateBVH
    grew to hold every frame's records (grow-only, src/main.cpp:1068-1077; restated
    by oracle.update_bvh). Growing is a union, so each distinct frame is applied once."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # noqa: E402  (checker only)
    import rtamd  # noqa: E402
    fk = rtamd.FlatScene(fs.shapes.copy(), fs.nodes.copy(), fs.indices, fs.camera, fs.light)
    for j in sorted(set(applied)):
        fk.shapes[ids] = frames[j]
        oracle.update_bvh(fk, ids)
    fk.shapes[ids] = frames[applied[-1]]
    return fk


def pmc_entry(key):
    path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        return json.load(f).get(key)


def roofline(info, kname, k_ms, pixels, b_ref, pmc, share=None):
    """The render kernel against its rooflines (see the module docstring).

    HBM: achieved = DRAM bytes per launch (PMC) / this run's kernel time; frac vs 8 TB/s.
    Issue: from the SQ passes of the same solo command (tools/sq_summary.py), the
    VALU and SALU instruction counts against the CU's issue rates give a floor per
    launch; issue.frac = that floor / this run's kernel time. `bound` names what
    binds: "hbm" if the HBM fraction is the larger, else "latency" -- neither pipe
    is saturated, and waves wait on dependent fetches (issue.wait_frac).

    share (strong lines): this rank renders that fraction of the frame's rows with
    the same kernel, and `pmc` is the workload's single-GPU entry. Its DRAM bytes
    are not this launch's (traffic null; achieved from the compulsory bytes), and
    its issue floors are scaled by the share: interleaved 8-row stripes give each
    rank the same mix of sky and car rows (tools/pmc_summary.py has no per-rank
    entry; PMC passes need a process of their own per GPU)."""
    compulsory = 16.0 * pixels + float(info.get("record_bytes", 0))
    k_s = k_ms * 1e-3
    measured = pmc.get("bytes") if pmc and share is None else None
    achieved = (measured if measured else compulsory) / k_s / 1e9
    frac = achieved / HBM_PEAK_GBS
    out = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": frac,
           "basis": ("measured DRAM bytes per launch (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, "
                     f"{pmc['source']}) / this run's mean kernel time") if measured else
                    "compulsory bytes per launch (16 B/pixel image store + the kernel's device records once) "
                    "/ this run's mean kernel time (no PMC entry for this workload)",
           "traffic": measured,
           "algorithmic_bytes_per_launch": compulsory,
           "algorithmic_GBps": compulsory / k_s / 1e9,
           "traffic_over_algorithmic": (measured / compulsory) if measured else None,
           "reference_equivalent_bytes_per_launch": b_ref,
           "reference_equivalent_GBps": b_ref / k_s / 1e9,
           "kernel": kname, "kernel_ms": k_ms}
    iss = pmc.get("issue") if pmc else None
    if iss and share is not None and iss.get("valu_floor_ms") is not None:
        iss = dict(iss, valu_floor_ms=iss["valu_floor_ms"] * share, salu_floor_ms=iss["salu_floor_ms"] * share,
                   row_share=share,
                   basis=f"single-GPU PMC of the same kernel ({pmc['source']}), issue floors x this rank's "
                         f"row share {share:.4f}")
    if iss:
        out["issue"] = dict(iss)
        if iss.get("valu_floor_ms") is not None:
            floor = max(iss["valu_floor_ms"], iss["salu_floor_ms"])
            out["issue"]["floor_ms"] = floor
            out["issue"]["frac"] = floor / k_ms
            out["issue"]["binding_pipe"] = "valu" if iss["valu_floor_ms"] >= iss["salu_floor_ms"] else "salu"
            if out["issue"]["frac"] > frac:
                out["bound"] = "latency"
                out["bound_detail"] = (
                    f"dependent-fetch latency: the busiest issue pipe ({out['issue']['binding_pipe']}) needs "
                    f"{floor:.3f} of the kernel's {k_ms:.3f} ms at full rate (frac {out['issue']['frac']:.2f}), "
                    f"HBM {frac:.3f}; waves wait {iss['wait_frac']:.0%} of their cycles")
    return out


def plan_inflight(inflight, W, H, world, strong, use_group, exported):
    """Frames in flight F and the GPU_MAX_HW_QUEUES value to set (None: keep `exported`).

    Enough of this rank's share of a frame to fill the GPU. A rank's share of a
    strong-scaled frame is too small (1/8 at 8 GPUs: ~4,000 tiles, its slowest pixels
    still ~0.22 ms), so strong mode keeps up to 8 frames in flight, each group on its own
    HIP stream. HIP maps streams onto GPU_MAX_HW_QUEUES hardware queues (default 4) and
    streams sharing a queue run in order, so the queue count is raised to 2F (at most 32)
    before the runtime starts: torch's own stream takes one more. Measured on one rank's
    1/8 share (tools/inflight_share.py, r02p): F = 8 gives 66 us/frame with 8 queues,
    41 us with 16; 32 queues with F >= 16 collapse (131-305 us). Config 2 with F = 4:
    0.049 ms with 4 queues, 0.033 with 8.
    """
    share_rows = -(-H // (world if strong else 1))
    tiles = ((W + 7) // 8) * ((share_rows + 7) // 8)
    if inflight > 0:
        F = inflight
    else:
        # 3 below 64k tiles: the 1080p car 0.1883 -> 0.1860 ms with 3 (4: 0.205; r03t)
        F = min(4, max(3 if tiles < 65536 else 2, -(-16384 // tiles) + 1))
        if use_group:  # at least the frames mode's F (one rank: the same frame), more for small shares
            F = min(8, max(F, -(-32768 // tiles)))
    if strong and not use_group:
        F = 1  # the torch path gathers one shared buffer per step
    have = int(exported) if str(exported).isdigit() else 4
    return F, (str(min(32, 2 * F)) if 2 * F > have else None)


def main():
    a = parse()
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(spawn_ranks(a))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    gloo = a.backend == "gloo"
    mode = a.mode if a.mode != "auto" else ("strong" if world > 1 else "frames")
    if mode == "frames" and world > 1:
        mode = "weak"
    strong = mode == "strong"
    use_group = strong and (a.gather == "rt" or (a.gather == "auto" and not gloo))
    if use_group and gloo:
        raise SystemExit("--gather rt needs the nccl backend (one GPU per rank)")
    cfg, W, H, mb, desc, target = WORKLOADS[a.config]
    F, hw_queues = plan_inflight(a.inflight, W, H, world, strong, use_group,
                                 os.environ.get("GPU_MAX_HW_QUEUES", ""))
    if hw_queues is not None:
        os.environ["GPU_MAX_HW_QUEUES"] = hw_queues  # before the HIP runtime starts

    import numpy as np
    import torch
    import torch.distributed as dist
    sys.path.insert(0, os.path.join(ROOT, "opengl-ray-tracer_amd"))
    import rtamd  # noqa: E402
    import tiling  # noqa: E402

    if world > 1 and gloo:
        torch.cuda.set_device(0)
        dist.init_process_group("gloo")
    elif world > 1:
        torch.cuda.set_device(local)
        with quiet_stdout():
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    # torch's work (gathers on the torch path, the stats all_reduce) on one non-default stream
    torch.cuda.set_stream(torch.cuda.Stream())

    sc = rtamd.Scene().generate(cfg, a.variant, W / H)
    sc_stats = sc.bvh_stats()
    if mode == "weak" and rank > 0:
        sc.orbit(target, float(rank))  # frame `rank` of the orbit: `rank` degrees about the look-at point
    fs = sc.serializeScene()
    kernel_id = {"auto": 0, "lane": 1, "packet": 2, "accel": 3}[a.kernel]

    plan = tiling.StripePlan(H, world if strong else 1, a.stripe)
    prank = rank if strong else 0
    rows = plan.rows(prank)

    # F frames in flight: F renderers per GPU (contexts, or the group's frame slots),
    # each with its own stream
    grp, ctxs, bufs = None, [], []
    if use_group:
        uid = [rtamd.group_unique_id() if rank == 0 else None]
        if world > 1:
            dist.broadcast_object_list(uid, src=0)
        with quiet_stdout():
            grp = rtamd.Group(uid=uid[0], nranks=world, rank=rank, device=local, frames=F)
        grp.upload(fs)
        grp.set_params(W, H, mb, not a.brute, a.fresnel, a.mt)
        for c_ in grp.contexts:
            c_.set_kernel(kernel_id)
            c_.set_schedule(SCHEDULES[a.schedule])
            c_.set_walk(a.walk)
            c_.debug_refit(a.refit)
        ctxs = list(grp.contexts)
    else:
        streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(F - 1)]
        for s_ in streams:
            c_ = rtamd.ComputeShader(torch.cuda.current_device())
            c_.set_stream(s_.cuda_stream)
            c_.upload(fs)
            c_.set_params(W, H, mb, not a.brute, a.fresnel, a.mt)
            c_.set_kernel(kernel_id)
            c_.set_schedule(SCHEDULES[a.schedule])
            c_.set_walk(a.walk)
            c_.debug_refit(a.refit)
            ctxs.append(c_)
            bufs.append(torch.empty((plan.rows_max, W, 4), dtype=torch.float32, device=dev))
    ctx = ctxs[0]

    # Work of this rank's rows on the reference walk (counting kernel, untimed). Over
    # rt_group the rows follow the root share, so rt_group_collect_stats counts them.
    def count_work():
        if use_group:
            st = grp.collect_stats(W, H, a.stripe)
            n = st["pixels"] // W
        else:
            st = ctx.collect_stats(W, H, plan.y0(prank), a.stripe, plan.world, rows)
            n = rows
        mine = torch.tensor([st["closest_rays"], st["shadow_rays"], rtamd.algorithmic_bytes(st, n * W, a.mt),
                             st["hits"]],
                            dtype=torch.float64, device="cpu" if gloo else dev)
        total = mine.clone()
        if world > 1:
            dist.all_reduce(total)
        return float(total[0] + total[1]), float(mine[2]), n  # all ranks' rays of one step

    share = None
    if use_group:
        share = 1 if a.root_share == "auto" else int(a.root_share)
        grp.set_root_share(share)
    rays_step, b_ref_rank, rows = count_work()

    cam, light = fs.camera, fs.light
    cams = camera_path(rtamd, sc, fs, a.camera_path, target)  # cams[i % len(cams)] for frame i
    last_cam = [None for _ in range(max(F, 1))]  # per renderer: the camera of its last frame
    anim = None
    if a.animate:
        if a.config not in (2, 3, 4) or (strong and not use_group):
            raise SystemExit("--animate: configs 2/3/4; with --gpus N > 1 over rt_group (--gather rt) or --mode weak")
        # the published scenes' animations (README.md:4): scene 1's bouncing spheres
        # (config 2), scene 2's turning wheels (configs 3/4)
        anim = sphere_frames(fs, 512) if a.config == 2 else wheel_frames(fs, 64)
        if a.upload == "device":
            if use_group:  # every member and frame slot (rt_group_set_animated)
                grp.set_animated(anim[0])
            else:
                for c_ in ctxs:
                    c_.set_animated(anim[0])
    # per renderer: the animation frames it was given, in order (over rt_group every slot
    # context is given every frame: one list)
    applied = [[] for _ in (ctxs if not use_group else [grp])]
    # --upload reference: each renderer's host keeps its own scene arrays, moved by the
    # reference's own upload calls (over rt_group: one host, its calls given to every slot)
    ref_up = ([rtamd.ReferenceUpload(fs, anim[0]) for _ in (ctxs if not use_group else [grp])]
              if anim is not None and a.upload == "reference" else None)

    def frame(i, inflight):
        if use_group:
            grp.set_camera(cams[i % len(cams)])    # SSBO 2 (src/main.cpp:328-330)
            last_cam[0] = i % len(cams)
            grp.set_light(light)   # SSBO 1 (:332-334)
            if ref_up is not None:  # the reference's upload calls, on every member and slot
                ref_up[0].upload(grp, anim[1][i % len(anim[1])])
                applied[0].append(i % len(anim[1]))
            elif anim is not None:
                grp.animate(anim[1][i % len(anim[1])])  # rt_group_animate: the device refit on every slot
                applied[0].append(i % len(anim[1]))
            grp.dispatch(W, H, a.stripe)  # this rank's stripes + send/recv to rank 0 + unstripe there
            if inflight == 1:
                group_sync()  # one frame at a time: the frame slots would otherwise overlap
            return
        c_ = ctxs[i % inflight]
        c_.set_camera(cams[i % len(cams)])
        last_cam[i % inflight] = i % len(cams)
        c_.set_light(light)
        if ref_up is not None:  # updateScene + updateBVH + their uploads, as the reference makes them
            ref_up[i % inflight].upload(c_, anim[1][i % len(anim[1])])
            applied[i % inflight].append(i % len(anim[1]))
        elif anim is not None:
            c_.animate(anim[1][i % len(anim[1])])  # updateScene + updateBVH on the device
            applied[i % inflight].append(i % len(anim[1]))
        buf = bufs[i % inflight]
        c_.dispatch_rows(W, H, plan.y0(prank), a.stripe, plan.world, rows, buf.data_ptr(), W * 16)
        if strong:
            tiling.gather_to_root(buf, plan)

    def group_sync():
        """rt_group_sync is bounded: a fan-in that never completes or an RCCL error
        ends the run with exit 4 instead of hanging in torch.cuda.synchronize()."""
        if grp is None:
            return
        try:
            grp.sync()
        except rtamd.RTError as e:
            print(f"bench.py rank {rank}: {e}", file=sys.stderr, flush=True)
            os._exit(4)

    def set_timing(on):
        """The renderers' device-time events (rt_set_kernel_timing; over rt_group also the
        phase events, rt_group_set_phase_timing). Each is a timestamped marker on the
        stream: a production loop records none, and they cost the car ~2 % in flight and
        ~5 us per waited frame (tools/group_cost.py, profiles/r04_group_cost.json). The
        passes that report device times record them; the timed frames and the waited
        frames do not."""
        for c_ in ctxs:
            c_.set_kernel_timing(on)
        if grp is not None:
            grp.set_phase_timing(on)

    def timed(inflight):
        """Wall time of a.steps frames between barriers, max over ranks."""
        for i in range(a.warmup * inflight):
            frame(i, inflight)
        group_sync()
        torch.cuda.synchronize()
        if grp is not None:
            grp.phase_times()  # drop the warm-up frames' phase times
        for c_ in ctxs:
            c_.kernel_times()  # drop warm-up dispatches
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(a.steps):
            frame(i, inflight)
        group_sync()
        torch.cuda.synchronize()  # the device: every renderer stream, RCCL and unstripe included
        if world > 1:
            dist.barrier()
        if grp is not None:
            phases[inflight] = grp.phase_times()
        el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device="cpu" if gloo else dev)
        if world > 1:
            dist.all_reduce(el, op=dist.ReduceOp.MAX)
        return float(el[0])

    # Strong mode over rt_group: before anything is timed, one gathered frame per frame
    # slot is compared bit for bit with rank 0's own single-GPU frame of the same camera.
    phases, selfcheck = {}, None
    if use_group:
        verdict = torch.zeros(1, dtype=torch.int64, device="cpu" if gloo else dev)
        want = None
        solo = None
        if rank == 0:
            solo = rtamd.ComputeShader(torch.cuda.current_device())
            solo.upload(fs)
            solo.set_params(W, H, mb, not a.brute, a.fresnel, a.mt)
            solo.set_kernel(kernel_id)
            if anim is not None and a.upload == "device":
                solo.set_animated(anim[0])
            solo_up = rtamd.ReferenceUpload(fs, anim[0]) if ref_up is not None else None
        bad = []
        for j in range(F):
            frame(j, F)
            group_sync()
            if rank == 0:
                solo.set_camera(cams[j % len(cams)])
                if solo_up is not None:  # the same frame's animation, given to one context
                    solo_up.upload(solo, anim[1][j % len(anim[1])])
                elif anim is not None:
                    solo.animate(anim[1][j % len(anim[1])])
                want = solo.render(W, H).view(np.uint32)
                bad.append(int((grp.read_image(W, H).view(np.uint32) != want).any(axis=-1).sum()))
        if solo is not None:
            solo.close()
        if rank == 0:
            verdict[0] = sum(bad)
            selfcheck = {"frames": F, "bad_pixels_per_slot": bad, "against": "rank 0's single-GPU frame (bit-exact)",
                         "ok": sum(bad) == 0}
        if world > 1:
            dist.broadcast(verdict, 0)
        if int(verdict[0]):
            print(f"bench.py rank {rank}: the gathered frame differs from the single-GPU frame: {bad}",
                  file=sys.stderr, flush=True)
            os._exit(5)

    # Root share (rt_group): with auto, every rank times the candidates the same way and
    # takes the same (max-over-ranks) verdict; the counted rays do not depend on it.
    share_probe = None
    if use_group and a.root_share == "auto":
        share_probe = {}
        steps = a.steps
        a.steps = max(4, 2 * F)
        set_timing(False)  # as the measured pass runs
        # rank 0's rows never cross a link: with more peers a larger share moves fewer bytes
        for k in ((1,) if world == 1 else (1, 2) if world < 4 else (1, 2, 3, 4)):
            grp.set_root_share(k)
            share_probe[k] = timed(F) / a.steps * 1e3
        a.steps = steps
        set_timing(True)
        best = min(share_probe, key=share_probe.get)
        grp.set_root_share(best)
        share = best
        share_probe = {str(k): v for k, v in share_probe.items()}
        rays_step, b_ref_rank, rows = count_work()  # this rank's rows at the chosen share

    serial = timed(1) if F > 1 else None  # device times recorded: the roofline's kernel time
    serial_kt = ctx.kernel_times() if F > 1 else None
    set_timing(F == 1)  # F = 1 (the profilers' --inflight 1): the main pass is the device-time pass
    # SURVEY §8(d)'s frame: upload + dispatch + completion, one at a time, FPS = 1 / median.
    # Each frame waits for its completion (the reference's loop, src/main.cpp:290-462), with
    # rt_set_latency_mode on: the setting for a host that waits for every frame.
    # The host sees a frame's end through the renderer's own wait (rt_sync_frame / the group's
    # bounded rt_group_sync), which polls an event instead of sleeping on the runtime's
    # completion interrupt; rt_sync_frame ends a latency-mode cost frame before the next
    # frame's tile-order kernels, which run behind it on the same stream. Over rt_group every rank starts each frame after a barrier,
    # so rank 0's frame includes the slowest peer's stripes crossing its link.
    serial_frames = []
    # at least three cost-order periods (rt_set_schedule: every 16th frame) before the waited
    # frames are timed, so latency mode's order (its split tiles recorded) has settled; fewer
    # where 48 frames would take over 0.1 s (config 5: 30; the brute-force 100k frames: none)
    est_ms = serial / a.steps * 1e3 if serial else None
    wait_warmup = max(a.warmup, 48 if est_ms is None else min(48, int(100.0 / max(est_ms, 1e-3))))
    if not (strong and not use_group):  # the torch-gather rehearsal has no waited-frame figure
        for c_ in ctxs:
            c_.set_latency_mode(1)

        def wait_frame():
            if grp is not None:
                group_sync()
            else:
                ctx.sync_frame()

        for i in range(wait_warmup):
            frame(i, 1)
            wait_frame()
        for i in range(a.steps):
            if world > 1:
                dist.barrier()
                torch.cuda.synchronize()
            t0 = time.perf_counter()
            frame(i, 1)
            wait_frame()
            serial_frames.append(time.perf_counter() - t0)
        for c_ in ctxs:
            c_.set_latency_mode(0)
            c_.kernel_times()
        if grp is not None:
            grp.phase_times()
    # The same waited frames from a C++ host (librthost.so rth_render_loop: the reference's
    # render loop over the C ABI, as a C++ host would run it, without the interpreter
    # between the calls). This is the figure reported as serial_frame_ms_median; the
    # Python loop's figure above is kept beside it.
    serial_frames_py = serial_frames
    serial_frames_host = []
    if grp is None and not strong:
        for c_ in ctxs:
            c_.set_latency_mode(1)
        frames_anim = anim[1] if anim is not None else None
        for n_ in (wait_warmup, a.steps):
            last_cam[0] = (n_ - 1) % len(cams)
            ms_ = rtamd.render_loop(ctx, cams, light, W, H, bufs[0].data_ptr(), W * 16, n_, True, anim=frames_anim,
                                    ref=ref_up[0] if ref_up is not None else None)
            if anim is not None:  # the C++ loop animates ctx 0 with frames 0, 1, ... (oracle bookkeeping)
                applied[0].extend(i % len(frames_anim) for i in range(n_))
        serial_frames_host = list(ms_ * 1e-3)
        for c_ in ctxs:
            c_.set_latency_mode(0)
        serial_frames = serial_frames_host
    serial_med_ranks = None
    if serial_frames and world > 1:
        med = [None] * world
        dist.all_gather_object(med, float(np.median(serial_frames)) * 1e3)
        serial_med_ranks = med
    # the same one-at-a-time frames with rt_set_latency_mode (what a host that waits for
    # each frame would set); reported beside serial_ms_per_step, not used for the roofline
    serial_lat = None
    if F > 1 and not use_group:
        ctx.set_latency_mode(1)
        serial_lat = timed(1)
        ctx.set_latency_mode(0)
        ctx.kernel_times()
    elapsed = timed(F)
    if F > 1:
        # the same frames in flight again with the device-time events, for the phase
        # times and kernel_ms_mean_inflight only (not timed)
        set_timing(True)
        steps = a.steps
        a.steps = max(2 * F, steps // 2)
        timed(F)
        a.steps = steps

    kt_if = np.concatenate([c_.kernel_times() for c_ in ctxs])
    rank_phases = None
    if grp is not None:
        mine = dict(phases.get(F, {}), rank=rank)
        rank_phases = [None] * world
        if world > 1:
            dist.all_gather_object(rank_phases, mine)
        else:
            rank_phases = [mine]
    # The render kernel's duration is taken where it runs alone (the one-frame-in-flight
    # pass): with frames in flight a dispatch's events also span the time it waits for
    # the other frame's waves to leave the CUs.
    kt = serial_kt if F > 1 else kt_if
    info = ctx.accel_info()
    kname = {1: "k_lane", 2: "k_packet", 3: "k_accel"}.get(info["last_kernel"], "?")
    k_ms = float(np.mean(kt)) if len(kt) else float("nan")
    k_med = float(np.median(kt)) if len(kt) else float("nan")

    if rank == 0:
        frames = a.steps * (world if mode == "weak" else 1)
        fps = frames / elapsed
        gather = None
        if strong:
            gather = ("rt_group: ncclSend/ncclRecv to rank 0 (RCCL over xGMI) + k_unstripe, C ABI (include/rt_group.h)"
                      if use_group else f"torch.distributed.gather ({a.backend}) + index_copy_ unpermute")
        suffix = "".join(f"_{n}" for n, on in (("brute", a.brute), ("mt", a.mt), ("fresnel", a.fresnel),
                                                  ("variant", a.variant), ("animate", a.animate)) if on)
        if a.camera_path != "static":
            suffix += "_" + a.camera_path
        refits = {"rebuilds": [c_.debug_anim_rebuilds() for c_ in ctxs], "refits": [c_.debug_refits() for c_ in ctxs]}
        # strong lines: the same kernel over this rank's rows; the single-GPU entry with its
        # issue floors scaled by the row share (roofline docstring)
        pmc = pmc_entry(f"config{a.config}_n{1 if strong else world}_{a.kernel}{suffix}")
        out = {
            "metric": METRIC,
            "value": rays_step * a.steps / elapsed / 1e6,
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": elapsed / a.steps * 1e3,
            "frames_in_flight": F,
            "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES", "4 (HIP default)"),
            "serial_ms_per_step": (serial if serial is not None else elapsed) / a.steps * 1e3,
            "serial_ms_per_step_latency_mode": (serial_lat / a.steps * 1e3) if serial_lat is not None else None,
            "serial_frame_ms_median": float(np.median(serial_frames)) * 1e3 if serial_frames else None,
            "serial_frame_ms_median_python": float(np.median(serial_frames_py)) * 1e3 if serial_frames_py else None,
            "serial_frame_median_mode": (("C++ host loop (librthost.so rth_render_loop: camera + light upload, "
                                          + ("rt_animate, " if anim is not None and ref_up is None else
                                             "rth_upload_animated (rt_update_shapes per record, rts_update_bvh, "
                                             "rt_update_nodes), " if ref_up is not None else "") +
                                          "dispatch, rt_sync per frame), rt_set_latency_mode on"
                                          ) if serial_frames_host else
                                         ("each frame waited for (rt_sync: host polls the stream), "
                                          "rt_set_latency_mode on, Python loop") if serial_frames and not use_group else
                                         ("each frame waited for on every rank (rt_group_sync), ranks start "
                                          "each frame after a barrier, rt_set_latency_mode on; rank 0's median")
                                         if serial_frames else None),
            "serial_frame_ms_median_per_rank": serial_med_ranks,
            "fps_serial_median": 1.0 / float(np.median(serial_frames)) if serial_frames else None,
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (procedural stand-in meshes, fixed seed; the reference's .obj assets are absent)",
            "backend": a.backend if world > 1 else None,
            "mode": mode,
            "ranks_seen": world,
            "config": {"workload": f"config {a.config}: {desc}" + (" (222-strip road)" if a.variant else ""),
                       "width": W, "height": H, "maxBounces": mb, "useBVH": int(not a.brute),
                       "useFresnel": int(a.fresnel), "triangle_test": "moller-trumbore" if a.mt else "barycentric",
                       "animate": (None if not a.animate else
                                   ("scene 1's three spheres bounce (bounceSphere, src/main.cpp:438-445)" if a.config == 2
                                    else "wheels turn (updateWheelAnimations)") +
                                   (", uploaded as the reference does (one rt_update_shapes per record, updateBVH "
                                    "on the host, rt_update_nodes; src/main.cpp:336-346), device refit per frame"
                                    if ref_up is not None else ", rt_animate (device refit) per frame")),
                       "shapes": len(fs.shapes), "bvh_nodes": len(fs.nodes),
                       "bvh_max_leaf": sc_stats["max_leaf"], "kernel": a.kernel, "walk": a.walk,
                       "parallelism": (f"row-stripes{a.stripe}x{world}+gather" if strong else
                                       f"frame-sharded x{world} (one frame per GPU per step, orbit 1 deg/rank)"
                                       if mode == "weak" else "1 GPU")},
            "gather": gather,
            "root_share": share,
            "root_share_probe_ms": share_probe,
            "group_selfcheck": selfcheck,
            "group_phases_ms": rank_phases,
            "fps": fps,
            "mrays_primary_per_s": W * H * fps / 1e6,
            "rays_per_step": rays_step,
            "kernel_ms_mean": k_ms,
            "kernel_ms_median": k_med,
            "kernel_ms_mean_inflight": float(np.mean(kt_if)) if len(kt_if) else float("nan"),
            "roofline": roofline(info, kname, k_ms, rows * W, b_ref_rank, pmc, share=rows / H if strong else None),
            "accel": info,
            "scene_updates": refits if anim is not None else None,
            "cpu_baseline": None,
            "parity": None,
        }
        thr = a.cpu_threads or host_cores()
        if world == 1 and not a.no_cpu:
            out["cpu_baseline"] = cpu_baseline(rtamd, fs, W, H, mb, a.cpu_seconds, thr,
                                               (not a.brute, a.fresnel, a.mt))
            out["cpu_baseline"]["reference_cpu_path"] = cpu_reference_1core(rtamd, a.cpu_seconds / 2, cfg, a.variant,
                                                                            W, H)
        moving = len(cams) > 1
        if moving:
            out["camera_path"] = {"kind": a.camera_path, "cameras": len(cams),
                                  "last_camera_per_renderer": [x for x in last_cam if x is not None]}
        if use_group and anim is not None:
            # rank 0's last gathered frame against the oracle rendering the group's scene
            # (every slot context was given every frame: the last records, and the node
            # boxes grown by all of them); outside the timed region, whole frame
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import oracle  # noqa: E402  (checker only)
            group_sync()
            img = grp.read_image(W, H)
            fk = (ref_up[0].scene(fs) if ref_up is not None else animated_oracle_scene(fs, anim[0], anim[1], applied[0]))
            fk.camera = cams[last_cam[0]:last_cam[0] + 1].copy()
            ref, _ = oracle.render(fk, W, H, oracle.params(W, H, mb, not a.brute, a.fresnel, a.mt), threads=thr)
            chk = parity_check([img], 0, ref, "")
            out["parity"] = dict(chk, frames_checked=1, rows_checked=[0, H],
                                 against=("oracle/rt_oracle.c (GLSL restated) on rank 0's last gathered frame: its "
                                          "camera, the group's last records and node boxes grown over every frame "
                                          "it was given"),
                                 animation_frames_applied=[len(applied[0])])
        if mode == "frames" and (anim is not None or moving):
            # every renderer's last timed frame against the oracle rendering that
            # renderer's scene: its last frame's camera, and when animated its last
            # records and the boxes grown by every frame it was given (outside the timed
            # region; whole frames)
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import oracle  # noqa: E402  (checker only)
            torch.cuda.synchronize()
            checks, host_nodes_ok = [], True
            for k, b_ in enumerate(bufs):
                if anim is not None and not applied[k]:
                    continue
                if last_cam[k] is None:
                    continue
                fk = (animated_oracle_scene(fs, anim[0], anim[1], applied[k]) if anim is not None else
                      rtamd.FlatScene(fs.shapes, fs.nodes, fs.indices, fs.camera, fs.light))
                fk.camera = cams[last_cam[k]:last_cam[k] + 1].copy()
                if ref_up is not None:  # the host's own updateBVH (rts_update_bvh) grew the same boxes
                    host_nodes_ok = host_nodes_ok and all(
                        np.array_equal(ref_up[k].nodes[f].view(np.uint32), fk.nodes[f].view(np.uint32))
                        for f in ("boundsMin", "boundsMax"))
                ref, _ = oracle.render(fk, W, H, oracle.params(W, H, mb, not a.brute, a.fresnel, a.mt), threads=thr)
                checks.append(parity_check([b_.cpu().numpy()], 0, ref, ""))
            out["parity"] = {"max_abs": max(c["max_abs"] for c in checks),
                             "bad_pixels": sum(c["bad_pixels"] for c in checks), "frames_checked": len(checks),
                             "tol": PARITY_TOL, "rows_checked": [0, H],
                             "against": ("oracle/rt_oracle.c (GLSL restated) on each renderer's last frame: its "
                                         "camera" + (", its last records, node boxes grown by oracle.update_bvh "
                                                     "(updateBVH restated) over every frame it was given"
                                                     if anim is not None else "")),
                             "animation_frames_applied": [len(x) for x in applied] if anim is not None else None,
                             "host_nodes_equal_oracle": host_nodes_ok if ref_up is not None else None,
                             "ok": all(c["ok"] for c in checks) and host_nodes_ok}
        if mode == "frames" and anim is None and not moving:
            # the timed frames themselves, against the oracle (outside the timed region)
            if out["cpu_baseline"] is not None:
                ry0, ref = cpu_baseline.last_image
            else:
                sys.path.insert(0, os.path.join(ROOT, "oracle"))
                import oracle  # noqa: E402  (checker only)
                ry0 = max(0, H // 2 - 8)
                ref, _ = oracle.render(fs, W, H, oracle.params(W, H, mb, not a.brute, a.fresnel, a.mt),
                                       y0=ry0, out_rows=min(16, H - ry0), threads=thr)
            torch.cuda.synchronize()
            out["parity"] = parity_check([b_.cpu().numpy() for b_ in bufs], ry0, ref,
                                         "oracle/rt_oracle.c (GLSL restated), rows of the same frame")
        print(json.dumps(out), flush=True)
        if out["parity"] is not None and not out["parity"]["ok"]:
            print(f"bench.py: the timed frames differ from the oracle: {out['parity']}", file=sys.stderr)
            sys.exit(3)
    if grp is not None:
        grp.close()
    for c_ in ctxs:
        c_.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
