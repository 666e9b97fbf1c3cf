"""bench.py's host logic on CPU: --gpus N launches torchrun as a child, a
WORLD_SIZE that disagrees with --gpus is refused before any GPU work, the
CPU baseline sizes itself to the host, the weak mode's orbit camera turns
about the config's own look-at point, and the roofline never claims more
than the HBM peak from the bytes it is given."""
import os
import subprocess
import sys

import numpy as np
import pytest

import bench
import rtamd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_gpus_spawns_torchrun_child(monkeypatch):
    seen = {}

    def fake_call(cmd):
        seen["cmd"] = cmd
        return 7

    monkeypatch.setattr(bench.subprocess, "call", fake_call)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "5"])
    assert bench.spawn_ranks(bench.parse(["--gpus", "4", "--steps", "5"])) == 7
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "127.0.0.1" in cmd
    assert cmd[-4:] == ["--gpus", "4", "--steps", "5"]


def test_world_size_mismatch_is_refused():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=60)
    assert r.returncode != 0
    assert "WORLD_SIZE=1" in r.stderr


def test_cpu_threads_follow_the_host(monkeypatch):
    monkeypatch.setenv("OMP_NUM_THREADS", "16")
    assert bench.host_cores() == 16
    monkeypatch.delenv("OMP_NUM_THREADS")
    assert bench.host_cores() == len(os.sched_getaffinity(0))
    assert bench.cpu_model() != ""


@pytest.mark.parametrize("cfg", [2, 3, 5])
def test_orbit_turns_about_the_look_at_point(cfg):
    _, W, H, _, _, target = bench.WORKLOADS[cfg]
    sc = rtamd.Scene().generate(cfg, 0, W / H)
    c0 = sc.camera()
    sc.orbit(target, 1.0)
    c1 = sc.camera()
    t = np.asarray(target, np.float64)
    p0 = c0["Position"][0].astype(np.float64) - t
    p1 = c1["Position"][0].astype(np.float64) - t
    assert p1[1] == pytest.approx(p0[1])  # about the vertical axis
    assert np.linalg.norm(p1) == pytest.approx(np.linalg.norm(p0), rel=1e-6)
    turn = np.degrees(np.arctan2(p0[0], p0[2]) - np.arctan2(p1[0], p1[2]))
    assert abs(abs(turn) - 1.0) < 1e-4
    # rank r's camera still looks at the same point as rank 0's
    for c, p in ((c0, p0), (c1, p1)):
        f = c["Front"][0].astype(np.float64)
        assert np.allclose(f, -p / np.linalg.norm(p), atol=1e-5)


def test_roofline_fraction_is_physical():
    info = {"record_bytes": 1_000_000}
    r = bench.roofline(info, "k_accel", 0.3, 1920 * 1080, 8.5e11, {"bytes": 45e6, "source": "x"})
    assert r["frac"] == pytest.approx(45e6 / 0.3e-3 / 1e9 / 8000)
    assert r["frac"] < 1 and r["traffic"] == 45e6
    assert r["reference_equivalent_GBps"] > 8000  # the skipped reference work is reported, not claimed
    r2 = bench.roofline(info, "k_accel", 0.3, 1920 * 1080, 8.5e11, None)
    assert r2["achieved"] == pytest.approx((16 * 1920 * 1080 + 1e6) / 0.3e-3 / 1e9)
    assert r2["traffic"] is None


def test_inflight_plan_and_hardware_queues():
    """Frames in flight per workload, and the hardware-queue count raised to 2F (<= 32)
    so that the F renderer streams and torch's own stream do not share queues."""
    # car, 1 GPU: 2 frames in flight, the box's 4 queues suffice
    assert bench.plan_inflight(0, 1920, 1080, 1, False, False, "4") == (3, "6")
    # 3840x2160: 2 frames
    assert bench.plan_inflight(0, 3840, 2160, 1, False, False, "4") == (2, None)
    # 800x600: 4 frames, 8 queues
    assert bench.plan_inflight(0, 800, 600, 1, False, False, "4") == (4, "8")
    # a rank's 1/8 stripe share over rt_group: 8 frames, 16 queues
    assert bench.plan_inflight(0, 1920, 1080, 8, True, True, "4") == (8, "16")
    # one rank over rt_group renders the single-GPU frame: the frames mode's F (round 3 gave it 2)
    assert bench.plan_inflight(0, 1920, 1080, 1, True, True, "4") == (3, "6")
    assert bench.plan_inflight(0, 1920, 1080, 2, True, True, "4") == (3, "6")
    # torch-gather strong path: one frame
    assert bench.plan_inflight(0, 1920, 1080, 2, True, False, "4") == (1, None)
    # an explicit F; never above 32 queues; an export that already suffices is kept
    assert bench.plan_inflight(20, 1920, 1080, 1, False, False, "") == (20, "32")
    assert bench.plan_inflight(8, 1920, 1080, 1, False, False, "16") == (8, None)


def test_parity_check_of_timed_frames():
    """bench.parity_check: every in-flight context's last frame against the oracle rows."""
    ref = np.random.default_rng(1).random((4, 8, 4)).astype(np.float32)
    good = np.zeros((10, 8, 4), np.float32)
    good[3:7] = ref
    r = bench.parity_check([good, good.copy()], 3, ref, "t")
    assert r["ok"] and r["bad_pixels"] == 0 and r["max_abs"] == 0 and r["frames_checked"] == 2
    assert r["rows_checked"] == [3, 7]
    bad = good.copy()
    bad[4, 2, 1] += 2e-4
    bad[5, 5, 0] = np.nan
    r = bench.parity_check([good, bad], 3, ref, "t")
    assert not r["ok"] and r["bad_pixels"] == 2 and r["max_abs"] == np.inf
    # a NaN the oracle also produces is not a mismatch
    ref2 = ref.copy()
    ref2[0, 0, 0] = np.nan
    g2 = good.copy()
    g2[3, 0, 0] = np.nan
    assert bench.parity_check([g2], 3, ref2, "t")["ok"]


def test_roofline_names_the_binding_resource():
    """With the SQ passes' issue floors the line says what binds: latency when the
    busiest issue pipe's floor is a larger fraction of the kernel time than HBM."""
    info = {"record_bytes": 1_000_000}
    iss = {"valu_floor_ms": 0.09, "salu_floor_ms": 0.11, "wait_frac": 0.3, "valu_busy": 0.5}
    r = bench.roofline(info, "k_accel", 0.3, 1920 * 1080, 8.5e11, {"bytes": 45e6, "source": "x", "issue": iss})
    assert r["bound"] == "latency" and r["issue"]["binding_pipe"] == "salu"
    assert r["issue"]["frac"] == pytest.approx(0.11 / 0.3) and r["frac"] < r["issue"]["frac"]
    # an HBM-heavy kernel keeps "hbm"
    r2 = bench.roofline(info, "k", 0.3, 1920 * 1080, 0.0, {"bytes": 2e9, "source": "x", "issue": iss})
    assert r2["bound"] == "hbm"


def test_strong_roofline_is_latency_with_scaled_issue_floors():
    """A strong line's kernel renders 1/P of the rows: the single-GPU PMC entry's
    DRAM bytes are not its own (traffic null), its issue floors scale by the row
    share, and the line names the latency bound rather than defaulting to hbm."""
    info = {"record_bytes": 1_000_000}
    iss = {"valu_floor_ms": 0.08, "salu_floor_ms": 0.07, "wait_frac": 0.3, "valu_busy": 0.6}
    pmc = {"bytes": 39e6, "source": "x", "issue": iss}
    r = bench.roofline(info, "k_accel", 0.05, 1920 * 135, 1e11, pmc, share=0.125)
    assert r["traffic"] is None and r["traffic_over_algorithmic"] is None
    assert r["achieved"] == pytest.approx((16 * 1920 * 135 + 1e6) / 0.05e-3 / 1e9)
    assert r["issue"]["valu_floor_ms"] == pytest.approx(0.01) and r["issue"]["row_share"] == 0.125
    assert r["issue"]["frac"] == pytest.approx(0.01 / 0.05)
    assert r["bound"] == "latency" and "row share" in r["issue"]["basis"]


def test_bouncing_spheres_and_their_oracle_scene():
    """bench --animate on config 2: scene 1's spheres 0-2 bounce as bounceSphere sets
    them (src/main.cpp:438-445, 1079-1082), and the oracle scene of a renderer that was
    given frames j1, j2, ... holds the last frame's records and node boxes grown to
    every frame's spheres (updateBVH is grow-only)."""
    fs = rtamd.generate(2, 0, 800, 600)
    ids, frames = bench.sphere_frames(fs, 512)
    assert list(ids) == [0, 1, 2] and len(frames) == 512
    base = fs.shapes[ids]
    for f in (0, 1, 77, 511):
        t = np.float32(f / 60.0)
        for k, (amp, fr) in enumerate(bench.BOUNCES):
            want = base["sphereCenter"][k][1] + np.float32(amp) * np.sin(np.float32(fr) * t)
            assert frames[f]["sphereCenter"][k][1] == want
            assert np.array_equal(frames[f]["sphereCenter"][k][[0, 2]], base["sphereCenter"][k][[0, 2]])
    applied = [3, 100, 250, 7]
    fk = bench.animated_oracle_scene(fs, ids, frames, applied)
    assert np.array_equal(fk.shapes[ids], frames[7]) and np.array_equal(fk.shapes[3:], fs.shapes[3:])
    assert np.array_equal(fs.shapes[ids], base)  # the caller's scene is untouched
    root = fk.nodes[-1]
    for j in applied:
        c, r = frames[j]["sphereCenter"], frames[j]["sphereRadius"]
        assert (root["boundsMin"] <= (c - r[:, None]).min(0)).all()
        assert (root["boundsMax"] >= (c + r[:, None]).max(0)).all()
    assert (fk.nodes["boundsMin"] <= fs.nodes["boundsMin"]).all()  # grow-only


@pytest.mark.parametrize("kind", ["orbit", "dolly"])
def test_camera_paths(kind):
    """--camera-path: orbit = 720 cameras 0.5 degrees apart about the look-at point, each
    looking at it; dolly = Camera::ProcessKeyboard steps of SPEED / 60 along Front, 96 in
    and 96 back to the start (src/camera.hpp:75-90)."""
    cfg, W, H, mb, _, target = bench.WORKLOADS[3]
    sc = rtamd.Scene().generate(cfg, 0, W / H)
    fs = sc.serializeScene()
    cams = bench.camera_path(rtamd, sc, fs, kind, target)
    assert cams.dtype == rtamd.CAMERA_DTYPE and cams.flags["C_CONTIGUOUS"]
    p0 = fs.camera["Position"][0].astype(np.float64)
    t = np.asarray(target, np.float64)
    if kind == "orbit":
        assert len(cams) == 720
        r0 = np.linalg.norm(p0 - t)
        for k in (0, 179, 359, 719):
            p = cams["Position"][k].astype(np.float64)
            assert abs(np.linalg.norm(p - t) - r0) < 1e-3 * r0
            d = (t - p) / np.linalg.norm(t - p)
            assert np.dot(d, cams["Front"][k]) > 0.9999  # looks at the target
        a = (cams["Position"][0].astype(np.float64) - t)[[0, 2]]  # azimuth about the vertical axis
        b = (cams["Position"][1].astype(np.float64) - t)[[0, 2]]
        ang = np.degrees(np.arccos(np.dot(a, b) / np.linalg.norm(a) / np.linalg.norm(b)))
        assert abs(ang - 0.5) < 1e-3
    else:
        assert len(cams) == 192
        step = np.linalg.norm(cams["Position"][1].astype(np.float64) - cams["Position"][0])
        assert abs(step - 0.25) < 1e-5
        assert np.allclose(cams["Position"][0], p0) and np.allclose(cams["Position"][-1], cams["Position"][1], atol=1e-4)
        assert (cams["Front"] == fs.camera["Front"][0]).all()
    assert bench.camera_path(rtamd, sc, fs, "static", target).shape == (1,)
