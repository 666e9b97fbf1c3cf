"""The reference's own per-frame upload through the drop-in ABI (-m gpu).

The reference animates by uploading: updateScene issues one glBufferSubData per
animated shape record (src/main.cpp:981-992), updateBVH grows the node objects on
the host (:1068-1077) and serializeBVH + one glBufferSubData re-upload the nodes
(:336-346). Its drop-ins are rt_update_shapes (per record) and rt_update_nodes.
The renderer applies whatever was written by the next dispatch as one device
refit (flush_updates in rt_kernels.hip): no accelerator rebuild unless a moved
shape changes its kind of bound or the new node boxes stop nesting. These tests
check that every frame is the oracle's frame of the host's own scene, that the
refit path equals a fresh upload of the same arrays bit for bit (including the
rebuild cases and the brute-force and Moller-Trumbore branches), and that no
rebuild happens on the published animations.
"""
import numpy as np
import pytest
import torch

import bench
import oracle
import rtamd

pytestmark = pytest.mark.gpu
TOL = 1e-4


@pytest.fixture(scope="module")
def ctx():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    c = rtamd.ComputeShader(0)
    yield c
    c.close()


@pytest.fixture(scope="module")
def fresh():
    """A second context: every scene uploaded whole (the accelerator built from scratch)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    c = rtamd.ComputeShader(0)
    yield c
    c.close()


def check(img, ref, what):
    diff = np.abs(img.astype(np.float64) - ref.astype(np.float64))
    bad = int((diff > TOL).any(axis=-1).sum())
    assert np.isfinite(img).all() == np.isfinite(ref).all(), what
    assert bad == 0, f"{what}: {bad} pixels over {TOL}, max diff {np.nanmax(diff):.3g}"


def same(a, b, what):
    bad = int((a.view(np.uint32) != b.view(np.uint32)).any(axis=-1).sum())
    assert bad == 0, f"{what}: {bad} pixels differ"


@pytest.mark.parametrize("cfg", [3, 2])
def test_reference_upload_loop_matches_oracle(ctx, cfg):
    """64 frames of main.cpp's loop call for call from the C++ host (librthost.so
    rth_render_loop_ref: camera, light, one rt_update_shapes per animated record,
    rts_update_bvh, one rt_update_nodes, dispatch, wait): config 3's four wheels turn
    (updateWheelAnimations), config 2's three spheres bounce (bounceSphere). Every
    frame equals the oracle's frame of the host's own scene (its records and its
    updateBVH-grown nodes); every frame is one device refit and none a rebuild; the
    last frame equals the same animation through rt_animate (the device's updateBVH)."""
    W, H = (192, 108) if cfg == 3 else (160, 120)
    mb = 3 if cfg == 3 else 1
    fs = rtamd.generate(cfg, 0, W, H)
    ids, frames = bench.wheel_frames(fs, 64) if cfg == 3 else bench.sphere_frames(fs, 64)
    ctx.upload(fs)
    ctx.set_params(W, H, mb, True)
    ctx.set_kernel(rtamd.KERNEL_AUTO)
    ru = rtamd.ReferenceUpload(fs, ids)
    out = torch.empty((H, W, 4), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    r0, f0 = ctx.debug_anim_rebuilds(), ctx.debug_refits()
    p = oracle.params(W, H, mb)
    for k in range(64):
        rtamd.render_loop(ctx, fs.camera, fs.light, W, H, out.data_ptr(), W * 16, 1, True, anim=[frames[k]], ref=ru)
        want, _ = oracle.render(ru.scene(fs), W, H, p)
        check(out.cpu().numpy(), want, f"config {cfg} frame {k}")
    assert ctx.debug_anim_rebuilds() == r0, "the published animation rebuilt the accelerator"
    assert ctx.debug_refits() - f0 == 64
    assert ctx.accel_info()["scene_tree"] == 1
    last = out.cpu().numpy()
    # the same frames through rt_animate (the node growth on the device)
    ctx.upload(fs)
    ctx.set_animated(ids)
    for k in range(64):
        ctx.animate(frames[k])
    got = ctx.read_nodes(len(fs.nodes))
    for f in ("boundsMin", "boundsMax"):
        assert np.array_equal(got[f].view(np.uint32), ru.nodes[f].view(np.uint32)), f
    same(ctx.render(W, H), last, "rt_animate against the reference's upload")


def _soup(seed, n_tri=1500):
    rng = np.random.default_rng(seed)
    sc = rtamd.Scene()
    for i in range(n_tri):
        c = rng.uniform(-20, 20, 3)
        c[1] = rng.uniform(-4, 4)
        v = c + rng.normal(size=(3, 3)) * rng.uniform(0.3, 2.0)
        sc.add_triangle(v[0], v[1], v[2], invert=bool(i % 2),
                        mat=rtamd.material(color=rng.uniform(0, 1, 3), specular=0.3 if i % 5 == 0 else 0.0))
    for _ in range(30):
        sc.add_sphere(rng.uniform(-20, 20, 3), rng.uniform(0.3, 2.5), mat=rtamd.material(color=rng.uniform(0, 1, 3)))
    sc.add_wall((-10, -10, -25), 20, 15, (0.1, 0.2, 1.0), mat=rtamd.material(specular=0.8))
    sc.add_plane((0, 0, 1), (0, 0, -40), mat=rtamd.material(color=(0.2, 0.5, 0.2), specular=0.0))
    sc.set_camera((5, -25, 45), 60, 4 / 3)
    sc.LookAt((0, 0, 0))
    sc.set_light((10, -30, 20), (1, 1, 1), 40)
    sc.buildBVH(6)
    return sc.serializeScene()


def _moved(shapes, ids, rng, k):
    s = shapes.copy()
    for i in ids:
        t = s["type"][i]
        d = (rng.normal(size=3) * 0.8).astype(np.float32)
        if t == 0:
            s["sphereCenter"][i] += d
        elif t == 2:
            s["wallStart"][i] += d
        elif t == 3:
            c = (s["triP1"][i].astype(np.float64) + s["triP2"][i] + s["triP3"][i]) / 3
            a = 0.2 * (k + 1)
            for f in ("triP1", "triP2", "triP3"):
                q = s[f][i].astype(np.float64) - c
                q = np.array([q[0] * np.cos(a) - q[2] * np.sin(a), q[1], q[0] * np.sin(a) + q[2] * np.cos(a)])
                s[f][i] = (q + c + d).astype(np.float32)
    return s


@pytest.mark.parametrize("seed", [1, 2])
def test_update_path_equals_fresh_upload(ctx, fresh, seed):
    """rt_update_shapes (single records and ranges) + rt_update_nodes, refit on the
    device, against the same arrays uploaded whole, bit for bit, for the BVH branch
    (barycentric and Moller-Trumbore) and the brute-force branch: moves the refit
    absorbs, a triangle collapsing to a sliver and node boxes that stop nesting
    (host rebuilds), node boxes alone, and shapes moved without a node update (the
    reference's frame then keeps the old boxes)."""
    W, H = 200, 150
    fs = _soup(seed)
    rng = np.random.default_rng(seed)
    tri = np.where(fs.shapes["type"] == 3)[0]
    ids = np.sort(np.concatenate([rng.choice(tri, 60, replace=False), np.where(fs.shapes["type"] == 0)[0][:6],
                                  np.where(fs.shapes["type"] == 2)[0]])).astype(np.int32)
    host = rtamd.FlatScene(fs.shapes.copy(), fs.nodes.copy(), fs.indices, fs.camera, fs.light)
    ctx.upload(fs)
    ctx.set_kernel(rtamd.KERNEL_AUTO)
    fresh.set_kernel(rtamd.KERNEL_AUTO)

    def frames(what):
        fresh.upload(host)
        for bvh, mt in ((True, False), (True, True), (False, False)):
            for c in (ctx, fresh):
                c.set_params(W, H, 3, bvh, False, mt)
            same(ctx.render(W, H), fresh.render(W, H), f"{what} bvh {bvh} mt {mt}")
        ctx.set_params(W, H, 3, True)

    frames("as uploaded")
    r0 = ctx.debug_anim_rebuilds()
    for k in range(3):  # the refit absorbs these
        host.shapes = _moved(host.shapes, ids, rng, k)
        lo = int(ids[0])
        ctx.update_shapes(lo, host.shapes[lo:lo + 1])
        for j in ids[1:]:
            ctx.update_shapes(int(j), host.shapes[j:j + 1])
        ctx.update_shapes(int(tri[5]), host.shapes[tri[5]:tri[5] + 3])  # a range, partly unmoved
        rtamd.update_bvh(host, ids)
        ctx.update_nodes(host.nodes)
        frames(f"step {k}")
    assert ctx.debug_anim_rebuilds() == r0
    # a moved triangle collapses to a sliver: no conservative bound, a host rebuild
    t = int(ids[np.isin(ids, tri)][0])
    host.shapes["triP3"][t] = host.shapes["triP1"][t] + (host.shapes["triP2"][t] - host.shapes["triP1"][t]) * 0.5
    ctx.update_shapes(t, host.shapes[t:t + 1])
    rtamd.update_bvh(host, np.array([t], np.int32))
    ctx.update_nodes(host.nodes)
    frames("sliver")
    assert ctx.debug_anim_rebuilds() == r0 + 1
    # node boxes alone, grown (still nested): a refit
    host.nodes["boundsMin"] -= np.float32(0.75)
    host.nodes["boundsMax"] += np.float32(0.75)
    ctx.update_nodes(host.nodes)
    frames("nodes grown")
    assert ctx.debug_anim_rebuilds() == r0 + 1
    # a leaf box that no longer lies in its parent's: the scene tree cannot hold, a rebuild
    leaf = int(np.where(host.nodes["leftChild"] == -1)[0][0])
    host.nodes["boundsMax"][leaf] += np.float32(50.0)
    ctx.update_nodes(host.nodes)
    frames("not nested")
    assert ctx.debug_anim_rebuilds() == r0 + 2
    # shapes moved with no node update: the old boxes decide which leaves are tested
    host.shapes = _moved(host.shapes, ids[:20], rng, 5)
    for j in ids[:20]:
        ctx.update_shapes(int(j), host.shapes[j:j + 1])
    frames("shapes only")
    p = oracle.params(W, H, 3)
    want, _ = oracle.render(host, W, H, p)
    check(ctx.render(W, H), want, "shapes only vs oracle")


def test_update_then_animate_and_readback(ctx):
    """rt_update_nodes followed by rt_animate in the same frame: the host's boxes
    apply first, then the device grows them (rt_read_nodes = updateBVH over the
    host's boxes); rt_update_shapes of shapes outside the animated set in between."""
    W, H = 160, 120
    fs = rtamd.generate(2, 0, W, H)
    ids, frames = bench.sphere_frames(fs, 4)
    ctx.upload(fs)
    ctx.set_params(W, H, 1, True)
    ctx.set_animated(ids)
    host = rtamd.FlatScene(fs.shapes.copy(), fs.nodes.copy(), fs.indices, fs.camera, fs.light)
    other = np.int32(len(fs.shapes) - 1)
    for k in range(4):
        host.nodes["boundsMax"][-1] += np.float32(0.5)
        ctx.update_nodes(host.nodes)
        moved = host.shapes[other:other + 1].copy()
        moved["material"]["color"] = np.float32([0.1 * k, 0.5, 0.9])
        host.shapes[other] = moved[0]
        ctx.update_shapes(int(other), moved)
        ctx.animate(frames[k])
        host.shapes[ids] = frames[k]
        rtamd.update_bvh(host, ids)
        got = ctx.read_nodes(len(host.nodes))
        for f in ("boundsMin", "boundsMax"):
            assert np.array_equal(got[f].view(np.uint32), host.nodes[f].view(np.uint32)), (k, f)
        want, _ = oracle.render(host, W, H, oracle.params(W, H, 1))
        check(ctx.render(W, H), want, f"frame {k}")


def test_kernel_timing_off_reports_nothing(ctx):
    """rt_set_kernel_timing(0): a dispatch records no events, and rt_last_kernel_ms
    refuses (RT_ERR_INVALID) instead of returning an earlier dispatch's time."""
    W, H = 64, 48
    fs = rtamd.generate(2, 0, W, H)
    ctx.upload(fs)
    ctx.set_params(W, H, 1, True)
    ctx.set_kernel_timing(1)
    ctx.render(W, H)
    assert ctx.last_kernel_ms() > 0
    ctx.set_kernel_timing(0)
    try:
        ctx.render(W, H)
        with pytest.raises(rtamd.RTError):
            ctx.last_kernel_ms()
        ctx.set_params(W, H, 1, False)  # the brute-force sub-context's path too
        ctx.render(W, H)
        with pytest.raises(rtamd.RTError):
            ctx.last_kernel_ms()
    finally:
        ctx.set_kernel_timing(1)


@pytest.mark.parametrize("mode", ["mt", "brute", "mt_brute"])
def test_animated_mt_and_brute_frames_refit(ctx, fresh, mode):
    """Moller-Trumbore and brute-force frames of an animated scene: the sub-contexts
    (the MT accelerator, the one-leaf brute tree) follow rt_animate / rt_update_shapes
    by the same device refit (MT: boxes, grazing cones, per-ray padding constants and
    axis slabs recomputed from the current records) instead of the literal scan or a
    rebuild. Every frame equals a fresh upload of the same scene (the accelerator built
    from scratch) bit for bit, and the oracle at the end."""
    W, H = 192, 108
    fs = rtamd.generate(3, 0, W, H)
    ids, frames = bench.wheel_frames(fs, 8)
    mt, bvh = "mt" in mode, mode != "brute" and mode != "mt_brute"
    ctx.upload(fs)
    ctx.set_params(W, H, 3, bvh, False, mt)
    ctx.set_kernel(rtamd.KERNEL_AUTO)
    ctx.set_animated(ids)
    host = rtamd.FlatScene(fs.shapes.copy(), fs.nodes.copy(), fs.indices, fs.camera, fs.light)
    ctx.render(W, H)  # the sub-context exists from here on
    for k in range(8):
        ctx.animate(frames[k])
        host.shapes[ids] = frames[k]
        oracle.update_bvh(host, ids)
        fresh.upload(host)
        fresh.set_params(W, H, 3, bvh, False, mt)
        fresh.set_kernel(rtamd.KERNEL_AUTO)
        same(ctx.render(W, H), fresh.render(W, H), f"{mode} frame {k}")
    assert ctx.accel_info()["last_kernel"] == rtamd.KERNEL_ACCEL
    want, _ = oracle.render(host, W, H, oracle.params(W, H, 3, bvh, False, mt))
    check(ctx.render(W, H), want, f"{mode} vs oracle")
    # the reference's own upload on the same context (no rt_animate): MT / brute too
    ctx.set_animated(np.zeros(0, np.int32))
    ru = rtamd.ReferenceUpload(host, ids)
    for k in range(4):
        ru.upload(ctx, frames[(k + 3) % 8])
        fresh.upload(ru.scene(host))
        same(ctx.render(W, H), fresh.render(W, H), f"{mode} reference upload {k}")


@pytest.mark.parametrize("refit", [-1, 0, 1, 2, 3, 4])
def test_refit_launch_modes_equal_fresh_upload(ctx, fresh, refit):
    """Every launch shape of k_refit (rt_debug_refit: 0 one launch ordered by tickets,
    1 two launches, 2 one launch reading the records itself, 3 one launch in start
    order, 4 as 2 from a device copy of the records; -1, the default, picks 1 or 2)
    refits the car's turning wheels to the frames of a fresh
    upload, bit for bit, barycentric (back-face cones recomputed) and Moller-Trumbore."""
    W, H = 192, 108
    fs = rtamd.generate(3, 0, W, H)
    ids, frames = bench.wheel_frames(fs, 6)
    try:
        for mt in (False, True):
            host = rtamd.FlatScene(fs.shapes.copy(), fs.nodes.copy(), fs.indices, fs.camera, fs.light)
            ctx.upload(fs)
            ctx.debug_refit(refit)
            ctx.set_params(W, H, 3, True, False, mt)
            ctx.set_kernel(rtamd.KERNEL_AUTO)
            ctx.set_animated(ids)
            ctx.render(W, H)
            r0 = ctx.debug_anim_rebuilds()
            for k in range(6):
                ctx.animate(frames[k])
                host.shapes[ids] = frames[k]
                oracle.update_bvh(host, ids)
                fresh.upload(host)
                fresh.set_params(W, H, 3, True, False, mt)
                fresh.set_kernel(rtamd.KERNEL_AUTO)
                same(ctx.render(W, H), fresh.render(W, H), f"refit {refit} mt {mt} frame {k}")
            assert ctx.debug_anim_rebuilds() == r0
    finally:
        ctx.debug_refit(-1)
        ctx.set_animated(np.zeros(0, np.int32))


# --------------------------------------------------------------------------
# The animated frame on the multi-GPU group (rt_group_update_shapes / _nodes,
# rt_group_set_animated / rt_group_animate; include/rt_group.h)

def _copy_surface(ptr, pitch, W, H):
    """rank 0's pitched RGBA32F surface (rt_group_device_image) to the host."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    out = np.empty((H, W, 4), np.float32)
    rc = hip.hipMemcpy2D(ctypes.c_void_p(out.ctypes.data), ctypes.c_size_t(W * 16), ctypes.c_void_p(ptr),
                         ctypes.c_size_t(pitch), ctypes.c_size_t(W * 16), ctypes.c_size_t(H), 2)  # DeviceToHost
    assert rc == 0, f"hipMemcpy2D {rc}"
    return out


@pytest.mark.parametrize("upload", ["device", "reference"])
@pytest.mark.parametrize("cfg", [3, 2])
@pytest.mark.parametrize("kind", ["copy8_3840x2160", "rccl1_1920x1080"])
def test_group_animated_frames(ctx, kind, cfg, upload):
    """16 animated frames through the group, 3 frames in flight: the car's wheels turn
    (config 3) or scene 1's spheres bounce (config 2), uploaded by rt_group_animate (the
    device's updateBVH) or by the reference's own calls on the group (one
    rt_group_update_shapes per animated record, updateBVH on the host, one
    rt_group_update_nodes: rth_group_upload_animated). Cases: 8 copy-transport members
    on one GPU at 3840x2160 (sky rows on: the band follows the grown root box every
    frame) and a 1-rank RCCL group (ncclCommInitRank) at 1920x1080. Every gathered
    frame equals a single context given the same calls, bit for bit; the last frame
    equals the oracle of the animated scene (4K: a band of rows through the scene);
    no slot context rebuilds its accelerator (src/main.cpp:336-346, 981-992, 1068-1077)."""
    W, H = (3840, 2160) if kind.startswith("copy8") else (1920, 1080)
    mb = 3 if cfg == 3 else 1
    F, n_frames = 3, 16
    fs = rtamd.generate(cfg, 0, W, H)
    ids, frames = bench.wheel_frames(fs, n_frames) if cfg == 3 else bench.sphere_frames(fs, 4 * n_frames)
    if cfg == 2:
        frames = frames[::4]  # 1/15 s apart: the spheres move visibly from frame to frame
    g = (rtamd.Group([0] * 8, rtamd.GATHER_COPY, frames=F) if kind.startswith("copy8") else
         rtamd.Group(uid=rtamd.group_unique_id(), nranks=1, rank=0, device=0, frames=F))
    try:
        g.set_timeout(60000)
        g.upload(fs)
        g.set_params(W, H, mb, True)
        ctx.upload(fs)
        ctx.set_params(W, H, mb, True)
        ctx.set_kernel(rtamd.KERNEL_AUTO)
        if upload == "device":
            g.set_animated(ids)
            ctx.set_animated(ids)
        else:
            ru_g, ru_c = rtamd.ReferenceUpload(fs, ids), rtamd.ReferenceUpload(fs, ids)
        rebuilds0 = [c.debug_anim_rebuilds() for c in g.contexts]
        k = 0
        bands = []
        while k < n_frames:
            burst = []
            for _ in range(min(F, n_frames - k)):  # F frames in flight, nothing waited between them
                if upload == "device":
                    g.animate(frames[k])
                else:
                    ru_g.upload(g, frames[k])
                g.dispatch(W, H, 8)
                burst.append((k, g.device_image()))
                bands.append(g.sky_band())
                k += 1
            g.sync()
            for j, (ptr, pitch) in burst:
                if upload == "device":
                    ctx.animate(frames[j])
                else:
                    ru_c.upload(ctx, frames[j])
                same(_copy_surface(ptr, pitch, W, H), ctx.render(W, H), f"{kind} config {cfg} {upload} frame {j}")
        assert [c.debug_anim_rebuilds() for c in g.contexts] == rebuilds0, "an accelerator was rebuilt"
        if g.nranks > 1 and cfg == 3:
            assert all(0 < y0 < y1 <= H for y0, y1 in bands), f"sky rows off: {bands}"  # the car's sky is on top
        last = _copy_surface(*g.device_image(), W, H)
        fk = (bench.animated_oracle_scene(fs, ids, frames, list(range(n_frames))) if upload == "device" else
              ru_g.scene(fs))
        p = oracle.params(W, H, mb)
        y0, rows = (H // 2 - 32, 64) if H > 1080 else (0, H)
        want, _ = oracle.render(fk, W, H, p, y0=y0, out_rows=rows, threads=16)
        check(last[y0:y0 + rows], want, f"{kind} config {cfg} {upload}: last frame against the oracle")
    finally:
        g.close()


def test_refit_set_stays_bounded(ctx, fresh):
    """A host that writes a different 1 % of config 5's 100,000 triangles every frame
    (rt_update_shapes, src/main.cpp:981-992) for 50 frames: the refit set drops the
    shapes written in earlier frames once they outnumber max(4096, S / 16) and the live
    ones (compact_refit_set), so a flush's pinned records stay bounded
    (rt_debug_refit_stats) instead of growing to every shape touched, and every frame
    equals a fresh upload of the same arrays, bit for bit."""
    W, H = 256, 144
    fs = rtamd.generate(5, 0, W, H)
    S = len(fs.shapes)
    rng = np.random.default_rng(11)
    ctx.upload(fs)
    ctx.set_params(W, H, 3, True)
    ctx.set_kernel(rtamd.KERNEL_AUTO)
    fresh.set_params(W, H, 3, True)
    shapes = fs.shapes.copy()
    order = rng.permutation(S)
    per = S // 100
    worst = {"entries": 0, "flush_bytes": 0}
    for k in range(50):
        ids = np.sort(order[k * per:(k + 1) * per])
        moved = _moved(shapes, ids, rng, k)
        shapes[ids] = moved[ids]
        for i in ids:  # one record per call, as updateScene writes them
            ctx.update_shapes(int(i), shapes[i:i + 1])
        got = ctx.render(W, H)
        st = ctx.debug_refit_stats()
        worst = {key: max(worst[key], st[key]) for key in worst}
        fresh.upload(rtamd.FlatScene(shapes, fs.nodes, fs.indices, fs.camera, fs.light))
        same(got, fresh.render(W, H), f"frame {k}")
    bound = 2 * per + max(4096, S // 16)
    assert ctx.debug_refit_stats()["compactions"] >= 1
    assert worst["entries"] <= bound, worst
    assert worst["flush_bytes"] <= bound * (rtamd.SHAPE_DTYPE.itemsize + 4), worst


def _rebuild_state(c):
    import ctypes as C
    fn = c._lib.rt_debug_rebuild_state
    fn.argtypes = [C.c_void_p, C.c_void_p]
    out = np.zeros(4, np.int32)
    assert fn(c._h, out.ctypes.data) == 0
    return dict(zip(["running", "requested", "swapped", "suspended"], out.tolist()))


def _async(c, on):
    import ctypes as C
    fn = c._lib.rt_debug_async_rebuild
    fn.argtypes = [C.c_void_p, C.c_int]
    assert fn(c._h, int(on)) == 0


@pytest.mark.parametrize("mode,asy", [("animate", 1), ("reference", 1), ("animate", 0)])
def test_async_rebuild_keeps_frames_exact(ctx, fresh, mode, asy):
    """A moved shape whose kind of bound changes (a wheel triangle collapsing to a sliver,
    then back) and node boxes that stop nesting make the refit ask for an accelerator
    rebuild. It runs on a host thread over a snapshot of the records while the frames go
    on; every frame, before, during and after the swap, equals a fresh upload of the same
    records bit for bit, and the rebuilt accelerator lands (swapped, the scene tree on
    again). The car's wheels turn every frame (rt_animate, or the reference's own uploads)."""
    import time
    W, H = 240, 135
    fs = rtamd.generate(3, 0, W, H)
    ids, wheel = bench.wheel_frames(fs, 40)
    host = rtamd.FlatScene(fs.shapes.copy(), fs.nodes.copy(), fs.indices, fs.camera, fs.light)
    ctx.upload(fs)
    ctx.set_params(W, H, 3, True)
    ctx.set_kernel(rtamd.KERNEL_AUTO)
    fresh.set_params(W, H, 3, True)
    _async(ctx, asy)
    if mode == "animate":
        ctx.set_animated(ids)
    else:
        ru = rtamd.ReferenceUpload(fs, ids)
    s0 = _rebuild_state(ctx)
    sliver = 7  # a wheel triangle (index into ids)
    saw_running, trace = False, []
    for k in range(40):
        recs = wheel[k].copy()
        if 5 <= k < 20:  # collapsed onto its first edge's midpoint: no conservative bound
            recs["triP3"][sliver] = recs["triP1"][sliver] + (recs["triP2"][sliver] - recs["triP1"][sliver]) * 0.5
        host.shapes[ids] = recs
        rtamd.update_bvh(host, ids)
        if mode == "animate":
            ctx.animate(recs)
        else:
            ru.upload(ctx, recs)
        if k == 25:  # a leaf box grown out of its parent's: the scene tree cannot hold
            leaf = int(np.where(host.nodes["leftChild"] == -1)[0][0])
            host.nodes["boundsMax"][leaf] += np.float32(40.0)
            if mode == "animate":
                ctx.update_nodes(host.nodes)
            else:
                ru.nodes["boundsMax"][leaf] += np.float32(40.0)
                ctx.update_nodes(ru.nodes)
        got = ctx.render(W, H)
        saw_running = saw_running or bool(_rebuild_state(ctx)["running"])
        trace.append(_rebuild_state(ctx)["requested"] - s0["requested"])
        fresh.upload(rtamd.FlatScene(host.shapes, host.nodes, fs.indices, fs.camera, fs.light))
        same(got, fresh.render(W, H), f"{mode} frame {k} {_rebuild_state(ctx)}")
    # let the last rebuild land, then one more frame through it
    t0 = time.time()
    while _rebuild_state(ctx)["running"] and time.time() - t0 < 30:
        time.sleep(0.01)
        got = ctx.render(W, H)
    same(ctx.render(W, H), fresh.render(W, H), f"{mode} after the swap")
    st = _rebuild_state(ctx)
    assert st["requested"] - s0["requested"] >= 2, st  # the sliver (at least) and the nesting
    assert (st["swapped"] - s0["swapped"] >= 1 or not asy) and not st["running"] and not st["suspended"], st
    print(f"rebuild {mode} async={asy}: {st}, a rebuild was seen running: {saw_running}, requests by frame {trace}")
