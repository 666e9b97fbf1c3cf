"""HIP renderer parity against the CPU oracle (-m gpu; needs an MI355X).

Every comparison goes through the C ABI (librtamd.so). Tolerance: 1e-4 per
channel (BASELINE.json north_star); the kernels are built to reproduce the
oracle's IEEE sequence, so the expected difference is 0 except for powf
(device ocml vs glibc), which only moves the specular term by ulps.
Oracle sizes are kept to a few seconds of CPU; full-size frames are checked
through size-independent properties (packet == lane, stripe-split invariance,
determinism, band == crop).
"""
import numpy as np
import pytest
import torch

import oracle
import rtamd

pytestmark = pytest.mark.gpu
TOL = 1e-4
CFG_BOUNCES = {1: 3, 2: 1, 3: 3, 5: 3}


@pytest.fixture(scope="module")
def ctx():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    c = rtamd.ComputeShader(0)
    yield c
    c.close()


def gpu_rows(ctx, fs, W, H, p, y0=0, rows=None, kernel=rtamd.KERNEL_PACKET):
    rows = H - y0 if rows is None else rows
    ctx.upload(fs)
    ctx.set_params(p.resX, p.resY, p.maxBounces, p.useBVH, p.useFresnel, p.useMollerTrumbore)
    ctx.set_kernel(kernel)
    out = torch.full((rows, W, 4), -7.0, dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()  # the renderer's stream does not wait on torch's
    ctx.dispatch_rows(W, H, y0, 1, 1, rows, out.data_ptr(), W * 16)
    ctx.sync()
    return out.cpu().numpy()


def check(img, ref, what):
    diff = np.abs(img.astype(np.float64) - ref.astype(np.float64))
    bad = int((diff > TOL).any(axis=-1).sum())
    assert np.isfinite(img).all() == np.isfinite(ref).all(), what
    assert bad == 0, f"{what}: {bad} pixels over {TOL}, max diff {np.nanmax(diff):.3g}"


CASES = [
    # cfg, W, H, y0, rows, maxBounces, bvh, fresnel, mt
    (1, 160, 120, 0, None, 3, 1, 0, 0),
    (1, 160, 120, 0, None, 3, 0, 0, 0),
    (2, 200, 150, 0, None, 1, 1, 0, 0),
    (2, 200, 150, 0, None, 4, 1, 1, 0),
    (2, 120, 90, 0, None, 2, 0, 1, 1),
    (2, 800, 600, 280, 24, 1, 1, 0, 0),
    (3, 1920, 1080, 520, 24, 3, 1, 0, 0),
    (3, 1920, 1080, 600, 16, 3, 1, 1, 1),
    (3, 240, 135, 0, None, 3, 0, 0, 0),
    (5, 1920, 1080, 500, 24, 3, 1, 0, 0),
    (5, 480, 270, 0, None, 2, 1, 1, 1),
]


KERNELS = [rtamd.KERNEL_ACCEL, rtamd.KERNEL_PACKET, rtamd.KERNEL_LANE]


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("case", CASES, ids=lambda c: "c%d_%dx%d_y%d_b%d_bvh%d_f%d_mt%d" % (
    c[0], c[1], c[2], c[3], c[5], c[6], c[7], c[8]))
def test_parity_vs_oracle(ctx, case, kernel):
    cfg, W, H, y0, rows, mb, bvh, fr, mt = case
    fs = rtamd.generate(cfg, 0, W, H)
    p = oracle.params(W, H, mb, bvh, fr, mt)
    ref, _ = oracle.render(fs, W, H, p, y0=y0, out_rows=rows)
    img = gpu_rows(ctx, fs, W, H, p, y0, rows, kernel)
    check(img, ref, f"cfg{cfg} kernel{kernel}")


@pytest.mark.parametrize("case", [(1, 160, 120, 0, 120, 3, 1), (1, 160, 120, 0, 120, 3, 0),
                                  (2, 200, 150, 0, 150, 1, 1), (2, 100, 75, 0, 75, 3, 0),
                                  (3, 1920, 1080, 520, 16, 3, 1), (5, 1920, 1080, 500, 16, 3, 1)])
def test_stats_match_oracle_counts(ctx, case):
    """The counting kernel's totals are the oracle's, exactly (they price B_alg)."""
    cfg, W, H, y0, rows, mb, bvh = case
    fs = rtamd.generate(cfg, 0, W, H)
    p = oracle.params(W, H, mb, bvh)
    _, st_ref = oracle.render(fs, W, H, p, y0=y0, out_rows=rows, stats=True)
    ctx.upload(fs)
    ctx.set_params(W, H, mb, bvh)
    st = ctx.collect_stats(W, H, y0, 1, 1, rows)
    assert st == st_ref


def test_golden_frames_on_gpu(golden_dir):
    """The committed oracle frames, rendered by the HIP kernels."""
    import os
    from make_golden import FRAME_CASES
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    data = np.load(os.path.join(golden_dir, "frames.npz"))
    c = rtamd.ComputeShader(0)
    for (cfg, w, h, mb, bvh, fr, mt) in FRAME_CASES:
        fs = rtamd.generate(cfg, 0, w, h)
        key = f"c{cfg}_w{w}_h{h}_b{mb}_bvh{bvh}_f{fr}_mt{mt}"
        for k in KERNELS:
            img = gpu_rows(c, fs, w, h, oracle.params(w, h, mb, bvh, fr, mt), kernel=k)
            check(img, data[key], key)
    c.close()


# --------------------------------------------------------------------------
# Full-size properties (no oracle at 1920x1080)

@pytest.mark.parametrize("cfg", [3, 5])
def test_full_frame_packet_equals_lane(ctx, cfg):
    W, H = 1920, 1080
    fs = rtamd.generate(cfg, 0, W, H)
    p = oracle.params(W, H, CFG_BOUNCES[cfg])
    a = gpu_rows(ctx, fs, W, H, p, kernel=rtamd.KERNEL_PACKET)
    b = gpu_rows(ctx, fs, W, H, p, kernel=rtamd.KERNEL_LANE)
    c = gpu_rows(ctx, fs, W, H, p, kernel=rtamd.KERNEL_ACCEL)
    assert ctx.accel_info()["last_kernel"] == rtamd.KERNEL_ACCEL
    assert np.array_equal(a, b)
    assert np.array_equal(a, c)
    assert (a[..., 3] == 1).all()


@pytest.mark.parametrize("cfg,kernel", [(3, rtamd.KERNEL_PACKET), (3, rtamd.KERNEL_ACCEL), (5, rtamd.KERNEL_ACCEL)])
def test_full_frame_stripes_reassemble(ctx, cfg, kernel):
    """Rendering the 4 interleaved stripe sets of a 4-GPU plan and scattering
    them back gives the single-dispatch frame, bit for bit (the multi-GPU path
    minus the RCCL gather); for the accelerated kernel also with the cost
    order, the counter-free dispatches and (config 5) ray compaction."""
    import tiling
    W, H = (1920, 1080) if cfg == 3 else (960, 544)
    fs = rtamd.generate(cfg, 0, W, H)
    p = oracle.params(W, H, 3)
    full = gpu_rows(ctx, fs, W, H, p, kernel=kernel)
    plan = tiling.StripePlan(H, 4, 8)
    bufs = torch.zeros((4, plan.rows_max, W, 4), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    for _ in range(3):  # later rounds reuse the cost order of each stripe set's tile count
        for r in range(4):
            ctx.dispatch_rows(W, H, plan.y0(r), 8, 4, plan.rows(r), bufs[r].data_ptr(), W * 16)
        ctx.sync()
        img = tiling.unpermute(bufs, plan).cpu().numpy()
        assert np.array_equal(img, full)


def test_deterministic_and_band_equals_crop(ctx):
    W, H = 1920, 1080
    fs = rtamd.generate(3, 0, W, H)
    p = oracle.params(W, H, 3)
    a = gpu_rows(ctx, fs, W, H, p)
    b = gpu_rows(ctx, fs, W, H, p)
    assert np.array_equal(a, b)
    band = gpu_rows(ctx, fs, W, H, p, y0=333, rows=77)
    assert np.array_equal(band, a[333:410])


def test_own_surface_dispatch_and_readback(ctx):
    W, H = 96, 64
    fs = rtamd.generate(2, 0, W, H)
    ctx.upload(fs)
    ctx.set_params(W, H, 1, True)
    ctx.set_kernel(rtamd.KERNEL_AUTO)
    img = ctx.render(W, H)
    ref, _ = oracle.render(fs, W, H, oracle.params(W, H, 1))
    check(img, ref, "own surface")
    ms = ctx.last_kernel_ms()
    assert ms > 0
    assert len(ctx.kernel_times()) >= 1


# --------------------------------------------------------------------------
# Edge cases the reference exercises implicitly

def _empty_scene(W, H):
    fs = rtamd.generate(1, 0, W, H)
    return rtamd.FlatScene(fs.shapes[:0].copy(), fs.nodes[:0].copy(), fs.indices[:0].copy(), fs.camera, fs.light)


@pytest.mark.parametrize("bvh", [1, 0])
def test_empty_scene_is_background(ctx, bvh):
    W, H = 37, 29  # not multiples of the 8x8 tile
    fs = _empty_scene(W, H)
    p = oracle.params(W, H, 3, bvh)
    ref, _ = oracle.render(fs, W, H, p)
    check(gpu_rows(ctx, fs, W, H, p), ref, "empty")


def test_no_nodes_with_shapes(ctx):
    """N = 0: the BVH branch sees nothing, the brute branch sees the shapes."""
    W, H = 64, 48
    fs = rtamd.generate(2, 0, W, H)
    fs0 = rtamd.FlatScene(fs.shapes, fs.nodes[:0].copy(), fs.indices[:0].copy(), fs.camera, fs.light)
    for bvh in (1, 0):
        p = oracle.params(W, H, 2, bvh)
        ref, _ = oracle.render(fs0, W, H, p)
        check(gpu_rows(ctx, fs0, W, H, p), ref, f"N=0 bvh{bvh}")


def test_zero_bounces_is_black(ctx):
    W, H = 32, 16
    fs = rtamd.generate(2, 0, W, H)
    img = gpu_rows(ctx, fs, W, H, oracle.params(W, H, 0))
    assert (img[..., :3] == 0).all() and (img[..., 3] == 1).all()


def test_bad_tree_is_rejected(ctx):
    fs = rtamd.generate(2, 0, 64, 48)
    bad = fs.nodes.copy()
    inner = np.where(bad["leftChild"] != -1)[0][0]
    bad["rightChild"][inner] = len(bad) + 5
    with pytest.raises(rtamd.RTError) as e:
        ctx.upload(rtamd.FlatScene(fs.shapes, bad, fs.indices, fs.camera, fs.light))
    assert e.value.code == -5
    badidx = fs.indices.copy()
    badidx[0] = len(fs.shapes)
    with pytest.raises(rtamd.RTError):
        ctx.upload(rtamd.FlatScene(fs.shapes, fs.nodes, badidx, fs.camera, fs.light))


def test_update_shapes_and_nodes(ctx):
    """Partial shape upload + node refit (the reference's animate path,
    src/main.cpp:336-346) match a full re-upload of the same arrays."""
    W, H = 160, 120
    fs = rtamd.generate(2, 0, W, H)
    ctx.upload(fs)
    ctx.set_params(W, H, 3, True)
    moved = fs.shapes.copy()
    moved["sphereCenter"][0] += np.float32([0, -2, 0])   # bounceSphere
    nodes = fs.nodes.copy()
    nodes["boundsMin"][-1] -= 3
    nodes["boundsMax"][-1] += 3
    ctx.update_shapes(0, moved[:1])
    ctx.update_nodes(nodes)
    out = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    ctx.dispatch_rows(W, H, 0, 1, 1, H, out.data_ptr(), W * 16)
    ctx.sync()
    fs2 = rtamd.FlatScene(moved, nodes, fs.indices, fs.camera, fs.light)
    ref, _ = oracle.render(fs2, W, H, oracle.params(W, H, 3))
    check(out.cpu().numpy(), ref, "update")
    changed = nodes.copy()
    changed["leftChild"][-1], changed["rightChild"][-1] = changed["rightChild"][-1], changed["leftChild"][-1]
    with pytest.raises(rtamd.RTError):
        ctx.update_nodes(changed)


def test_pitched_destination(ctx):
    W, H = 72, 40
    fs = rtamd.generate(2, 0, W, H)
    p = oracle.params(W, H, 2)
    ctx.upload(fs)
    ctx.set_params(W, H, 2, True)
    pitch_px = W + 5
    out = torch.full((H, pitch_px, 4), 9.0, dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    ctx.dispatch_rows(W, H, 0, 1, 1, H, out.data_ptr(), pitch_px * 16)
    ctx.sync()
    o = out.cpu().numpy()
    ref, _ = oracle.render(fs, W, H, p)
    check(o[:, :W], ref, "pitched")
    assert (o[:, W:] == 9.0).all()


# --------------------------------------------------------------------------
# The accelerator's exactness on adversarial scenes: giant leaves that mix
# bounded shapes with unbounded ones (planes, ±Y walls, thin triangles,
# triangles whose stored plane is off their vertices), exact distance ties.

def _soup(seed, n_tri=2500):
    rng = np.random.default_rng(seed)
    sc = rtamd.Scene()
    for i in range(n_tri):
        c = rng.uniform(-20, 20, 3)
        c[1] = rng.uniform(-4, 4)
        v = c + rng.normal(size=(3, 3)) * rng.uniform(0.3, 2.0)
        if i % 97 == 0:  # sliver: third vertex on the first edge
            v[2] = v[0] + (v[1] - v[0]) * 0.37 + rng.normal(size=3) * 1e-4
        sc.add_triangle(v[0], v[1], v[2], invert=bool(i % 2),
                        mat=rtamd.material(color=rng.uniform(0, 1, 3), specular=0.3 if i % 5 == 0 else 0.0))
    for i in range(40):
        sc.add_sphere(rng.uniform(-20, 20, 3), rng.uniform(0.3, 2.5),
                      mat=rtamd.material(color=rng.uniform(0, 1, 3)))
    sc.add_wall((-30, 6, -30), 60, 60, (0, 1, 0), mat=rtamd.material(color=(0.6, 0.2, 0.3), specular=0.0))
    sc.add_wall((-10, -10, -25), 20, 15, (0.1, 0.2, 1.0), mat=rtamd.material(specular=0.8))
    sc.add_plane((0, 0, 1), (0, 0, -40), mat=rtamd.material(color=(0.2, 0.5, 0.2), specular=0.0))
    sc.set_camera((5, -25, 45), 60, 4 / 3)
    sc.LookAt((0, 0, 0))
    sc.set_light((10, -30, 20), (1, 1, 1), 40)
    sc.buildBVH(1)  # one split: two leaves of ~1,300 shapes each
    fs = sc.serializeScene()
    tri = np.where(fs.shapes["type"] == 3)[0]
    # stored plane shifted off the vertices for a few triangles
    fs.shapes["planeD"][tri[::211]] += np.float32(0.5)
    return fs


@pytest.mark.parametrize("seed", [1, 2])
@pytest.mark.parametrize("fresnel", [0, 1])
def test_accel_exact_on_adversarial_soup(ctx, seed, fresnel):
    W, H = 200, 150
    fs = _soup(seed)
    p = oracle.params(W, H, 3, True, fresnel)
    ref, _ = oracle.render(fs, W, H, p)
    img = gpu_rows(ctx, fs, W, H, p, kernel=rtamd.KERNEL_ACCEL)
    info = ctx.accel_info()
    assert info["built"] and info["last_kernel"] == rtamd.KERNEL_ACCEL and info["always_prims"] > 0
    assert info["scene_tree"] == 1
    check(img, ref, f"soup {seed}")


def test_accel_ties_resolve_like_the_reference(ctx):
    """Each road triangle duplicated with another colour: identical distances;
    the reference keeps the first in its walk order."""
    W, H = 1920, 1080
    fs = rtamd.generate(3, 0, W, H)
    road = np.where((fs.shapes["type"] == 3) & (fs.shapes["material"]["specularStrength"] > 0.2))[0]
    dup = fs.shapes[road].copy()
    dup["material"]["color"] = (1.0, 0.0, 0.0)
    shapes = np.concatenate([fs.shapes, dup])
    sc_nodes, sc_idx = oracle.build_bvh(shapes, 25)
    fs2 = rtamd.FlatScene(shapes, sc_nodes, sc_idx, fs.camera, fs.light)
    p = oracle.params(W, H, 3)
    ref, _ = oracle.render(fs2, W, H, p, y0=900, out_rows=40)
    for k in KERNELS:
        img = gpu_rows(ctx, fs2, W, H, p, y0=900, rows=40, kernel=k)
        check(img, ref, f"ties kernel {k}")


def test_far_camera_falls_back_exactly(ctx):
    """A camera far outside the scene's magnitude skips the accelerator (its
    padding is relative to the scene); the frame still matches the oracle."""
    W, H = 64, 48
    fs = rtamd.generate(2, 0, W, H)
    cam = fs.camera.copy()
    cam["Position"] = cam["Position"] - cam["Front"] * np.float32(60000.0)
    fs2 = rtamd.FlatScene(fs.shapes, fs.nodes, fs.indices, cam, fs.light)
    p = oracle.params(W, H, 2)
    ref, _ = oracle.render(fs2, W, H, p)
    img = gpu_rows(ctx, fs2, W, H, p, kernel=rtamd.KERNEL_AUTO)
    assert ctx.accel_info()["last_kernel"] == rtamd.KERNEL_PACKET
    check(img, ref, "far camera")


@pytest.mark.parametrize("walk", [0, 1, 99])
@pytest.mark.parametrize("scene", ["c2", "c3", "c5", "soup"])
def test_scene_tree_equals_reference_tree(ctx, scene, walk):
    """The scene tree (rt_set_tree, accel.h SceneTree) against the reference
    tree walk: identical full frames for every walk policy."""
    if scene == "soup":
        W, H, mb = 800, 600, 3
        fs = _soup(1)
    else:
        cfg = int(scene[1])
        W, H = (800, 600) if cfg == 2 else (1920, 1080)
        mb = CFG_BOUNCES[cfg]
        fs = rtamd.generate(cfg, 0, W, H)
    p = oracle.params(W, H, mb)
    ctx.set_walk(walk)
    try:
        ctx.set_tree(rtamd.TREE_REFERENCE)
        a = gpu_rows(ctx, fs, W, H, p, kernel=rtamd.KERNEL_ACCEL)
        ctx.set_tree(rtamd.TREE_SCENE)
        b = gpu_rows(ctx, fs, W, H, p, kernel=rtamd.KERNEL_ACCEL)
    finally:
        ctx.set_walk(-1)
        ctx.set_tree(rtamd.TREE_SCENE)
    info = ctx.accel_info()
    assert info["scene_tree"] == 1 and info["tree_nested"] == 1 and info["last_kernel"] == rtamd.KERNEL_ACCEL
    bad = int((a != b).any(axis=-1).sum())
    assert bad == 0, f"{bad} pixels differ between the scene tree and the reference tree"


@pytest.mark.parametrize("cap", [1, 3, 6])
@pytest.mark.parametrize("scene", ["c3", "c5", "soup"])
def test_scene_tree_stack_overflow_is_exact(ctx, scene, cap):
    """Scene-tree walks whose stack runs out (capped by rt_debug_scene_stack)
    finish on the reference tree: still the reference tree's image."""
    if scene == "soup":
        W, H, fs = 400, 300, _soup(2)
    else:
        W, H = 960, 540
        fs = rtamd.generate(int(scene[1]), 0, W, H)
    p = oracle.params(W, H, 3)
    ctx.set_walk(-1)
    ctx.set_tree(rtamd.TREE_REFERENCE)
    a = gpu_rows(ctx, fs, W, H, p, kernel=rtamd.KERNEL_ACCEL)
    ctx.set_tree(rtamd.TREE_SCENE)
    try:
        for walk in (0, 1, 99):
            ctx.set_walk(walk)
            ctx.debug_scene_stack(cap)
            b = gpu_rows(ctx, fs, W, H, p, kernel=rtamd.KERNEL_ACCEL)
            assert ctx.accel_info()["scene_tree"] == 1
            bad = int((a != b).any(axis=-1).sum())
            assert bad == 0, f"walk {walk} cap {cap}: {bad} pixels differ"
    finally:
        ctx.debug_scene_stack(0)
        ctx.set_walk(-1)


@pytest.mark.parametrize("walk", [0, 1, 99])
def test_walk_policies_identical(ctx, walk):
    """Packet / per-lane / hybrid walks render the same frame (config 5 rows)."""
    W, H = 1920, 1080
    fs = rtamd.generate(5, 0, W, H)
    p = oracle.params(W, H, 3)
    ref, _ = oracle.render(fs, W, H, p, y0=480, out_rows=16)
    ctx.set_walk(walk)
    try:
        img = gpu_rows(ctx, fs, W, H, p, y0=480, rows=16, kernel=rtamd.KERNEL_ACCEL)
    finally:
        ctx.set_walk(-1)
    check(img, ref, f"walk {walk}")


@pytest.mark.gpu
@pytest.mark.parametrize("sched", [rtamd.SCHED_COST, rtamd.SCHED_COST_XCD])
def test_cost_schedule_identical_images(ctx, sched):
    """rt_set_schedule: the cost-ordered dispatch (default) and its XCD-banded
    variant render the same image as row-major, frame after frame (every pixel
    written: the surface is NaN before each dispatch), and across a change of
    tile count."""
    fs = rtamd.generate(3, 0, 320, 180)
    ctx.upload(fs)
    ctx.set_params(320, 180, 3, True)
    ctx.set_kernel(rtamd.KERNEL_ACCEL)
    ctx.set_schedule(rtamd.SCHED_ROWS)
    ref = ctx.render(320, 180)
    ctx.set_schedule(sched)
    full = torch.empty((180, 320, 4), dtype=torch.float32, device="cuda")
    # dispatch 1 records tile work, 2-16 reuse its order with the counter-free kernel,
    # 17 records again (the order is re-derived every 16th dispatch)
    for i in range(18):
        full.fill_(float("nan"))
        torch.cuda.synchronize()  # the renderer's stream does not wait on torch's
        ctx.dispatch_rows(320, 180, 0, 1, 1, 180, full.data_ptr(), 320 * 16)
        ctx.sync()
        img = full.cpu().numpy()
        if not np.array_equal(img, ref):
            nan = int(np.isnan(img).any(-1).sum())
            bad = np.argwhere((img != ref).any(-1))
            pytest.fail(f"frame {i}: {len(bad)} pixels differ ({nan} unwritten), first {bad[:4].tolist()}, "
                        f"got {img[tuple(bad[0])].tolist()} want {ref[tuple(bad[0])].tolist()}")
    band = ctx.render(320, 180)[40:120]
    out = torch.zeros((80, 320, 4), dtype=torch.float32, device="cuda")
    for _ in range(2):  # alternate tile counts: the order sets must stay consistent
        ctx.dispatch_rows(320, 180, 40, 80, 1, 80, out.data_ptr(), 320 * 16)
        ctx.sync()
        assert np.array_equal(out.cpu().numpy(), band)
        assert np.array_equal(ctx.render(320, 180), ref)
    ctx.set_kernel(rtamd.KERNEL_AUTO)
    ctx.set_schedule(rtamd.SCHED_COST)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,W,H,mb", [(2, 400, 300, 1), (3, 640, 360, 3), (5, 320, 180, 3), (3, 3840, 2160, 3)])
def test_latency_mode_exact(ctx, cfg, W, H, mb):
    """rt_set_latency_mode: the split-walk instance without a queue and the heaviest tiles
    as four waves (or, on config 5, compaction as usual), and at 3840x2160 (129,600 tiles,
    over latency mode's 16 tiles per wave slot) the default mode's dispatch: every pixel
    equals the default mode's frame, frame after frame, and the oracle on a band."""
    fs = rtamd.generate(cfg, 0, W, H)
    ctx.upload(fs)
    ctx.set_params(W, H, mb, True)
    ctx.set_kernel(rtamd.KERNEL_ACCEL)
    try:
        ref = ctx.render(W, H)
        ctx.set_latency_mode(1)
        full = torch.empty((H, W, 4), dtype=torch.float32, device="cuda")
        for _ in range(10):
            full.fill_(float("nan"))
            torch.cuda.synchronize()  # the renderer's stream does not wait on torch's
            ctx.dispatch_rows(W, H, 0, 1, 1, H, full.data_ptr(), W * 16)
            ctx.sync()
            img = full.cpu().numpy()
            assert np.array_equal(img, ref), f"latency mode: {int((img != ref).any(axis=-1).sum())} px"
        y0 = H // 2
        o, _ = oracle.render(fs, W, H, oracle.params(W, H, mb), y0=y0, out_rows=8)
        check(img[y0:y0 + 8], o, "latency mode vs oracle")
    finally:
        ctx.set_latency_mode(0)
        ctx.set_kernel(rtamd.KERNEL_AUTO)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,W,H,mb", [(2, 400, 300, 1), (3, 320, 180, 3)])
def test_heaviest_slots_walk_per_lane_exact(ctx, cfg, W, H, mb):
    """rt_debug_lane_k: the heaviest dispatch slots walk their camera rays and / or
    their shadow rays per lane (LDS stacks even in an all-packet frame). Every pixel
    equals the row-major frame's, frame after frame."""
    fs = rtamd.generate(cfg, 0, W, H)
    ctx.upload(fs)
    ctx.set_params(W, H, mb, True)
    ctx.set_kernel(rtamd.KERNEL_ACCEL)
    try:
        ctx.set_schedule(rtamd.SCHED_ROWS)
        ref = ctx.render(W, H)
        ctx.set_schedule(rtamd.SCHED_COST)
        full = torch.empty((H, W, 4), dtype=torch.float32, device="cuda")
        for k, mode in [(64, 1), (64, 2), (10 ** 6, 3), (16, 2), (-1, 2), (0, 0)]:
            ctx.debug_lane_k(k, mode)
            for _ in range(10):
                full.fill_(float("nan"))
                torch.cuda.synchronize()  # the renderer's stream does not wait on torch's
                ctx.dispatch_rows(W, H, 0, 1, 1, H, full.data_ptr(), W * 16)
                ctx.sync()
                img = full.cpu().numpy()
                assert np.array_equal(img, ref), f"lane_k {k}:{mode}: {int((img != ref).any(axis=-1).sum())} px"
    finally:
        ctx.debug_lane_k(-1, 2)
        ctx.set_kernel(rtamd.KERNEL_AUTO)


@pytest.mark.gpu
def test_cost_order_ranks_by_wall_time(ctx):
    """The cost order (rt_debug_sched_order) is a permutation of the frame's tiles, and
    with the wall-time measure its head is the tiles that took longest: a tile whose
    camera rays all miss the root box (sky) costs next to nothing, so the first 16 are
    all tiles through the scene."""
    W, H = 320, 180
    fs = rtamd.generate(3, 0, W, H)
    ctx.upload(fs)
    ctx.set_params(W, H, 3, True)
    ctx.set_schedule(rtamd.SCHED_COST)
    ctx.debug_cost_time(1)
    try:
        img = None
        for _ in range(20):
            img = ctx.render(W, H)
        tx, ty = (W + 7) // 8, (H + 7) // 8
        order = ctx.debug_sched_order(tx * ty)
        assert sorted(order.tolist()) == list(range(tx * ty))
        # a background-only tile is constant along each of its rows (the gradient runs in y)
        sky_like = []
        for t in order[:16].tolist():
            y0, x0 = (t // tx) * 8, (t % tx) * 8
            blk = img[y0:y0 + 8, x0:x0 + 8, :3]
            sky_like.append(bool(np.all(blk == blk[:, :1, :])))  # constant along each row
        assert not any(sky_like), f"head tiles {order[:16].tolist()} include background-only tiles"
    finally:
        ctx.debug_cost_time(-1)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,W,H,mb", [(3, 320, 180, 3), (5, 320, 180, 3)])
def test_cost_measures_exact(ctx, cfg, W, H, mb):
    """rt_debug_cost_time: the cost order ranks tiles by their waves' wall time (the
    default) or by their lanes' node steps + tests. Either order, with and without
    latency mode (its split heavy tiles record the sum of their parts), frame after
    frame writes every pixel with the row-major frame's value."""
    fs = rtamd.generate(cfg, 0, W, H)
    ctx.upload(fs)
    ctx.set_params(W, H, mb, True)
    try:
        ctx.set_schedule(rtamd.SCHED_ROWS)
        ref = ctx.render(W, H)
        ctx.set_schedule(rtamd.SCHED_COST)
        full = torch.empty((H, W, 4), dtype=torch.float32, device="cuda")
        for cm in (0, 1, -1):
            for lat in (0, 1):
                ctx.debug_cost_time(cm)
                ctx.set_latency_mode(lat)
                for _ in range(12):
                    full.fill_(float("nan"))
                    torch.cuda.synchronize()  # the renderer's stream does not wait on torch's
                    ctx.dispatch_rows(W, H, 0, 1, 1, H, full.data_ptr(), W * 16)
                    ctx.sync()
                    img = full.cpu().numpy()
                    assert np.array_equal(img, ref), f"cost {cm} latency {lat}: {int((img != ref).any(axis=-1).sum())} px"
    finally:
        ctx.debug_cost_time(-1)
        ctx.set_latency_mode(0)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,W,H,mb", [(2, 400, 300, 1), (3, 320, 180, 3), (5, 320, 180, 3)])
def test_heavy_tiles_as_several_waves_exact(ctx, cfg, W, H, mb):
    """rt_debug_heavy: the heaviest tiles of the cost order run as 2/4/8/16/32 waves, one
    band of pixels each. Frame after frame (cost-recording dispatches included),
    every pixel is written (NaN-poisoned surface) with the row-major frame's value,
    also on a stripe set (a rank's rows) and with compaction (config 5 queues rays
    from the split waves)."""
    fs = rtamd.generate(cfg, 0, W, H)
    ctx.upload(fs)
    ctx.set_params(W, H, mb, True)
    ctx.set_kernel(rtamd.KERNEL_ACCEL)
    try:
        ctx.set_schedule(rtamd.SCHED_ROWS)
        ref = ctx.render(W, H)
        ctx.set_schedule(rtamd.SCHED_COST)
        full = torch.empty((H, W, 4), dtype=torch.float32, device="cuda")
        for k, parts in [(-1, 4), (16, 8), (64, 4), (10 ** 6, 2), (7, 8), (40, 16), (12, 32)]:
            ctx.debug_heavy(k, parts)
            for _ in range(10):
                full.fill_(float("nan"))
                torch.cuda.synchronize()  # the renderer's stream does not wait on torch's
                ctx.dispatch_rows(W, H, 0, 1, 1, H, full.data_ptr(), W * 16)
                ctx.sync()
                img = full.cpu().numpy()
                assert np.array_equal(img, ref), f"heavy {k}:{parts}: {int((img != ref).any(axis=-1).sum())} px"
        rows = sum(min(8, H - y) for y in range(8, H, 24))  # rank 1 of 3, 8-row stripes
        part = torch.empty((rows, W, 4), dtype=torch.float32, device="cuda")
        want = np.concatenate([ref[y:y + 8] for y in range(8, H, 24)])
        ctx.debug_heavy(32, 8)
        for _ in range(10):
            part.fill_(float("nan"))
            torch.cuda.synchronize()  # the renderer's stream does not wait on torch's
            ctx.dispatch_rows(W, H, 8, 8, 3, rows, part.data_ptr(), W * 16)
            ctx.sync()
            assert np.array_equal(part.cpu().numpy(), want)
    finally:
        ctx.debug_heavy(-1, 4)
        ctx.set_kernel(rtamd.KERNEL_AUTO)


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", [rtamd.KERNEL_ACCEL, rtamd.KERNEL_PACKET])
def test_obj_scene_parity(ctx, kernel):
    """A scene read from OBJ text (rts_parse_obj: a subdivided sphere-ish blob
    of quads and triangles, plus a floor) renders like the oracle."""
    lines, k = [], 12
    for i in range(k + 1):
        th = np.pi * i / k
        for j in range(2 * k):
            ph = np.pi * j / k
            lines.append(f"v {np.sin(th) * np.cos(ph) * 3:.6f} {np.cos(th) * 3:.6f} {np.sin(th) * np.sin(ph) * 3:.6f}")
    for i in range(k):
        for j in range(2 * k):
            a, b = i * 2 * k + j + 1, i * 2 * k + (j + 1) % (2 * k) + 1
            lines.append(f"f {a} {b} {b + 2 * k} {a + 2 * k}")
    sc = rtamd.Scene()
    assert sc.parse_obj("\n".join(lines), origin=(0, 0, -5), oriented=True) == 2 * k * 2 * k
    sc.add_plane((0, 1, 0), (0, 4, 0))
    sc.set_camera((6, -4, 10), 60, 4 / 3)
    sc.LookAt((0, 0, -5))
    sc.set_light((5, -10, 5), (1, 1, 1), 30)
    sc.buildBVH(15)
    fs = sc.serializeScene()
    W, H = 128, 96
    p = oracle.params(W, H, 3)
    ref, _ = oracle.render(fs, W, H, p)
    check(gpu_rows(ctx, fs, W, H, p, kernel=kernel), ref, f"obj kernel{kernel}")


# --------------------------------------------------------------------------
# Device-side animation (rt_set_animated / rt_animate): updateScene +
# updateBVH + serializeBVH (src/main.cpp:336-346, 981-992, 1068-1077) on the
# device, against oracle.update_bvh (the restated updateBVH) + oracle.render.

def _rotate(points, center, axis, angle):
    """Rodrigues rotation about `axis` through `center` (float64, then float32)."""
    a = np.asarray(axis, np.float64) / np.linalg.norm(axis)
    p = points.astype(np.float64) - center
    c, s = np.cos(angle), np.sin(angle)
    r = p * c + np.cross(a, p) * s + np.outer(p @ a, a) * (1 - c)
    return (r + center).astype(np.float32)


def _animation_steps(fs, ids, steps, renormal):
    """Yields successive records of shapes `ids`: spheres bounce on Y
    (bounceSphere, src/main.cpp:1079-1082), triangles turn about an axis
    (updateWheelAnimations :1084-1109, stored normals left as they were unless
    `renormal`), walls slide."""
    base = fs.shapes[ids].copy()
    for k in range(1, steps + 1):
        rec = base.copy()
        sph = rec["type"] == 0
        rec["sphereCenter"][sph, 1] = base["sphereCenter"][sph, 1] + np.float32(2 * np.sin(0.7 * k))
        tri = np.where(rec["type"] == 3)[0]
        if tri.size:
            cen = base["triP1"][tri].astype(np.float64).mean(0)
            for f in ("triP1", "triP2", "triP3"):
                rec[f][tri] = _rotate(base[f][tri], cen, (0.3, 0.2, 1.0), 0.35 * k)
            if renormal:
                e1 = rec["triP2"][tri].astype(np.float64) - rec["triP1"][tri]
                e2 = rec["triP3"][tri].astype(np.float64) - rec["triP1"][tri]
                n = np.cross(e1, e2)
                n /= np.linalg.norm(n, axis=1, keepdims=True)
                rec["planeNormal"][tri] = n.astype(np.float32)
                rec["planeD"][tri] = -(n * rec["triP1"][tri]).sum(1).astype(np.float32)
        wal = rec["type"] == 2
        rec["wallStart"][wal] = base["wallStart"][wal] + np.float32([1.5 * k, 0.0, -0.5 * k])
        yield rec


def _refit_case(ctx, fs, ids, steps, kernel, W=160, H=120, renormal=False, mutate=None):
    ref = rtamd.FlatScene(fs.shapes.copy(), fs.nodes.copy(), fs.indices, fs.camera, fs.light)
    ctx.upload(fs)
    ctx.set_params(W, H, 3, True)
    ctx.set_kernel(kernel)
    ctx.set_animated(ids)
    p = oracle.params(W, H, 3)
    for k, rec in enumerate(_animation_steps(fs, ids, steps, renormal)):
        if mutate is not None:
            mutate(k, rec)
        ref.shapes[ids] = rec
        oracle.update_bvh(ref, ids)
        ctx.animate(rec)
        got = ctx.read_nodes(len(ref.nodes))
        for f in ("boundsMin", "boundsMax"):
            assert np.array_equal(got[f], ref.nodes[f]), f"step {k}: {f} differs from updateBVH"
        for f in ("leftChild", "rightChild", "startShapeIdx", "numShapes"):
            assert np.array_equal(got[f], ref.nodes[f])
        img = ctx.render(W, H)
        want, _ = oracle.render(ref, W, H, p)
        check(img, want, f"refit step {k} kernel {kernel}")
    return ref


@pytest.mark.parametrize("kernel", [rtamd.KERNEL_ACCEL, rtamd.KERNEL_PACKET])
@pytest.mark.parametrize("depth", [1, 8])
def test_device_refit_matches_update_bvh(ctx, kernel, depth):
    fs = _soup(3, n_tri=1200)
    fs.nodes, fs.indices = oracle.build_bvh(fs.shapes, depth)
    types = fs.shapes["type"]
    ids = np.concatenate([np.where(types == 0)[0][:12], np.where(types == 3)[0][100:260],
                          np.where(types == 2)[0]]).astype(np.int32)
    _refit_case(ctx, fs, ids, 4, kernel)


def test_device_refit_moved_normals_and_far_moves(ctx):
    """Triangle normals recomputed (the back-face cones above them must give
    way) and a sphere thrown far outside the scene (its boxes grow past the
    scene's magnitude)."""
    fs = _soup(4, n_tri=1200)
    fs.nodes, fs.indices = oracle.build_bvh(fs.shapes, 6)
    types = fs.shapes["type"]
    ids = np.concatenate([np.where(types == 0)[0][:6], np.where(types == 3)[0][:300]]).astype(np.int32)

    def far(k, rec):
        if k == 2:
            rec["sphereCenter"][0] = (400.0, 30.0, -200.0)
    _refit_case(ctx, fs, ids, 4, rtamd.KERNEL_ACCEL, renormal=True, mutate=far)


def test_device_refit_class_change_rebuilds(ctx):
    """A triangle that collapses to a sliver (no conservative bound) and a
    sphere that becomes infinite: the host rebuild path, same frames."""
    fs = _soup(5, n_tri=800)
    fs.nodes, fs.indices = oracle.build_bvh(fs.shapes, 5)
    types = fs.shapes["type"]
    ids = np.concatenate([np.where(types == 0)[0][:4], np.where(types == 3)[0][:50]]).astype(np.int32)

    def degenerate(k, rec):
        if k >= 1:
            t = np.where(rec["type"] == 3)[0][1]  # [0] is one of _soup's slivers already
            rec["triP3"][t] = rec["triP1"][t] + (rec["triP2"][t] - rec["triP1"][t]) * np.float32(0.5)
        if k == 3:
            rec["sphereRadius"][0] = np.float32(np.inf)
    r0 = ctx.debug_anim_rebuilds()
    _refit_case(ctx, fs, ids, 4, rtamd.KERNEL_ACCEL, mutate=degenerate)
    assert ctx.debug_anim_rebuilds() - r0 == 2  # the sliver at step 1, the infinite sphere at step 3
    ctx.set_kernel(rtamd.KERNEL_AUTO)


def test_device_refit_equals_host_path(ctx):
    """The device refit and the reference's own host path (update_shapes +
    update_nodes with updateBVH's boxes) give the same frame."""
    W, H = 200, 150
    fs = _soup(6, n_tri=1000)
    fs.nodes, fs.indices = oracle.build_bvh(fs.shapes, 10)
    ids = np.where(fs.shapes["type"] == 0)[0].astype(np.int32)
    ref = _refit_case(ctx, fs, ids, 2, rtamd.KERNEL_AUTO, W, H)
    a = ctx.render(W, H)
    ctx.upload(fs)
    ctx.update_shapes(0, ref.shapes)
    ctx.update_nodes(ref.nodes)
    assert np.array_equal(ctx.render(W, H), a)
    with pytest.raises(rtamd.RTError):
        ctx.set_animated(np.array([0, 0], np.int32))  # duplicates
    with pytest.raises(rtamd.RTError):
        ctx.set_animated(np.array([len(fs.shapes)], np.int32))


@pytest.mark.parametrize("tail", [0, 1, 2, 3])
def test_ray_compaction_exact(ctx, tail):
    """rt_set_tail: bounces of the rays still alive run compacted in k_accel_tail;
    the frame is the uncompacted one bit for bit, across dispatches whose tile
    (and region) counts change, and the oracle's on a band."""
    W, H = 960, 540
    fs = rtamd.generate(3, 0, W, H)
    p = oracle.params(W, H, 3)
    ctx.set_tail(0)
    try:
        ref = gpu_rows(ctx, fs, W, H, p, kernel=rtamd.KERNEL_ACCEL)
        ctx.set_tail(tail)
        for _ in range(2):
            img = gpu_rows(ctx, fs, W, H, p, kernel=rtamd.KERNEL_ACCEL)
            assert np.array_equal(img, ref), f"tail {tail}: {int((img != ref).any(axis=-1).sum())} pixels differ"
            band = gpu_rows(ctx, fs, W, H, p, y0=200, rows=40, kernel=rtamd.KERNEL_ACCEL)  # fewer regions
            assert np.array_equal(band, ref[200:240])
        o, _ = oracle.render(fs, W, H, p, y0=256, out_rows=16)
        check(img[256:272], o, f"tail {tail} vs oracle")
        fs5 = rtamd.generate(5, 0, 640, 360)
        p5 = oracle.params(640, 360, 3)
        ctx.set_tail(0)
        a = gpu_rows(ctx, fs5, 640, 360, p5, kernel=rtamd.KERNEL_ACCEL)
        ctx.set_tail(tail)
        b = gpu_rows(ctx, fs5, 640, 360, p5, kernel=rtamd.KERNEL_ACCEL)
        assert np.array_equal(a, b)
    finally:
        ctx.set_tail(-1)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,W,H", [(3, 960, 540), (5, 640, 360)])
def test_split_walks_exact(ctx, cfg, W, H):
    """lane_walk_any: waves with few rays split each ray's walk over a group of idle
    lanes (compacted kernels, rt_set_tail). Every split setting renders the unsplit
    frame bit for bit: closest hits and shadows, the scene tree's overflow fallback
    to the reference tree (scene stack capped at 2), Moller-Trumbore, and the oracle
    on a band."""
    fs = rtamd.generate(cfg, 0, W, H)
    p = oracle.params(W, H, 3)
    try:
        ctx.set_tail(2)
        ctx.debug_split(0, 8)
        ref = gpu_rows(ctx, fs, W, H, p, kernel=rtamd.KERNEL_ACCEL)
        for mx, g in [(16, 8), (32, 16), (32, 2), (8, 64), (32, 64)]:
            ctx.debug_split(mx, g)
            img = gpu_rows(ctx, fs, W, H, p, kernel=rtamd.KERNEL_ACCEL)
            assert np.array_equal(img, ref), f"split {mx}:{g}: {int((img != ref).any(axis=-1).sum())} pixels differ"
        ctx.debug_scene_stack(2)
        img = gpu_rows(ctx, fs, W, H, p, kernel=rtamd.KERNEL_ACCEL)
        assert np.array_equal(img, ref), "split with scene-stack overflow"
        ctx.debug_scene_stack(0)
        ctx.set_tree(rtamd.TREE_REFERENCE)  # binary reference nodes in the shared part
        assert np.array_equal(gpu_rows(ctx, fs, W, H, p, kernel=rtamd.KERNEL_ACCEL), ref), "split, reference tree"
        ctx.set_tree(rtamd.TREE_SCENE)
        y0 = H // 2
        o, _ = oracle.render(fs, W, H, p, y0=y0, out_rows=8)
        check(img[y0:y0 + 8], o, "split vs oracle")
        if cfg == 3:  # Moller-Trumbore (its own accelerator, settings inherited)
            pm = oracle.params(W, H, 3, useMT=True)
            ctx.debug_split(0, 8)
            mref = gpu_rows(ctx, fs, W, H, pm, kernel=rtamd.KERNEL_ACCEL)
            ctx.debug_split(32, 16)
            assert np.array_equal(gpu_rows(ctx, fs, W, H, pm, kernel=rtamd.KERNEL_ACCEL), mref)
    finally:
        ctx.debug_split(16, 8)
        ctx.debug_scene_stack(0)
        ctx.set_tree(rtamd.TREE_SCENE)
        ctx.set_tail(-1)


def test_alternating_dispatches_stay_exact(ctx):
    """State carried between dispatches (cost order sets, counter-free dispatches,
    compaction counters by parity and region count) across changing dispatch
    shapes, scenes and compaction settings: every frame equals its first render."""
    shapes = [(640, 360, 0, None), (640, 360, 96, 64), (320, 180, 0, None), (640, 360, 8, 200)]
    refs = {}
    for it in range(3):
        for cfg in (5, 3):
            fs = rtamd.generate(cfg, 0, 640, 360)
            for k, (W, H, y0, rows) in enumerate(shapes):
                for tail in (-1, 2, 0):
                    ctx.set_tail(tail)
                    p = oracle.params(W, H, 3)
                    img = gpu_rows(ctx, fs, W, H, p, y0=y0, rows=rows, kernel=rtamd.KERNEL_ACCEL)
                    key = (cfg, k)
                    if key not in refs:
                        refs[key] = img
                    bad = int((img != refs[key]).any(axis=-1).sum())
                    assert bad == 0, f"iteration {it} config {cfg} shape {k} tail {tail}: {bad} pixels differ"
    ctx.set_tail(-1)


@pytest.mark.parametrize("cfg", [3, 2])
def test_animated_scene_tree_equals_reference_tree(ctx, cfg):
    """Animated scenes keep the scene tree (rt_animate refits its boxes, items and,
    for unbounded shapes, opens its kNoPrune part): full frames after each refit
    equal the reference-tree walk bit for bit, and the oracle on a band. Config 3:
    the four wheels turn (updateWheelAnimations, src/main.cpp:1084-1109); config 2:
    its spheres bounce (bounceSphere, :1079-1082) and the floor wall slides."""
    W, H = (1920, 1080) if cfg == 3 else (800, 600)
    fs = rtamd.generate(cfg, 0, W, H)
    if cfg == 3:
        ids = np.arange(3380, 3380 + 640, dtype=np.int32)
    else:
        types = fs.shapes["type"]
        ids = np.concatenate([np.where(types == 0)[0][:8], np.where(types == 2)[0]]).astype(np.int32)
    ref = rtamd.FlatScene(fs.shapes.copy(), fs.nodes.copy(), fs.indices, fs.camera, fs.light)
    ctx.upload(fs)
    mb = CFG_BOUNCES[cfg]
    ctx.set_params(W, H, mb, True)
    ctx.set_kernel(rtamd.KERNEL_AUTO)
    ctx.set_animated(ids)
    assert ctx.accel_info()["scene_tree"] == 1
    out = torch.empty((H, W, 4), dtype=torch.float32, device="cuda")
    for k, rec in enumerate(_animation_steps(fs, ids, 3, renormal=False)):
        ref.shapes[ids] = rec
        oracle.update_bvh(ref, ids)
        ctx.animate(rec)
        frames = []
        for tree in (rtamd.TREE_SCENE, rtamd.TREE_REFERENCE):
            ctx.set_tree(tree)
            torch.cuda.synchronize()
            ctx.dispatch_rows(W, H, 0, 1, 1, H, out.data_ptr(), W * 16)
            ctx.sync()
            frames.append(out.cpu().numpy())
        ctx.set_tree(rtamd.TREE_SCENE)
        assert np.array_equal(frames[0], frames[1]), f"step {k}"
        y0 = H // 2 - 8
        want, _ = oracle.render(ref, W, H, oracle.params(W, H, mb), y0=y0, out_rows=16)
        check(frames[0][y0:y0 + 16], want, f"animated step {k}")
    assert ctx.debug_anim_rebuilds() >= 0
