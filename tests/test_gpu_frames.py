"""Whole-frame and multi-GPU-path parity on the GPU (-m gpu; needs an MI355X).

* Full frames of configs 2, 3 and 5 at their BASELINE sizes against the
  OpenMP oracle (not bands): every pixel within 1e-4 per channel.
* Camera diversity on the production kernel: the weak bench mode's orbit
  cameras, a camera inside the car's body, grazing views along the road,
  and axis-aligned views whose centre rays have exactly-zero direction
  components (the slab test's inf/NaN path, gpu_shader.comp:364-377).
* Config 4 (3840x2160): oracle bands at the top, through the car and at the
  bottom for the accelerated and the packet kernel; the 8-rank stripe set
  reassembled by rt_group (copy transport on one GPU) equals the single
  dispatch bit for bit; the 1-rank RCCL group (ncclCommInitRank) equals it too.
* Root shares (rt_group_set_root_share): rank 0 taking 2-64 stripes per period
  reassembles to the single dispatch for 2-8 copy-transport ranks.
* tests/native/group_check: a C++ host that links librtamd.so through the C
  ABI alone and checks every group case bit for bit (1080p-class and 4K).

Tolerance 1e-4 per channel (BASELINE.json north_star); measured 0.
"""
import os
import subprocess

import numpy as np
import pytest
import torch

import oracle
import rtamd

pytestmark = pytest.mark.gpu
TOL = 1e-4
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def ctx():
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


def render(ctx, fs, W, H, mb, kernel=rtamd.KERNEL_AUTO, y0=0, rows=None):
    rows = H - y0 if rows is None else rows
    ctx.upload(fs)
    ctx.set_params(W, H, mb, True, False, False)
    ctx.set_kernel(kernel)
    out = torch.full((rows, W, 4), -7.0, dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    ctx.dispatch_rows(W, H, y0, 1, 1, rows, out.data_ptr(), W * 16)
    ctx.sync()
    return out.cpu().numpy()


# --------------------------------------------------------------------------
# Full frames against the oracle

@pytest.mark.parametrize("cfg,W,H,mb", [(2, 800, 600, 1), (3, 1920, 1080, 3), (5, 1920, 1080, 3)],
                         ids=["config2_800x600", "config3_1920x1080", "config5_1920x1080"])
def test_full_frame_vs_oracle(ctx, cfg, W, H, mb):
    fs = rtamd.generate(cfg, 0, W, H)
    img = render(ctx, fs, W, H, mb)
    assert ctx.accel_info()["last_kernel"] == rtamd.KERNEL_ACCEL
    ref, _ = oracle.render(fs, W, H, oracle.params(W, H, mb))
    check(img, ref, f"config {cfg} full frame")


# --------------------------------------------------------------------------
# Camera diversity (production kernel vs oracle, reduced size)

def _camera_scene(cfg, W, H, pos=None, target=None, orbit=None, basis=None):
    sc = rtamd.Scene().generate(cfg, 0, W / H)
    if orbit is not None:
        sc.orbit(orbit[0], orbit[1])
    if pos is not None and target is not None:
        sc.set_camera(pos, 60.0, W / H)
        sc.LookAt(target)
    fs = sc.serializeScene()
    if basis is not None:
        # an exact axis-aligned camera record (LookAt's trigonometry leaves ~1e-8 residues)
        front, up, right = basis
        fs.camera["Position"] = pos
        fs.camera["Front"] = front
        fs.camera["Up"] = up
        fs.camera["Right"] = right
    return fs


CAMERAS = {
    # weak-mode orbit frames (bench.py: rank r turns r degrees about the look-at point)
    "orbit1_car": (3, dict(orbit=((0.0, 0.0, 0.0), 1.0))),
    "orbit7_car": (3, dict(orbit=((0.0, 0.0, 0.0), 7.0))),
    "orbit3_monkey": (2, dict(orbit=((0.0, 10.0, -8.0), 3.0))),
    "orbit5_random": (5, dict(orbit=((0.0, 0.0, 0.0), 5.0))),
    # inside the car body (ellipsoid about (0,-3.4,0)), looking along +x and back at the cabin
    "inside_car": (3, dict(pos=(0.0, -3.4, 0.0), target=(10.0, -3.0, 1.0))),
    "inside_car_up": (3, dict(pos=(1.0, -3.0, 0.5), target=(1.5, -9.0, 0.2))),
    # grazing views along the road plane y = 0 (just above it: y is down)
    "grazing_road": (3, dict(pos=(0.0, -0.05, 45.0), target=(0.0, -0.02, 0.0))),
    "grazing_road_side": (3, dict(pos=(60.0, -0.2, 3.0), target=(-10.0, -0.1, -2.0))),
    # axis-aligned: front exactly -z / -x, so the centre column/row rays have zero components
    "axis_minus_z": (3, dict(pos=(0.0, -2.0, 40.0), basis=((0, 0, -1), (0, 1, 0), (1, 0, 0)))),
    "axis_minus_x": (3, dict(pos=(60.0, -2.0, 0.0), basis=((-1, 0, 0), (0, 1, 0), (0, 0, -1)))),
    "axis_random_cloud": (5, dict(pos=(0.0, 0.0, 60.0), basis=((0, 0, -1), (0, 1, 0), (1, 0, 0)))),
    "axis_down_car": (3, dict(pos=(0.0, -30.0, 0.0), basis=((0, 1, 0), (0, 0, -1), (1, 0, 0)))),
}


@pytest.mark.parametrize("name", sorted(CAMERAS))
def test_camera_vs_oracle(ctx, name):
    cfg, kw = CAMERAS[name]
    W, H = 480, 270  # even: the centre column/row have NDC exactly 0
    fs = _camera_scene(cfg, W, H, **kw)
    mb = 3
    img = render(ctx, fs, W, H, mb)
    ref, _ = oracle.render(fs, W, H, oracle.params(W, H, mb))
    check(img, ref, name)
    if name.startswith("axis"):
        _, d = oracle.get_ray(fs.camera, 0.0, 0.0)
        assert (d == 0).sum() == 2, d  # the centre ray runs along an axis: two zero components


# --------------------------------------------------------------------------
# Config 4: 3840x2160

W4, H4 = 3840, 2160
BANDS4 = {"top": (0, 16), "car": (1040, 24), "bottom": (2144, 16)}


@pytest.fixture(scope="module")
def car4k():
    return rtamd.generate(3, 0, W4, H4)


@pytest.mark.parametrize("kernel", [rtamd.KERNEL_ACCEL, rtamd.KERNEL_PACKET], ids=["accel", "packet"])
@pytest.mark.parametrize("band", sorted(BANDS4))
def test_config4_bands_vs_oracle(ctx, car4k, band, kernel):
    y0, rows = BANDS4[band]
    img = render(ctx, car4k, W4, H4, 3, kernel, y0, rows)
    ref, _ = oracle.render(car4k, W4, H4, oracle.params(W4, H4, 3), y0=y0, out_rows=rows)
    check(img, ref, f"4K {band}")
    if band == "car":
        assert (np.abs(img[..., :3] - img[:1, :1, :3]) > 0).any()  # the band really crosses the scene


@pytest.fixture(scope="module")
def frame4k(ctx, car4k):
    return render(ctx, car4k, W4, H4, 3)


@pytest.mark.parametrize("kernel", [rtamd.KERNEL_AUTO, rtamd.KERNEL_PACKET], ids=["auto", "packet"])
def test_config4_group_of_8_reassembles(frame4k, car4k, kernel):
    """The 8-GPU plan of config 4 (8-row stripes, rank r = stripes r, r+8, ...),
    run as 8 group members on this GPU: the gathered frame is the single dispatch."""
    g = rtamd.Group([0] * 8, rtamd.GATHER_COPY)
    try:
        assert (g.nranks, g.nlocal, g.transport) == (8, 8, rtamd.GATHER_COPY)
        g.upload(car4k)
        g.set_params(W4, H4, 3)
        for m in g.members:
            m.set_kernel(kernel)
        for _ in range(2):
            img = g.render(W4, H4, 8)
            assert np.array_equal(img, frame4k)
        with pytest.raises(rtamd.RTError):
            g.read_image(W4, H4 - 8)  # a short destination is refused
    finally:
        g.close()


@pytest.mark.parametrize("ranks,share,stripe", [(2, 2, 8), (3, 2, 8), (4, 2, 8), (8, 2, 8), (2, 3, 5), (5, 1, 7),
                                                (8, 3, 3), (3, 64, 1)])
def test_group_root_share_reassembles(ctx, ranks, share, stripe):
    """rt_group_set_root_share: rank 0 renders `share` stripes of every period of
    share + P - 1 (straight into its staging), the others one each; the gathered
    frame is the single dispatch bit for bit, also when the share changes between
    frames (buffers resize) and for heights that end inside a period."""
    W, H = 480, 270
    fs = rtamd.generate(3, 0, W, H)
    ref = render(ctx, fs, W, H, 3)
    g = rtamd.Group([0] * ranks, rtamd.GATHER_COPY)
    try:
        g.upload(fs)
        g.set_params(W, H, 3)
        for k in (share, 1, share):
            g.set_root_share(k)
            assert np.array_equal(g.render(W, H, stripe), ref), f"share {k}"
            st = g.collect_stats(W, H, stripe)
            assert st["pixels"] == W * H  # the members' rows cover the frame once
    finally:
        g.close()


def test_rccl_rank_group_root_share(ctx):
    """A 1-rank RCCL group at root share 2: rank 0 owns every row (nothing to send)."""
    W, H = 640, 360
    fs = rtamd.generate(3, 0, W, H)
    ref = render(ctx, fs, W, H, 3)
    g = rtamd.Group(uid=rtamd.group_unique_id(), nranks=1, rank=0, device=0)
    try:
        g.upload(fs)
        g.set_params(W, H, 3)
        g.set_root_share(2)
        for _ in range(2):
            assert np.array_equal(g.render(W, H, 8), ref)
        with pytest.raises(rtamd.RTError):
            g.set_root_share(0)
    finally:
        g.close()


def test_rccl_rank_group_equals_single_dispatch(ctx):
    """rt_group_create_rank with one rank: ncclCommInitRank + unstripe."""
    W, H = 640, 360
    fs = rtamd.generate(3, 0, W, H)
    ref = render(ctx, fs, W, H, 3)
    g = rtamd.Group(uid=rtamd.group_unique_id(), nranks=1, rank=0, device=0)
    try:
        assert g.transport == rtamd.GATHER_RCCL
        g.upload(fs)
        g.set_params(W, H, 3)
        for _ in range(3):
            img = g.render(W, H, 8)
            assert np.array_equal(img, ref)
    finally:
        g.close()


@pytest.mark.parametrize("args", [["480", "270", "3"], ["800", "600", "2", "6"], ["3840", "2160", "3", "8"]],
                         ids=["car_480x270", "monkey_800x600", "car_3840x2160_8ranks"])
def test_native_group_host(args):
    """C++ host through the C ABI only (tests/native/group_check.cpp)."""
    exe = os.path.join(ROOT, "tests", "native", "build", "group_check")
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "native")], check=True)
    r = subprocess.run([exe] + args, capture_output=True, text=True, timeout=100)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK" in r.stdout.splitlines()[-1]


# --------------------------------------------------------------------------
# The brute-force branch (useBVH = 0, gpu_shader.comp:523-620) on the accelerator

def render_p(ctx, fs, W, H, mb, bvh, kernel, y0=0, rows=None, fresnel=False):
    rows = H - y0 if rows is None else rows
    ctx.upload(fs)
    ctx.set_params(W, H, mb, bvh, fresnel, False)
    ctx.set_kernel(kernel)
    out = torch.full((rows, W, 4), -7.0, dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    ctx.dispatch_rows(W, H, y0, 1, 1, rows, out.data_ptr(), W * 16)
    ctx.sync()
    return out.cpu().numpy()


@pytest.mark.parametrize("cfg,W,H,mb,fresnel", [(2, 800, 600, 1, False), (2, 400, 300, 4, True),
                                                (3, 1920, 1080, 3, False), (5, 240, 136, 3, False)],
                         ids=["config2", "config2_fresnel_b4", "config3_1080p", "config5_240x136"])
def test_brute_branch_accelerated_equals_scan(ctx, cfg, W, H, mb, fresnel):
    """useBVH = 0 through the accelerated one-leaf context equals the literal
    brute scan (k_packet) bit for bit, frame after frame."""
    fs = rtamd.generate(cfg, 0, W, H)
    scan = render_p(ctx, fs, W, H, mb, False, rtamd.KERNEL_PACKET, fresnel=fresnel)
    assert ctx.accel_info()["last_kernel"] == rtamd.KERNEL_PACKET
    ctx.kernel_times()
    for _ in range(2):
        fast = render_p(ctx, fs, W, H, mb, False, rtamd.KERNEL_AUTO, fresnel=fresnel)
        assert ctx.accel_info()["last_kernel"] == rtamd.KERNEL_ACCEL
        assert np.array_equal(fast, scan)
    assert len(ctx.kernel_times()) == 2  # timed on the context's own events


def test_brute_branch_vs_oracle_band(ctx):
    W, H = 1920, 1080
    fs = rtamd.generate(3, 0, W, H)
    img = render_p(ctx, fs, W, H, 3, False, rtamd.KERNEL_AUTO, 520, 16)
    ref, _ = oracle.render(fs, W, H, oracle.params(W, H, 3, False), y0=520, out_rows=16)
    check(img, ref, "brute band")


def test_brute_branch_follows_shape_updates(ctx):
    """rt_update_shapes rebuilds the brute context's copy before the next brute frame."""
    W, H = 320, 180
    fs = rtamd.generate(3, 0, W, H)
    render_p(ctx, fs, W, H, 3, False, rtamd.KERNEL_AUTO)
    moved = fs.shapes[-100:].copy()
    moved["sphereCenter"] += np.float32(2.5)
    ctx.update_shapes(len(fs.shapes) - 100, moved)
    out = torch.empty((H, W, 4), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    ctx.dispatch_rows(W, H, 0, 1, 1, H, out.data_ptr(), W * 16)
    ctx.sync()
    fs2 = rtamd.FlatScene(np.concatenate([fs.shapes[:-100], moved]), fs.nodes, fs.indices, fs.camera, fs.light)
    ref, _ = oracle.render(fs2, W, H, oracle.params(W, H, 3, False))
    check(out.cpu().numpy(), ref, "brute after update_shapes")


# --------------------------------------------------------------------------
# Moller-Trumbore frames (useMollerTrumbore = 1) on the MT accelerator

def render_mt(ctx, fs, W, H, mb, bvh, kernel, y0=0, rows=None, fresnel=False):
    rows = H - y0 if rows is None else rows
    ctx.upload(fs)
    ctx.set_params(W, H, mb, bvh, fresnel, True)
    ctx.set_kernel(kernel)
    out = torch.full((rows, W, 4), -7.0, dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    ctx.dispatch_rows(W, H, y0, 1, 1, rows, out.data_ptr(), W * 16)
    ctx.sync()
    return out.cpu().numpy()


@pytest.mark.parametrize("cfg,W,H,mb,bvh,fresnel", [(2, 800, 600, 1, True, False), (2, 400, 300, 4, True, True),
                                                    (3, 1920, 1080, 3, True, False), (5, 240, 136, 3, True, False),
                                                    (2, 200, 150, 3, False, False), (3, 240, 136, 3, False, True)],
                         ids=["config2", "config2_fresnel_b4", "config3_1080p", "config5_240x136",
                              "config2_brute", "config3_brute_fresnel"])
def test_mt_accelerated_equals_literal(ctx, cfg, W, H, mb, bvh, fresnel):
    """useMollerTrumbore = 1 through the MT accelerator (and, for useBVH = 0, the
    one-leaf tree's MT accelerator) equals the literal k_packet walk bit for bit."""
    fs = rtamd.generate(cfg, 0, W, H)
    lit = render_mt(ctx, fs, W, H, mb, bvh, rtamd.KERNEL_PACKET, fresnel=fresnel)
    for _ in range(2):
        fast = render_mt(ctx, fs, W, H, mb, bvh, rtamd.KERNEL_AUTO, fresnel=fresnel)
        assert ctx.accel_info()["last_kernel"] == rtamd.KERNEL_ACCEL
        assert np.array_equal(fast, lit)


@pytest.mark.parametrize("k,parts", [(16, 8), (64, 4), (8, 2)])
def test_mt_heavy_tiles_split_equals_literal(ctx, k, parts):
    """MT frames over the car's shallow tree walk every bounce as packets, so the
    heavy-tile split (the heaviest k tiles of the cost order as `parts` waves, here
    forced with rt_debug_heavy) applies to them: frames after the first (cost order
    in place, tiles split) equal the literal k_packet MT frame bit for bit."""
    W, H = 800, 600
    fs = rtamd.generate(3, 0, W, H)
    lit = render_mt(ctx, fs, W, H, 3, True, rtamd.KERNEL_PACKET)
    ctx.debug_heavy(k, parts)
    try:
        ctx.upload(fs)
        ctx.set_params(W, H, 3, True, False, True)
        ctx.set_kernel(rtamd.KERNEL_AUTO)
        for i in range(3):
            out = torch.full((H, W, 4), float("nan"), dtype=torch.float32, device="cuda")
            torch.cuda.synchronize()
            ctx.dispatch_rows(W, H, 0, 1, 1, H, out.data_ptr(), W * 16)
            ctx.sync()
            assert ctx.accel_info()["last_kernel"] == rtamd.KERNEL_ACCEL
            assert np.array_equal(out.cpu().numpy(), lit), f"frame {i}"
    finally:
        ctx.debug_heavy(-1, 4)


def test_mt_vs_oracle_band(ctx):
    W, H = 1920, 1080
    fs = rtamd.generate(3, 0, W, H)
    img = render_mt(ctx, fs, W, H, 3, True, rtamd.KERNEL_AUTO, 520, 16)
    ref, _ = oracle.render(fs, W, H, oracle.params(W, H, 3, True, False, True), y0=520, out_rows=16)
    check(img, ref, "MT band")


@pytest.mark.parametrize("name", ["grazing_road", "axis_minus_z", "inside_car", "orbit7_car"])
def test_mt_cameras_vs_oracle(ctx, name):
    cfg, kw = CAMERAS[name]
    W, H = 480, 270
    fs = _camera_scene(cfg, W, H, **kw)
    img = render_mt(ctx, fs, W, H, 3, True, rtamd.KERNEL_AUTO)
    ref, _ = oracle.render(fs, W, H, oracle.params(W, H, 3, True, False, True))
    check(img, ref, name)


def test_rgb_format_equals_rgba(ctx):
    """rt_dispatch_rows_fmt(RT_FORMAT_RGB32F): packed 12-byte pixels equal the RGBA
    image's RGB (alpha is always 1); a pitch below 12*W is refused."""
    W, H = 1920, 1080
    fs = rtamd.generate(3, 0, W, H)
    rgba = render(ctx, fs, W, H, 3)
    y0, rows = 400, 136
    out = torch.full((rows, W * 3), -7.0, dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    ctx.dispatch_rows_rgb(W, H, y0, 8, 1, rows, out.data_ptr(), W * 12)
    ctx.sync()
    got = out.cpu().numpy().reshape(rows, W, 3)
    assert np.array_equal(got, rgba[y0:y0 + rows, :, :3])
    assert (rgba[..., 3] == 1).all()
    with pytest.raises(rtamd.RTError):
        ctx.dispatch_rows_rgb(W, H, y0, 8, 1, rows, out.data_ptr(), W * 12 - 4)


@pytest.mark.parametrize("y0,stripe,period,rows", [(0, 16, 24, 720), (8, 8, 64, 136), (0, 1080, 1080, 1080)],
                         ids=["root_share2_of_3", "rank1_of_8", "all_rows"])
def test_image_rows_format_writes_in_place(ctx, y0, stripe, period, rows):
    """RT_FORMAT_RGBA32F_IMAGE (rt_group's rank 0): each rendered row lands at its
    image row of a whole W x H surface, equal to the single dispatch there, and every
    other row keeps what was in it."""
    W, H = 1920, 1080
    fs = rtamd.generate(3, 0, W, H)
    rgba = render(ctx, fs, W, H, 3)
    out = torch.full((H, W, 4), -7.0, dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    ctx.dispatch_rows_ex(W, H, y0, stripe, period, rows, out.data_ptr(), W * 16, fmt=rtamd.FORMAT_RGBA32F_IMAGE)
    ctx.sync()
    got = out.cpu().numpy()
    mine = np.array([y0 + (r // stripe) * period + r % stripe for r in range(rows)])
    mine = mine[mine < H]
    assert np.array_equal(got[mine], rgba[mine])
    rest = np.setdiff1d(np.arange(H), mine)
    assert (got[rest] == -7.0).all()
    with pytest.raises(rtamd.RTError):  # the pitch must hold 16 B per pixel
        ctx.dispatch_rows_ex(W, H, y0, stripe, period, rows, out.data_ptr(), W * 12,
                             fmt=rtamd.FORMAT_RGBA32F_IMAGE)


# --------------------------------------------------------------------------
# The reference's default scene (SCENE = 3, generateScene3, src/main.cpp:1196-1229)

@pytest.mark.parametrize("mt", [0, 1], ids=["barycentric", "moller_trumbore"])
@pytest.mark.parametrize("bvh", [1, 0], ids=["bvh_branch", "brute_branch"])
@pytest.mark.parametrize("kernel", [rtamd.KERNEL_AUTO, rtamd.KERNEL_PACKET], ids=["auto", "packet"])
def test_default_scene3_vs_oracle(ctx, bvh, mt, kernel):
    """One triangle and no tree (N = 0, I = 0): the brute branch renders the
    triangle, the BVH branch (which the GLSL starts at bvhNodes[-1]) sees nothing.
    Whole 800x600 frames, 3 bounces, Fresnel off and on."""
    W, H = 800, 600
    fs = rtamd.generate(6, 0, W, H)
    assert len(fs.nodes) == 0 and len(fs.indices) == 0 and len(fs.shapes) == 1
    ctx.upload(fs)
    ctx.set_kernel(kernel)
    try:
        for fres in (0, 1):
            ctx.set_params(W, H, 3, bool(bvh), bool(fres), bool(mt))
            out = torch.full((H, W, 4), -7.0, dtype=torch.float32, device="cuda")
            torch.cuda.synchronize()
            ctx.dispatch_rows(W, H, 0, 1, 1, H, out.data_ptr(), W * 16)
            ctx.sync()
            img = out.cpu().numpy()
            ref, _ = oracle.render(fs, W, H, oracle.params(W, H, 3, bvh, fres, mt))
            check(img, ref, f"scene 3 bvh={bvh} mt={mt} fresnel={fres}")
            bg, _ = oracle.render(fs, W, H, oracle.params(W, H, 3, 1))
            lit = int((img != bg).any(axis=-1).sum())
            assert (lit == 0) if bvh else (lit > 1000), lit
    finally:
        ctx.set_kernel(rtamd.KERNEL_AUTO)


# --------------------------------------------------------------------------
# The bench's steady state, frame by frame (bench.py frames mode)

@pytest.fixture(scope="module")
def car_full_ref():
    W, H = 1920, 1080
    fs = rtamd.generate(3, 0, W, H)
    ref, _ = oracle.render(fs, W, H, oracle.params(W, H, 3))
    return fs, ref


def test_bench_steady_state_frames_vs_oracle(car_full_ref):
    """What bench.py times: F contexts on their own streams (F = the bench's own
    plan, 3 at 1080p), frames dealt round-robin with nothing waited on between
    them, the cost-ordered schedule (re-derived every 16th dispatch; the dispatches
    between run the counter-free instance with the auto lane_k slots), 1920x1080,
    depth 3, on 2F hardware queues (tests/conftest.py raises GPU_MAX_HW_QUEUES
    before the runtime starts, as bench.py does). Each of the 24 frames goes to its
    own buffer and every one is checked against one full-frame oracle render
    (gpu_shader.comp:433-624)."""
    import bench
    fs, ref = car_full_ref
    W, H, n = 1920, 1080, 24
    F, _ = bench.plan_inflight(0, W, H, 1, False, False, "4")
    assert F == 3
    assert int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) >= 2 * F
    streams = [torch.cuda.Stream() for _ in range(F)]
    ctxs = []
    try:
        for st in streams:
            c = rtamd.ComputeShader(0)
            c.set_stream(st.cuda_stream)
            c.upload(fs)
            c.set_params(W, H, 3, True, False, False)
            c.set_schedule(rtamd.SCHED_COST)
            ctxs.append(c)
        outs = [torch.full((H, W, 4), -7.0, dtype=torch.float32, device="cuda") for _ in range(n)]
        torch.cuda.synchronize()
        for i in range(n):
            c = ctxs[i % F]
            c.set_camera(fs.camera)
            c.set_light(fs.light)
            c.dispatch_rows(W, H, 0, 1, 1, H, outs[i].data_ptr(), W * 16)
        torch.cuda.synchronize()
        assert all(c.accel_info()["last_kernel"] == rtamd.KERNEL_ACCEL for c in ctxs)
        for i, o in enumerate(outs):
            check(o.cpu().numpy(), ref, f"steady-state frame {i} (context {i % F})")
    finally:
        for c in ctxs:
            c.close()


# --------------------------------------------------------------------------
# rt_group frames in flight (rt_group_set_frames): one communicator, F slots

def _orbit_cameras(W, H, n):
    cams = []
    for d in range(n):
        sc = rtamd.Scene().generate(3, 0, W / H)
        sc.orbit((0.0, 0.0, 0.0), 3.0 * d)
        cams.append(sc.serializeScene().camera)
    return cams


def _in_flight_check(ctx, g, fs, W, H, stripe):
    """Frames with a different camera each, dispatched back to back with nothing
    waited on: for every prefix length n the last frame (read_image) equals the
    single dispatch of its camera, so no slot's buffers leak into another's."""
    cams = _orbit_cameras(W, H, 5)
    refs = []
    for c in cams:
        ctx.upload(rtamd.FlatScene(fs.shapes, fs.nodes, fs.indices, c, fs.light))
        ctx.set_params(W, H, 3, True, False, False)
        ctx.set_kernel(rtamd.KERNEL_AUTO)
        out = torch.full((H, W, 4), -7.0, dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        ctx.dispatch_rows(W, H, 0, 1, 1, H, out.data_ptr(), W * 16)
        ctx.sync()
        refs.append(out.cpu().numpy())
    assert not np.array_equal(refs[0], refs[1])
    g.upload(fs)
    g.set_params(W, H, 3)
    for n in range(1, 2 * g.frames + 2):
        for i in range(n):
            g.set_camera(cams[i % len(cams)])
            g.dispatch(W, H, stripe)
        img = g.read_image(W, H)
        assert np.array_equal(img, refs[(n - 1) % len(cams)]), f"{n} frames in flight"


@pytest.mark.parametrize("ranks,frames,share", [(8, 3, 1), (4, 8, 2), (2, 2, 1), (8, 8, 1), (8, 8, 2)])
def test_group_frames_in_flight_copy(ctx, ranks, frames, share):
    W, H = 480, 270
    fs = rtamd.generate(3, 0, W, H)
    g = rtamd.Group([0] * ranks, rtamd.GATHER_COPY, frames=frames)
    try:
        assert g.frames == frames and len(g.contexts) == ranks * frames and len(g.members) == ranks
        g.set_root_share(share)
        _in_flight_check(ctx, g, fs, W, H, 8)
        ph = g.phase_times()
        assert ph["frames"] > 0 and ph["render_ms"] > 0 and ph["fanin_ms"] > 0 and ph["unstripe_ms"] > 0
        assert ph["frame_ms"] >= ph["render_ms"]
        with pytest.raises(rtamd.RTError):
            g._chk(g._lib.rt_group_set_frames(g._h, 2), "rt_group_set_frames")  # only before the upload
    finally:
        g.close()


def test_rccl_rank_group_frames_in_flight(ctx):
    """One RCCL rank (ncclCommInitRank) with 4 frame slots on one communicator;
    the bounded sync and the asynchronous-error poll report success."""
    W, H = 640, 360
    fs = rtamd.generate(3, 0, W, H)
    g = rtamd.Group(uid=rtamd.group_unique_id(), nranks=1, rank=0, device=0, frames=4)
    try:
        assert g.transport == rtamd.GATHER_RCCL and g.frames == 4
        g.set_timeout(30000)
        _in_flight_check(ctx, g, fs, W, H, 8)
        g.check()
        g.sync()
        ph = g.phase_times()
        # one rank renders the single-GPU frame straight into its surface: no fan-in, no scatter
        assert ph["frames"] > 0 and ph["render_ms"] > 0 and ph["unstripe_ms"] == 0 and ph["fanin_ms"] == 0
    finally:
        g.close()


def test_host_render_loop_frames(ctx):
    """librthost.so rth_render_loop (the reference's render loop, src/main.cpp:290-462, as
    a C++ host over the C ABI): waited and back-to-back frames, cameras cycling, leave
    the last camera's frame; one time per waited frame."""
    W, H = 640, 360
    fs = rtamd.generate(3, 0, W, H)
    cams = np.concatenate([_orbit_cameras(W, H, 3)[k] for k in (1, 2)])
    refs = []
    for c in cams:
        ctx.upload(rtamd.FlatScene(fs.shapes, fs.nodes, fs.indices, c, fs.light))
        ctx.set_params(W, H, 3)
        refs.append(ctx.render(W, H))
    ctx.upload(fs)
    ctx.set_params(W, H, 3)
    out = torch.full((H, W, 4), -7.0, dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    ms = rtamd.render_loop(ctx, cams, fs.light, W, H, out.data_ptr(), W * 16, 5, True)
    assert ms.shape == (5,) and (ms > 0).all()
    assert np.array_equal(out.cpu().numpy(), refs[0])  # frame 4 took cams[4 % 2]
    ms = rtamd.render_loop(ctx, cams, fs.light, W, H, out.data_ptr(), W * 16, 6, False)
    assert ms.shape == (1,) and ms[0] > 0
    assert np.array_equal(out.cpu().numpy(), refs[1])
    with pytest.raises(rtamd.RTError):
        rtamd.render_loop(ctx, cams, fs.light, W, H, out.data_ptr(), W * 12, 1, True)  # pitch < 16 W


def test_host_render_loop_animated(ctx):
    """rth_render_loop_anim: the C++ loop animating the car's wheels (rt_animate before
    each dispatch) leaves the same frame and node boxes as the same animation frames
    given one by one through the Python binding."""
    import bench
    W, H = 480, 270
    fs = rtamd.generate(3, 0, W, H)
    ids, frames = bench.wheel_frames(fs, 7)
    out = torch.full((H, W, 4), -7.0, dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    ctx.upload(fs)
    ctx.set_params(W, H, 3)
    ctx.set_animated(ids)
    ms = rtamd.render_loop(ctx, fs.camera, fs.light, W, H, out.data_ptr(), W * 16, 10, True, anim=frames)
    assert ms.shape == (10,) and (ms > 0).all()
    got, got_nodes = out.cpu().numpy(), ctx.read_nodes(len(fs.nodes))
    two = rtamd.ComputeShader(0)
    try:
        two.upload(fs)
        two.set_params(W, H, 3)
        two.set_animated(ids)
        for i in range(10):
            two.set_camera(fs.camera)
            two.set_light(fs.light)
            two.animate(frames[i % 7])
        want = two.render(W, H)
        assert np.array_equal(got, want)
        assert np.array_equal(got_nodes, two.read_nodes(len(fs.nodes)))
    finally:
        two.close()
        ctx.upload(fs)


@pytest.mark.parametrize("ranks,share", [(2, 1), (3, 2), (8, 1)])
def test_group_sky_rows_identical(ctx, ranks, share):
    """rt_group_set_sky_rows: the peers keep the background-only rows (every corner of
    the root box on one side of the row's camera-ray plane) off the fan-in and rank 0
    writes their background. Frames with the car camera (its top ~26 % of rows is
    sky), a camera tilted up into the sky, one looking down at the road, and the
    brute branch (where the root box does not gate) equal the single dispatch, with
    the shortcut on and off."""
    W, H = 480, 270
    base = rtamd.generate(3, 0, W, H)
    cams = [base.camera]
    for tgt in ((0.0, -60.0, 0.0), (0.0, 30.0, 0.0)):
        sc = rtamd.Scene().generate(3, 0, W / H)
        sc.LookAt(tgt)
        cams.append(sc.serializeScene().camera)
    g = rtamd.Group([0] * ranks, rtamd.GATHER_COPY, frames=2)
    try:
        g.upload(base)
        g.set_root_share(share)
        for bvh in (True, False):
            g.set_params(W, H, 3, bvh)
            for cam in cams:
                fs = rtamd.FlatScene(base.shapes, base.nodes, base.indices, cam, base.light)
                ctx.upload(fs)
                ctx.set_params(W, H, 3, bvh)
                ref = ctx.render(W, H)
                for on in (True, False):
                    g.set_sky_rows(on)
                    g.set_camera(cam)
                    assert np.array_equal(g.render(W, H, 8), ref), f"bvh={bvh} sky_rows={on}"
    finally:
        g.close()


def test_group_refuses_members_changed_behind_its_back(ctx):
    """The sky-row band is computed from the group's camera and root box on every
    rank. A member whose camera or node boxes were changed through its own context
    would draw geometry in rows the band sends as sky, so with sky rows on the frame
    is refused (RT_ERR_INVALID) before anything is posted; with sky rows off it is
    that member's view; group calls make the members agree again. With the phase
    events off, frames stay bounded by slot back-pressure and exact."""
    W, H = 480, 270
    base = rtamd.generate(3, 0, W, H)
    sc = rtamd.Scene().generate(3, 0, W / H)
    sc.LookAt((0.0, 30.0, 0.0))
    other = sc.serializeScene().camera
    g = rtamd.Group([0, 0], rtamd.GATHER_COPY, frames=2)
    try:
        g.upload(base)
        g.set_params(W, H, 3, True)
        ctx.upload(base)
        ctx.set_params(W, H, 3, True)
        assert np.array_equal(g.render(W, H, 8), ctx.render(W, H))
        for m in g.contexts:
            m.set_camera(other)
        with pytest.raises(rtamd.RTError) as e:
            g.dispatch(W, H, 8)
        assert e.value.code == -1
        ctx.set_camera(other)
        want = ctx.render(W, H)
        g.set_sky_rows(False)
        assert np.array_equal(g.render(W, H, 8), want)
        g.set_sky_rows(True)
        g.set_camera(other)
        assert np.array_equal(g.render(W, H, 8), want)
        nodes = base.nodes.copy()
        nodes["boundsMax"][-1] += np.float32(1.0)
        for m in g.contexts[g.frames:2 * g.frames]:  # every frame slot of member 1
            m.update_nodes(nodes)
        with pytest.raises(rtamd.RTError):
            g.dispatch(W, H, 8)
        g.set_sky_rows(False)
        g.set_phase_timing(False)
        for _ in range(6):
            g.dispatch(W, H, 8)
        g.sync()
        assert np.array_equal(g.read_image(W, H), want)
    finally:
        g.close()


@pytest.mark.parametrize("order_stream", [0, 1, 2])
def test_moving_camera_cost_order_exact(ctx, order_stream):
    """Latency mode with a camera that moves every frame: each dispatch re-derives the
    cost order from its tiles' whole wall times dilated by one tile (k_cost_dilate, then
    k_tile_order) for the next. Every frame equals the row-major frame of its own camera,
    and a still camera after the moves (the still policy again) too. With the order's
    kernels on the order stream (rt_debug_order_stream 1, 2) the next dispatch waits for
    them on the device; mode 2 also with 12 frames in flight between waits (a torn order
    would leave NaN tiles of the poisoned surfaces, or draw a tile twice). Each moving
    frame is waited for by rt_sync_frame (its frame event, before the order's kernels)."""
    import bench
    W, H = 320, 180
    cfg, _, _, mb, _, target = bench.WORKLOADS[3]
    sc = rtamd.Scene().generate(cfg, 0, W / H)
    fs = sc.serializeScene()
    cams = bench.camera_path(rtamd, sc, fs, "orbit", target)[:48:6]  # 8 cameras, 3 degrees apart
    ctx.upload(fs)
    ctx.set_params(W, H, mb, True)
    ctx.set_kernel(rtamd.KERNEL_ACCEL)
    refs = []
    try:
        ctx.set_schedule(rtamd.SCHED_ROWS)
        for cam in cams:
            ctx.set_camera(cam)
            refs.append(ctx.render(W, H))
        ctx.set_schedule(rtamd.SCHED_COST)
        ctx.set_latency_mode(1)
        ctx.debug_order_stream(order_stream)
        full = torch.empty((H, W, 4), dtype=torch.float32, device="cuda")
        if order_stream == 2:
            ctx.debug_sched_period(1)  # every dispatch a cost frame: its order on the order stream
            outs = torch.full((12, H, W, 4), float("nan"), dtype=torch.float32, device="cuda")
            torch.cuda.synchronize()
            for k in range(12):
                ctx.set_camera(cams[k % len(cams)])
                ctx.dispatch_rows(W, H, 0, 1, 1, H, outs[k].data_ptr(), W * 16)
            ctx.sync()
            got = outs.cpu().numpy()
            for k in range(12):
                assert np.array_equal(got[k], refs[k % len(cams)]), f"in flight frame {k}"
            ctx.debug_sched_period(16)
        for rnd in range(3):
            for i, cam in enumerate(cams):
                ctx.set_camera(cam)
                full.fill_(float("nan"))
                torch.cuda.synchronize()  # the renderer's stream does not wait on torch's
                ctx.dispatch_rows(W, H, 0, 1, 1, H, full.data_ptr(), W * 16)
                ctx.sync_frame()  # the frame's end: the cost order may still run behind it
                img = full.cpu().numpy()
                assert np.array_equal(img, refs[i]), f"round {rnd} camera {i}: {int((img != refs[i]).any(axis=-1).sum())} px"
        # the order the last moving frame queued behind its frame event: whole once the
        # stream drains (rt_debug_sched_order synchronizes it)
        tiles = ((W + 7) // 8) * ((H + 7) // 8)
        assert np.array_equal(np.sort(ctx.debug_sched_order(tiles)), np.arange(tiles))
        for _ in range(20):  # held still: the still policy's split frames
            ctx.dispatch_rows(W, H, 0, 1, 1, H, full.data_ptr(), W * 16)
            ctx.sync()
            assert np.array_equal(full.cpu().numpy(), refs[-1])
    finally:
        ctx.debug_order_stream(0)
        ctx.set_latency_mode(0)
        ctx.set_schedule(rtamd.SCHED_COST)
        ctx.set_kernel(rtamd.KERNEL_AUTO)
        ctx.set_camera(fs.camera)
