"""Opt-in device BVH build (rt_build_lbvh), -m gpu.

The LBVH is not the reference builder's tree, so the parity target is the
oracle rendering the SAME tree (read back through the C ABI): the frame the
reference shader would produce if its host had uploaded that tree. The tree
itself is checked structurally and its boxes against the oracle's restated
updateBVH (growToInclude of each shape into every node that lists it).
"""
import numpy as np
import pytest
import torch

import oracle
import rtamd
from test_gpu_parity import CFG_BOUNCES, TOL, _soup, check, gpu_rows

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    c = rtamd.ComputeShader(0)
    yield c
    c.close()


def lbvh(ctx, fs):
    ctx.upload(fs)
    ms = ctx.build_lbvh()
    nodes, idx = ctx.read_tree()
    return rtamd.FlatScene(fs.shapes, nodes, idx, fs.camera, fs.light), ms


def check_structure(fs2):
    nodes, idx = fs2.nodes, fs2.indices
    S = len(fs2.shapes)
    assert len(nodes) == max(2 * S - 1, 0) and len(idx) == S
    assert sorted(idx.tolist()) == list(range(S))  # every shape in exactly one leaf
    if S == 0:
        return
    leaf = nodes["leftChild"] == -1
    assert leaf.sum() == S and (nodes["numShapes"][leaf] == 1).all()
    assert (nodes["startShapeIdx"][leaf] == np.arange(len(nodes))[leaf]).all()
    inner = np.where(~leaf)[0]
    L, R = nodes["leftChild"][inner], nodes["rightChild"][inner]
    assert ((L >= 0) & (L < len(nodes)) & (R >= 0) & (R < len(nodes))).all()
    kids = np.concatenate([L, R])
    assert len(np.unique(kids)) == len(kids) == len(nodes) - 1  # a tree: each node has one parent
    assert (len(nodes) - 1) not in kids  # root at N-1 (gpu_shader.comp:386)
    # inner box = union of its children, range = the children's ranges side by side
    lo, hi = nodes["boundsMin"], nodes["boundsMax"]
    assert np.array_equal(lo[inner], np.minimum(lo[L], lo[R]))
    assert np.array_equal(hi[inner], np.maximum(hi[L], hi[R]))
    st, n = nodes["startShapeIdx"], nodes["numShapes"]
    assert (st[inner] == st[L]).all() and (st[L] + n[L] == st[R]).all() and (n[inner] == n[L] + n[R]).all()


@pytest.mark.parametrize("cfg", [2, 3, 5])
def test_lbvh_structure(ctx, cfg):
    fs = rtamd.generate(cfg, 0, 320, 240)
    fs2, ms = lbvh(ctx, fs)
    check_structure(fs2)
    assert ms > 0
    info = ctx.accel_info()
    assert info["built"] == 1 and info["tree_nested"] == 1


def test_lbvh_boxes_are_reference_bounding_boxes(ctx):
    """Node boxes = the reference's growToInclude of every shape a node lists
    (oracle updateBVH from empty boxes), bit for bit."""
    fs = rtamd.generate(2, 0, 200, 150)
    fs2, _ = lbvh(ctx, fs)
    empty = fs2.nodes.copy()
    empty["boundsMin"] = np.float32(np.inf)
    empty["boundsMax"] = np.float32(-np.inf)
    grown = rtamd.FlatScene(fs2.shapes, empty, fs2.indices, fs2.camera, fs2.light)
    oracle.update_bvh(grown, np.arange(len(fs2.shapes), dtype=np.int32))
    assert np.array_equal(grown.nodes["boundsMin"], fs2.nodes["boundsMin"])
    assert np.array_equal(grown.nodes["boundsMax"], fs2.nodes["boundsMax"])


CASES = [  # cfg, W, H, y0, rows
    (2, 200, 150, 0, None),
    (3, 1920, 1080, 560, 24),
    (5, 480, 270, 0, None),
]


@pytest.mark.parametrize("kernel", [rtamd.KERNEL_ACCEL, rtamd.KERNEL_PACKET, rtamd.KERNEL_LANE])
@pytest.mark.parametrize("case", CASES, ids=lambda c: "c%d_%dx%d" % c[:3])
def test_lbvh_frame_matches_oracle_on_the_same_tree(ctx, case, kernel):
    cfg, W, H, y0, rows = case
    fs = rtamd.generate(cfg, 0, W, H)
    fs2, _ = lbvh(ctx, fs)
    p = oracle.params(W, H, CFG_BOUNCES[cfg])
    rows = H - y0 if rows is None else rows
    ref, _ = oracle.render(fs2, W, H, p, y0=y0, out_rows=rows)
    # gpu_rows uploads fs2: the same tree the device built, through the host path
    img = gpu_rows(ctx, fs2, W, H, p, y0=y0, rows=rows, kernel=kernel)
    check(img, ref, f"lbvh config {cfg} kernel {kernel}")
    # and the adopted device tree renders that frame without the round trip
    ctx.upload(fs)
    ctx.build_lbvh()
    ctx.set_kernel(kernel)
    out = torch.full((rows, W, 4), -7.0, dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    ctx.dispatch_rows(W, H, y0, 1, 1, rows, out.data_ptr(), W * 16)
    ctx.sync()
    assert np.array_equal(out.cpu().numpy(), img)


def test_lbvh_soup_with_planes_and_walls(ctx):
    """Planes (no box), ±Y walls and slivers under the LBVH: oracle parity."""
    W, H = 200, 150
    fs2, _ = lbvh(ctx, _soup(3))
    check_structure(fs2)
    p = oracle.params(W, H, 3)
    ref, _ = oracle.render(fs2, W, H, p)
    img = gpu_rows(ctx, fs2, W, H, p, kernel=rtamd.KERNEL_ACCEL)
    check(img, ref, "lbvh soup")


@pytest.mark.parametrize("n", [0, 1, 2, 3])
def test_lbvh_tiny_scenes(ctx, n):
    fs = rtamd.generate(1, 0, 64, 48)
    shapes = fs.shapes[:n].copy()
    nodes, idx = oracle.build_bvh(shapes, 5) if n else (np.zeros(0, rtamd.NODE_DTYPE), np.zeros(0, np.int32))
    fs1 = rtamd.FlatScene(shapes, nodes, idx, fs.camera, fs.light)
    fs2, _ = lbvh(ctx, fs1)
    check_structure(fs2)
    p = oracle.params(64, 48, 2)
    ref, _ = oracle.render(fs2, 64, 48, p)
    img = gpu_rows(ctx, fs2, 64, 48, p, kernel=rtamd.KERNEL_ACCEL)
    check(img, ref, f"{n} shapes")
