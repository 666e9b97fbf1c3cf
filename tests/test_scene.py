"""Host scene library (librtscene.so): generators, builder properties, the
reference rules that change serialised bytes."""
import hashlib

import numpy as np
import pytest

import oracle
import rtamd


@pytest.mark.parametrize("cfg,variant,shapes,tris", [(1, 0, 5, 0), (2, 0, 1240, 1209), (3, 0, 4122, 4022),
                                                     (3, 1, 4342, 4242), (5, 0, 100000, 100000)])
def test_config_shape_counts(cfg, variant, shapes, tris):
    fs = rtamd.generate(cfg, variant, 1920, 1080)
    assert len(fs.shapes) == shapes
    assert int((fs.shapes["type"] == rtamd.TRIANGLE).sum()) == tris


def test_car_bvh_degenerates_like_the_reference():
    """A 2-triangle road collapses the spatial-midpoint builder."""
    sc = rtamd.Scene().generate(3, 0, 16 / 9)
    st = sc.bvh_stats()
    s, n, i = sc.counts()
    assert (s, n, i) == (4122, 3, 4122)
    assert st["leaves"] == 2 and st["max_leaf"] > 2000


def test_random_mesh_bvh_is_deep():
    sc = rtamd.Scene().generate(5, 0, 16 / 9)
    st = sc.bvh_stats()
    s, n, _ = sc.counts()
    assert n > 180000 and st["max_leaf"] <= 4 and st["max_stack"] <= 64


def test_generators_are_deterministic():
    h = [hashlib.sha256(rtamd.generate(2, 0, 800, 600).shapes.tobytes()).hexdigest() for _ in range(2)]
    assert h[0] == h[1]


def test_postorder_root_last():
    fs = rtamd.generate(2, 0, 800, 600)
    nodes = fs.nodes
    root = len(nodes) - 1
    for k, nd in enumerate(nodes):
        if nd["leftChild"] != -1:
            # children are serialised before their parent (src/main.cpp:1163-1170)
            assert nd["leftChild"] < k and nd["rightChild"] < k
    assert nodes[root]["numShapes"] == len(fs.shapes)


def test_triangle_normal_and_invert():
    sc = rtamd.Scene()
    a, b, c = (0, 0, 0), (5, 0, 0), (2.5, -5, 0)
    sc.add_triangle(a, b, c)
    sc.add_triangle(a, b, c, invert=True)
    s = sc.serializeScene().shapes
    assert np.allclose(s["planeNormal"][0], [0, 0, -1]) and s["planeD"][0] == 0
    assert np.array_equal(s["planeNormal"][1], -s["planeNormal"][0])


def test_mesh_orientation_rule_is_opt_in():
    """generateScene1/2 rebuild mesh triangles from their vertices, which drops
    mesh2triangles' flip (src/main.cpp:654,671,763 vs src/mesh.hpp:178-184)."""
    v = np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0]], np.float32)
    i = np.array([0, 1, 2], np.uint32)
    sc = rtamd.Scene()
    sc.add_mesh(v, i, origin=(0, 0, 5))
    sc.add_mesh(v, i, origin=(0, 0, 5), oriented=True)
    s = sc.serializeScene().shapes
    # winding normal (0,0,1); centre has z > 0 -> dot > 0 -> the oriented copy flips
    assert np.allclose(s["planeNormal"][0], [0, 0, 1])
    assert np.allclose(s["planeNormal"][1], [0, 0, -1])


def test_camera_lookat_orthonormal():
    fs = rtamd.generate(3, 0, 1920, 1080)
    c = fs.camera[0]
    F, U, R = (np.asarray(c[k], np.float64) for k in ("Front", "Up", "Right"))
    for v in (F, U, R):
        assert abs(np.linalg.norm(v) - 1) < 1e-6
    assert abs(F @ U) < 1e-6 and abs(F @ R) < 1e-6
    target = np.zeros(3) - np.asarray(c["Position"], np.float64)
    assert np.allclose(F, target / np.linalg.norm(target), atol=1e-6)


def test_cpu_raytracer_primary_hits_match_oracle_brute():
    """cpuRayTracer (CPU phong, black background) and the GLSL brute branch see
    the same closest shape: where the GLSL frame hits something with maxBounces=1
    the CPU frame's pixel is lit by the same shape."""
    W, H = 96, 72
    fs = rtamd.generate(1, 0, W, H)
    cpu = oracle.cpu_raytracer(fs, W, H)
    gl, _ = oracle.render(fs, W, H, oracle.params(W, H, 1, useBVH=False))
    bg = np.zeros((H, W, 3), np.float32)
    for y in range(H):
        t = np.float32(y) / np.float32(H)
        bg[y] = np.float32([0.05, 0.07, 0.1]) + t * (np.float32([0.5, 0.7, 1.0]) - np.float32([0.05, 0.07, 0.1]))
    gl_hit = np.any(np.abs(gl[..., :3] - bg) > 1e-6, axis=-1)
    cpu_hit = np.any(cpu[..., :3] != 0, axis=-1)
    assert gl_hit.sum() > 100
    assert (cpu_hit & ~gl_hit).sum() == 0
    assert np.all(cpu[..., 3] == 1)


def test_errors_are_status_codes():
    sc = rtamd.Scene()
    with pytest.raises(rtamd.RTError):
        sc.add_mesh(np.zeros((3, 3), np.float32), np.array([0, 1, 5], np.uint32))
    with pytest.raises(rtamd.RTError):
        sc.generate(4)


def test_default_scene3_single_triangle_no_tree():
    """The reference's default scene (`int SCENE = 3`, src/main.cpp:46; generateScene3
    :1196-1229): one triangle with the Material() defaults, Camera() at (0,-10,40)
    looking at the origin, the scene-2 light, and no buildBVH call -- zero nodes and
    zero bvhIndices. The brute branch sees the triangle, the BVH branch nothing."""
    sc = rtamd.Scene().generate(6, 0, 800 / 600)
    assert sc.counts() == (1, 0, 0)
    fs = sc.serializeScene()
    s = fs.shapes[0]
    assert int(s["type"]) == 3
    np.testing.assert_array_equal(s["triP1"], [0, 0, 0])
    np.testing.assert_array_equal(s["triP2"], [5, 0, 0])
    np.testing.assert_array_equal(s["triP3"], [2.5, -5, 0])
    np.testing.assert_array_equal(s["planeNormal"], [0, 0, -1])  # normalize(cross(b-a, c-a))
    np.testing.assert_array_equal(fs.camera["Position"][0], [0, -10, 40])
    assert float(fs.camera["fov"][0]) == 60.0 and abs(float(fs.camera["aspectRatio"][0]) - 4 / 3) < 1e-7
    W, H = 200, 150
    bg, _ = oracle.render(fs, W, H, oracle.params(W, H, 3, 1))
    for mt in (0, 1):
        img, _ = oracle.render(fs, W, H, oracle.params(W, H, 3, 0, 0, mt))
        hit = (img != bg).any(axis=-1)
        assert 50 < int(hit.sum()) < W * H // 4, mt
        # the base vertex (0,0,0) is the look-at point (NDC 0 = row H/2); row 0 is NDC +1
        # along Up ~ (0,0.97,0.24), so the apex at y = -5 lies in the rows below
        ys = np.nonzero(hit.any(axis=1))[0]
        assert ys.min() == H // 2 and ys.max() < H * 3 // 4
