"""OBJ ingestion and image dump, host library, CPU.

The reference loads meshes with assimp (src/model.hpp:49-168, aiProcess_Triangulate)
and presents the RGBA32F texture on a screen quad (shaders/shader.frag). Neither
runs here (assimp and its assets are absent; no GL), so these tests pin the
restated behaviour: fan triangulation of polygons, OBJ index forms, the
mesh2triangles origin/orientation rule via rts_add_mesh, and exact PFM / clamped
PPM output. Parity with assimp itself is unpinned.
"""
import numpy as np
import pytest

import oracle
import rtamd

CUBE = """# unit cube, quads, mixed corner forms
o cube
v 0 0 0
v 1 0 0
v 1 1 0
v 0 1 0
v 0 0 1
v 1 0 1
v 1 1 1
v 0 1 1
vt 0 0
vn 0 0 1
f 1 2 3 4
f 5/1 8/1 7/1 6/1
f 1//1 5//1 6//1 2//1
f 2/1/1 6/1/1 7/1/1 3/1/1
f -5 -8 -4 -1
f 4 3 7 8
"""


def _tris(fs):
    t = fs.shapes[fs.shapes["type"] == 3]
    return np.stack([t["triP1"], t["triP2"], t["triP3"]], axis=1)


def test_obj_fan_triangulation_matches_add_mesh():
    a = rtamd.Scene()
    n = a.parse_obj(CUBE, origin=(1, 2, 3))
    assert n == 12
    b = rtamd.Scene()
    v = np.array([[0, 0, 0], [1, 0, 0], [1, 1, 0], [0, 1, 0], [0, 0, 1], [1, 0, 1], [1, 1, 1], [0, 1, 1]], np.float32)
    faces = [[0, 1, 2, 3], [4, 7, 6, 5], [0, 4, 5, 1], [1, 5, 6, 2], [3, 0, 4, 7], [3, 2, 6, 7]]
    idx = [[f[0], f[k], f[k + 1]] for f in faces for k in (1, 2)]
    b.add_mesh(v, np.array(idx, np.uint32), origin=(1, 2, 3))
    for sc in (a, b):
        sc.set_camera((0, 0, 10), 60, 1.0)
        sc.LookAt((0, 0, 0))
        sc.buildBVH(15)
    fa, fb = a.serializeScene(), b.serializeScene()
    assert fa.shapes.tobytes() == fb.shapes.tobytes()
    assert fa.nodes.tobytes() == fb.nodes.tobytes()
    assert np.array_equal(_tris(fa)[0], np.array([[1, 2, 3], [2, 2, 3], [2, 3, 3]], np.float32))


def test_obj_oriented_flag_and_file(tmp_path):
    p = tmp_path / "cube.obj"
    p.write_text(CUBE.replace("\n", "\r\n"))  # CRLF files too
    a, b = rtamd.Scene(), rtamd.Scene()
    assert a.load_obj(str(p), oriented=True) == 12
    b.parse_obj(CUBE, oriented=True)
    for sc in (a, b):
        sc.buildBVH(15)
    assert a.serializeScene().shapes.tobytes() == b.serializeScene().shapes.tobytes()


@pytest.mark.parametrize("bad", ["f 1 2\n", "v 0 0 0\nf 1 2 3\n", "v 0 0\n", "v 0 0 0\nv 1 0 0\nv 0 1 0\nf 0 1 2\n",
                                 "v 0 0 0\nv 1 0 0\nv 0 1 0\nf -4 -1 -2\n", "v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 x 3\n"])
def test_obj_malformed_is_an_error(bad):
    with pytest.raises(rtamd.RTError) as e:
        rtamd.Scene().parse_obj(bad)
    assert e.value.code == -3


def test_obj_missing_file(tmp_path):
    with pytest.raises(rtamd.RTError) as e:
        rtamd.Scene().load_obj(str(tmp_path / "nope.obj"))
    assert e.value.code == -2


def test_obj_scene_renders_like_the_oracle():
    """An OBJ-loaded mesh goes through the same builder and serialiser: the
    oracle's whole frame of it equals the frame of the same triangles added
    with add_mesh (host side; GPU parity of such scenes is in test_gpu_parity)."""
    a = rtamd.Scene()
    a.parse_obj(CUBE, origin=(-0.5, -0.5, -0.5))
    a.set_camera((2.0, 1.5, 3.0), 60, 4 / 3)
    a.LookAt((0, 0, 0))
    a.set_light((3, 3, 3), (1, 1, 1), 10)
    a.buildBVH(15)
    fs = a.serializeScene()
    img, _ = oracle.render(fs, 64, 48, oracle.params(64, 48, 2))
    assert np.isfinite(img).all() and img[..., :3].max() > 0


def test_write_ppm_and_pfm(tmp_path):
    rng = np.random.default_rng(3)
    img = rng.uniform(-0.5, 1.5, (5, 7, 4)).astype(np.float32)
    img[0, 0, 0] = np.nan
    p, f = tmp_path / "a.ppm", tmp_path / "a.pfm"
    rtamd.write_image(str(p), img, rtamd.IMAGE_PPM)
    rtamd.write_image(str(f), img, rtamd.IMAGE_PFM)
    raw = p.read_bytes()
    assert raw.startswith(b"P6\n7 5\n255\n")
    px = np.frombuffer(raw[len(b"P6\n7 5\n255\n"):], np.uint8).reshape(5, 7, 3)
    want = np.rint(np.clip(np.nan_to_num(img[..., :3], nan=0.0), 0, 1) * 255).astype(np.uint8)
    assert np.array_equal(px, want)
    raw = f.read_bytes()
    hdr = b"PF\n7 5\n-1.0\n"
    assert raw.startswith(hdr)
    got = np.frombuffer(raw[len(hdr):], "<f4").reshape(5, 7, 3)[::-1]  # PFM: bottom row first
    assert np.array_equal(got, img[..., :3], equal_nan=True)


def test_write_image_rejects_bad_arguments(tmp_path):
    with pytest.raises(ValueError):
        rtamd.write_image(str(tmp_path / "x.ppm"), np.zeros((4, 4, 3), np.float32))
    with pytest.raises(rtamd.RTError):
        rtamd.write_image(str(tmp_path / "x.ppm"), np.zeros((4, 4, 4), np.float32), fmt=7)
