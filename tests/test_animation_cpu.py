"""updateBVH (src/main.cpp:1068-1077) restated in the oracle (orc_update_bvh),
checked on CPU against a second, independent restatement written here over the
reference's own data structures (per-node shapesIndices, as split() keeps them
on inner nodes too, src/main.cpp:1128-1144) and against its defining
properties: grow-only, idempotent on unmoved shapes, untouched elsewhere.
The device refit (rt_animate) is checked against orc_update_bvh on the GPU
(tests/test_gpu_parity.py, test_device_refit_*).
"""
import os
import subprocess

import numpy as np
import pytest

import oracle
import rtamd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _points(rec):
    """BoundingBox::growToInclude(shape) (BoundingBox.hpp:50-95) as the points it adds."""
    t = int(rec["type"])
    if t == 0:
        c, r = rec["sphereCenter"].astype(np.float32), np.float32(rec["sphereRadius"])
        return [c + r, c - r]
    if t == 2:
        e = np.zeros(3, np.float32)
        oracle.lib().orc_wall_end(oracle._p(np.ascontiguousarray(rec.reshape(1))), oracle._p(e))
        return [rec["wallStart"].astype(np.float32), e]
    if t == 3:
        if all(np.isfinite(rec[f][0]) for f in ("triP1", "triP2", "triP3")):
            return [rec[f].astype(np.float32) for f in ("triP1", "triP2", "triP3")]
    return []


def _shape_sets(nodes, idx):
    """Per node, the reference's shapesIndices: a leaf's own, an inner node's the union below."""
    sets = [None] * len(nodes)

    def get(k):
        if sets[k] is None:
            n = nodes[k]
            if n["leftChild"] == -1:
                sets[k] = set(int(i) for i in idx[n["startShapeIdx"]:n["startShapeIdx"] + n["numShapes"]])
            else:
                sets[k] = get(int(n["leftChild"])) | get(int(n["rightChild"]))
        return sets[k]
    for k in range(len(nodes)):
        get(k)
    return sets


def _update_bvh_py(shapes, nodes, idx, animated):
    out = nodes.copy()
    sets = _shape_sets(nodes, idx)
    for k in range(len(out)):
        lo, hi = out["boundsMin"][k].copy(), out["boundsMax"][k].copy()
        for i in sorted(sets[k]):
            if i not in animated:
                continue
            for p in _points(shapes[i]):
                for a in range(3):  # glm::min(Min, p): (p < Min) ? p : Min
                    lo[a] = p[a] if p[a] < lo[a] else lo[a]
                    hi[a] = p[a] if hi[a] < p[a] else hi[a]
        out["boundsMin"][k], out["boundsMax"][k] = lo, hi
    return out


def _scene(seed, depth):
    rng = np.random.default_rng(seed)
    sc = rtamd.Scene()
    for _ in range(120):
        c = rng.uniform(-10, 10, 3)
        v = c + rng.normal(size=(3, 3))
        sc.add_triangle(v[0], v[1], v[2])
    for _ in range(15):
        sc.add_sphere(rng.uniform(-10, 10, 3), rng.uniform(0.2, 1.5))
    sc.add_wall((-5, -2, -5), 4, 3, (0.2, 0.1, 1.0))
    sc.add_wall((3, 1, 2), 2, 5, (1.0, 0.0, 0.3))
    sc.add_plane((0, 1, 0), (0, 5, 0))
    sc.set_camera((0, 0, 30), 60, 4 / 3)
    sc.set_light((5, -10, 5), (1, 1, 1), 30)
    sc.buildBVH(depth)
    return sc.serializeScene()


def _move(shapes, ids, rng):
    s = shapes.copy()
    for i in ids:
        t = s["type"][i]
        if t == 0:
            s["sphereCenter"][i] += rng.normal(size=3).astype(np.float32) * 3
        elif t == 2:
            s["wallStart"][i] += rng.normal(size=3).astype(np.float32) * 3
        elif t == 3:
            d = rng.normal(size=3).astype(np.float32) * 3
            for f in ("triP1", "triP2", "triP3"):
                s[f][i] += d
    return s


@pytest.mark.parametrize("depth", [0, 3, 15])
@pytest.mark.parametrize("seed", [1, 2])
def test_update_bvh_matches_independent_restatement(depth, seed):
    fs = _scene(seed, depth)
    rng = np.random.default_rng(seed)
    ids = rng.choice(len(fs.shapes), 25, replace=False).astype(np.int32)
    for step in range(3):
        fs.shapes = _move(fs.shapes, ids, rng)
        want = _update_bvh_py(fs.shapes, fs.nodes, fs.indices, set(int(i) for i in ids))
        oracle.update_bvh(fs, ids)
        for f in ("boundsMin", "boundsMax", "leftChild", "rightChild", "startShapeIdx", "numShapes"):
            assert np.array_equal(fs.nodes[f], want[f]), (step, f)


def test_update_bvh_properties():
    fs = _scene(7, 10)
    before = fs.nodes.copy()
    ids = np.arange(0, len(fs.shapes), 3, dtype=np.int32)
    oracle.update_bvh(fs, ids)  # unmoved: the built boxes already hold every shape
    assert np.array_equal(fs.nodes, before)
    rng = np.random.default_rng(0)
    fs.shapes = _move(fs.shapes, ids, rng)
    oracle.update_bvh(fs, ids)
    grown = fs.nodes
    assert (grown["boundsMin"] <= before["boundsMin"]).all() and (grown["boundsMax"] >= before["boundsMax"]).all()
    sets = _shape_sets(before, fs.indices)
    moved = set(int(i) for i in ids)
    for k in range(len(grown)):
        if not (sets[k] & moved):
            assert np.array_equal(grown[k], before[k])  # nodes not listing a moved shape keep their box
        for i in sets[k] & moved:
            for p in _points(fs.shapes[i]):
                assert (grown["boundsMin"][k] <= p).all() and (p <= grown["boundsMax"][k]).all()
    oracle.update_bvh(fs, ids)  # idempotent
    assert np.array_equal(fs.nodes, grown)


def test_update_bvh_rejects_bad_ids():
    fs = _scene(3, 4)
    with pytest.raises(RuntimeError):
        oracle.update_bvh(fs, np.array([len(fs.shapes)], np.int32))


def test_class_check_equals_classify():
    """rt_animate's per-frame class check (rta::classify_class: classify's class
    without the box, squared forms of its square-root tests with a 1e-9 margin and
    classify itself inside it) equals classify on 400k triangles, many placed at
    its thresholds, and on degenerate / non-finite records (tests/native/class_check.cpp)."""
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "native"), "build/class_check"], check=True)
    r = subprocess.run([os.path.join(ROOT, "tests", "native", "build", "class_check")], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "class_check ok" in r.stdout and " 0 mismatches" in r.stdout


@pytest.mark.parametrize("depth", [0, 3, 15])
@pytest.mark.parametrize("seed", [1, 2])
def test_host_update_bvh_equals_oracle(depth, seed):
    """rts_update_bvh (librtscene.so: the updateBVH a host keeping the reference's own
    upload runs before rt_update_nodes) grows the same boxes, bit for bit, as the
    oracle's restatement, over moving frames."""
    fs = _scene(seed, depth)
    rng = np.random.default_rng(100 + seed)
    ids = np.sort(rng.choice(len(fs.shapes), 30, replace=False)).astype(np.int32)
    mine = rtamd.FlatScene(fs.shapes.copy(), fs.nodes.copy(), fs.indices, fs.camera, fs.light)
    for step in range(4):
        fs.shapes = _move(fs.shapes, ids, rng)
        mine.shapes = fs.shapes.copy()
        oracle.update_bvh(fs, ids)
        rtamd.update_bvh(mine, ids)
        for f in ("boundsMin", "boundsMax", "leftChild", "rightChild", "startShapeIdx", "numShapes"):
            assert np.array_equal(mine.nodes[f].view(np.uint32 if mine.nodes[f].dtype.kind == "f" else np.int32),
                                  fs.nodes[f].view(np.uint32 if fs.nodes[f].dtype.kind == "f" else np.int32)), (step, f)
    with pytest.raises(rtamd.RTError):
        rtamd.update_bvh(mine, np.array([len(fs.shapes)], np.int32))
