"""oracle.py — TEST INFRASTRUCTURE ONLY.

ctypes wrapper of the CPU oracle (oracle/build/liboracle.so, restating
src/shaders/gpu_shader.comp, cpuRayTracer and the BVH builder) and of the
reference-header harness (oracle/_ref/libref.so). Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg import this module,
and only as the checker / the CPU baseline; the product never does.
"""
from __future__ import annotations

import ctypes as C
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "opengl-ray-tracer_amd"))
import rtamd  # noqa: E402  (record layouts and rt_params/rt_stats structs)

_P, _I, _F = C.c_void_p, C.c_int, C.c_float

ORACLE_SYMBOLS = {
    "orc_render": (_I, [_P, _I, _P, _I, _P, _I, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P, _P, _I]),
    "orc_cpu_raytracer": (_I, [_P, _I, _P, _P, _I, _I, _I, _I, _P, _I]),
    "orc_build_bvh": (_I, [_P, _I, _I, _P, _I, _P, _I, _P, _P]),
    "orc_intersect": (_I, [_P, _P, _P, _I, _P]),
    "orc_intersect_cpu": (_I, [_P, _P, _P, _P]),
    "orc_get_ray": (_I, [_P, _F, _F, _P, _P]),
    "orc_ray_aabb": (_I, [_P, _P, _P, _P]),
    "orc_wall_end": (_I, [_P, _P]),
    "orc_update_bvh": (_I, [_P, _I, _P, _I, _P, _I, _P, _I]),
}

REF_SYMBOLS = {
    "ref_layout": (_I, [_P, _I]),
    "ref_sphere_isect": (_I, [_P, _F, _P, _P, _P]),
    "ref_plane_isect": (_I, [_P, _P, _P, _P, _P, _P]),
    "ref_wall_isect": (_I, [_P, _F, _F, _P, _P, _P, _P, _P]),
    "ref_wall_end": (_I, [_P, _F, _F, _P, _P]),
    "ref_light_color": (_I, [_P, _P, _F, _P]),
    "ref_material_default": (_I, [_P]),
}

_lib = None


def lib():
    global _lib
    if _lib is None:
        path = os.path.join(HERE, "build", "liboracle.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run `make -C oracle`")
        _lib = rtamd._bind(C.CDLL(path), ORACLE_SYMBOLS)
    return _lib


def ref_lib():
    """The reference's compiled headers, or None when /root/reference was absent at build time."""
    path = os.path.join(HERE, "_ref", "libref.so")
    if not os.path.exists(path):
        return None
    return rtamd._bind(C.CDLL(path), REF_SYMBOLS)


def _p(a):
    return C.c_void_p(a.ctypes.data) if a is not None and a.size else None


def params(resX, resY, maxBounces=3, useBVH=True, useFresnel=False, useMT=False):
    return rtamd.rt_params(float(resX), float(resY), int(maxBounces), int(bool(useBVH)), int(bool(useFresnel)),
                           int(bool(useMT)))


def render(fs: rtamd.FlatScene, width, height, p=None, y0=0, stripe=1, step=1, out_rows=None, stats=False,
           threads=0):
    """orc_render: the GLSL main() restated; returns (image[out_rows, W, 4], stats dict or None)."""
    if p is None:
        p = params(width, height)
    rows = (height - y0) if out_rows is None else out_rows
    out = np.zeros((rows, width, 4), np.float32)
    st = rtamd.rt_stats()
    rc = lib().orc_render(_p(fs.shapes), len(fs.shapes), _p(fs.nodes), len(fs.nodes), _p(fs.indices),
                          len(fs.indices), _p(fs.camera), _p(fs.light), C.byref(p), width, height, y0, stripe, step,
                          rows, _p(out), C.byref(st) if stats else None, threads)
    if rc != 0:
        raise RuntimeError(f"orc_render rc={rc}")
    return out, (st.as_dict() if stats else None)


def cpu_raytracer(fs: rtamd.FlatScene, width, height, y0=0, y1=None, threads=1, out=None):
    """cpuRayTracer (src/main.cpp:848-894) restated; rows [y0, y1)."""
    y1 = height if y1 is None else y1
    if out is None:
        out = np.zeros((y1 - y0, width, 4), np.float32)
    rc = lib().orc_cpu_raytracer(_p(fs.shapes), len(fs.shapes), _p(fs.camera), _p(fs.light), width, height, y0, y1,
                                 _p(out), threads)
    if rc != 0:
        raise RuntimeError(f"orc_cpu_raytracer rc={rc}")
    return out


def build_bvh(shapes: np.ndarray, max_depth: int):
    """Independent restatement of buildBVH + serializeBVH; returns (nodes, indices)."""
    shapes = rtamd.as_records(shapes, rtamd.SHAPE_DTYPE)
    n, i = C.c_int(), C.c_int()
    lib().orc_build_bvh(_p(shapes), len(shapes), max_depth, None, 0, None, 0, C.byref(n), C.byref(i))
    nodes = np.zeros(n.value, rtamd.NODE_DTYPE)
    idx = np.zeros(i.value, np.int32)
    rc = lib().orc_build_bvh(_p(shapes), len(shapes), max_depth, _p(nodes), n.value, _p(idx), i.value, C.byref(n),
                             C.byref(i))
    if rc != 0:
        raise RuntimeError("orc_build_bvh failed")
    return nodes, idx


def update_bvh(fs: rtamd.FlatScene, ids):
    """updateBVH (src/main.cpp:1068-1077) restated: grows fs.nodes in place for the
    animated shapes `ids` at their current records in fs.shapes."""
    ids = np.ascontiguousarray(ids, np.int32)
    rc = lib().orc_update_bvh(_p(fs.shapes), len(fs.shapes), _p(fs.nodes), len(fs.nodes), _p(fs.indices),
                              len(fs.indices), _p(ids), len(ids))
    if rc != 0:
        raise RuntimeError(f"orc_update_bvh rc={rc}")


def intersect(shape_rec: np.ndarray, o, d, use_mt=False):
    shape_rec = rtamd.as_records(shape_rec, rtamd.SHAPE_DTYPE)
    o = np.asarray(o, np.float32)
    d = np.asarray(d, np.float32)
    hit = np.zeros(3, np.float32)
    t = lib().orc_intersect(_p(shape_rec), _p(o), _p(d), int(use_mt), _p(hit))
    return t, hit


def intersect_cpu(shape_rec: np.ndarray, o, d):
    shape_rec = rtamd.as_records(shape_rec, rtamd.SHAPE_DTYPE)
    o = np.asarray(o, np.float32)
    d = np.asarray(d, np.float32)
    hit = np.zeros(3, np.float32)
    t = lib().orc_intersect_cpu(_p(shape_rec), _p(o), _p(d), _p(hit))
    return t, hit


def get_ray(cam: np.ndarray, ndcx, ndcy):
    o = np.zeros(3, np.float32)
    d = np.zeros(3, np.float32)
    lib().orc_get_ray(_p(cam), float(ndcx), float(ndcy), _p(o), _p(d))
    return o, d
