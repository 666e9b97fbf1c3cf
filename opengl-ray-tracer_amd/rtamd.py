"""rtamd — Python host binding of the MI355X ray tracer.

Thin ctypes layer over the two product libraries built in-tree by
``opengl-ray-tracer_amd/Makefile``:

* ``lib/librtamd.so``  — the HIP renderer, C ABI ``include/rt_api.h``: the drop-in
  for the reference's compute-shader dispatch (``src/computeShader.hpp``,
  ``src/main.cpp:238-370``).
* ``lib/librtscene.so`` — the host scene library, C ABI ``include/rt_scene.h``:
  shapes, ``buildBVH``/``split``, ``serializeScene`` (``src/main.cpp:806-1193``).

Class and method names mirror the reference (``Scene.buildBVH``,
``Scene.serializeScene``, ``ComputeShader.dispatch`` ...). Loading fails loudly:
there is no CPU fallback anywhere in this module.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# RTAMD_LIBDIR: another build's directory (librtamd.so, librtscene.so, librthost.so), for
# A/B profiling of build variants (tools/build_var.sh); the default is the in-tree lib/
LIBDIR = os.environ.get("RTAMD_LIBDIR") or os.path.join(HERE, "lib")

# ---------------------------------------------------------------------------
# Record layouts (include/rt_flat.h; sizes pinned by static asserts there).

def _vec(off):
    return [("x", off), ("y", off + 4), ("z", off + 8)]


MATERIAL_DTYPE = np.dtype({
    "names": ["color", "fresnelStrength", "ambientStrength", "diffuseStrength", "specularStrength", "shininess"],
    "formats": [("<f4", 3), "<f4", "<f4", "<f4", "<f4", "<i4"],
    "offsets": [0, 12, 16, 20, 24, 28],
    "itemsize": 32,
})

SHAPE_DTYPE = np.dtype({
    "names": ["type", "material", "sphereCenter", "sphereRadius", "planeNormal", "planeD",
              "wallStart", "wallWidth", "wallHeight", "triP1", "triP2", "triP3"],
    "formats": ["<i4", MATERIAL_DTYPE, ("<f4", 3), "<f4", ("<f4", 3), "<f4",
                ("<f4", 3), "<f4", "<f4", ("<f4", 3), ("<f4", 3), ("<f4", 3)],
    "offsets": [0, 32, 64, 76, 80, 92, 96, 108, 112, 144, 160, 176],
    "itemsize": 192,
})

NODE_DTYPE = np.dtype({
    "names": ["boundsMin", "boundsMax", "leftChild", "rightChild", "startShapeIdx", "numShapes"],
    "formats": [("<f4", 3), ("<f4", 3), "<i4", "<i4", "<i4", "<i4"],
    "offsets": [0, 16, 32, 36, 40, 44],
    "itemsize": 48,
})

CAMERA_DTYPE = np.dtype({
    "names": ["Position", "aspectRatio", "Front", "Up", "Right", "fov"],
    "formats": [("<f4", 3), "<f4", ("<f4", 3), ("<f4", 3), ("<f4", 3), "<f4"],
    "offsets": [0, 12, 16, 32, 48, 64],
    "itemsize": 80,
})

LIGHT_DTYPE = np.dtype({
    "names": ["position", "color"],
    "formats": [("<f4", 3), ("<f4", 3)],
    "offsets": [0, 16],
    "itemsize": 32,
})

SPHERE, PLANE, WALL, TRIANGLE = 0, 1, 2, 3
KERNEL_AUTO, KERNEL_LANE, KERNEL_PACKET, KERNEL_ACCEL = 0, 1, 2, 3
SCHED_ROWS, SCHED_COST, SCHED_COST_XCD = 0, 1, 2
TREE_REFERENCE, TREE_SCENE = 0, 1


class rt_params(C.Structure):
    """Uniforms of gpu_shader.comp:126-130."""
    _fields_ = [("resX", C.c_float), ("resY", C.c_float), ("maxBounces", C.c_int), ("useBVH", C.c_int),
                ("useFresnel", C.c_int), ("useMollerTrumbore", C.c_int)]


class rt_accel_info(C.Structure):
    _fields_ = [(n, C.c_int) for n in ("built", "local_nodes", "local_leaves", "bounded_prims", "always_prims",
                                       "max_stack", "last_kernel", "scene_tree", "scene_nodes", "scene_items",
                                       "scene_height", "tree_nested", "record_bytes")]


class rt_stats(C.Structure):
    _fields_ = [("pixels", C.c_uint64), ("closest_rays", C.c_uint64), ("shadow_rays", C.c_uint64),
                ("node_visits", C.c_uint64), ("bvh_tests", C.c_uint64 * 4), ("brute_tests", C.c_uint64 * 4),
                ("closest_updates", C.c_uint64), ("hits", C.c_uint64)]

    def as_dict(self):
        return {"pixels": self.pixels, "closest_rays": self.closest_rays, "shadow_rays": self.shadow_rays,
                "node_visits": self.node_visits, "bvh_tests": list(self.bvh_tests),
                "brute_tests": list(self.brute_tests), "closest_updates": self.closest_updates, "hits": self.hits}


# Bytes of the reference's records that a test of each shape type reads
# (SURVEY §8(d)): 4 B type tag + sphere 16 | plane 16 | wall 36 | triangle 52 (36 for MT).
P_TYPE = {0: 4 + 16, 1: 4 + 16, 2: 4 + 36, 3: 4 + 52}
P_TYPE_MT = {0: 4 + 16, 1: 4 + 16, 2: 4 + 36, 3: 4 + 36}


def algorithmic_bytes(st: dict, pixels_written: int, use_mt: bool = False) -> int:
    """B_alg of SURVEY §8(d): 40 B per node visit, (4 B index + record bytes) per
    BVH leaf test, record bytes per brute-force test, 32 B material per closest
    update, 16 B per RGBA32F pixel store."""
    p = P_TYPE_MT if use_mt else P_TYPE
    b = 40 * st["node_visits"] + 32 * st["closest_updates"] + 16 * pixels_written
    b += sum((4 + p[t]) * n for t, n in enumerate(st["bvh_tests"]))
    b += sum(p[t] * n for t, n in enumerate(st["brute_tests"]))
    return int(b)


STATUS = {0: "ok", -1: "invalid argument", -2: "HIP runtime error", -3: "device allocation failed",
          -4: "scene, camera or light not uploaded", -5: "node/index arrays out of range or deeper than the 64-entry stack",
          -6: "no such HIP device", -7: "RCCL call failed (the group's communicator is aborted)",
          -8: "timed out waiting for a group's frames (the communicator is aborted)"}


class RTError(RuntimeError):
    def __init__(self, what, code):
        super().__init__(f"{what} failed: {STATUS.get(code, code)} ({code})")
        self.code = code


def _ptr(a):
    return C.c_void_p(a.ctypes.data) if a is not None and a.size else None


def as_records(a, dtype):
    """Contiguous array with exactly the C record layout. numpy may pack a
    padded structured dtype (np.concatenate does), which would hand the C side
    records of the wrong size."""
    a = np.asarray(a)
    if a.dtype != dtype:
        a = a.astype(dtype)
    return np.ascontiguousarray(a)


_P = C.c_void_p
_I = C.c_int


def _load(name):
    path = os.path.join(LIBDIR, name)
    if not os.path.exists(path):
        raise RuntimeError(f"{path} is missing: build it with `make -C opengl-ray-tracer_amd` "
                           f"(or __graft_entry__.build()); there is no fallback path")
    return C.CDLL(path)


_scene_lib = None
_rt_lib = None

SCENE_SYMBOLS = {
    "rts_new": (_P, []), "rts_free": (None, [_P]), "rts_clear": (_I, [_P]),
    "rts_add_sphere": (_I, [_P, _P, C.c_float, _P]),
    "rts_add_plane": (_I, [_P, _P, _P, _P]),
    "rts_add_wall": (_I, [_P, _P, C.c_float, C.c_float, _P, _P]),
    "rts_add_triangle": (_I, [_P, _P, _P, _P, _I, _P]),
    "rts_add_mesh": (_I, [_P, _P, _I, _P, _I, _P, _P]),
    "rts_add_mesh_oriented": (_I, [_P, _P, _I, _P, _I, _P, _P]),
    "rts_set_camera": (_I, [_P, _P, C.c_float, C.c_float]),
    "rts_camera_look_at": (_I, [_P, _P]),
    "rts_set_light": (_I, [_P, _P, _P, C.c_float]),
    "rts_build_bvh": (_I, [_P, _I]),
    "rts_counts": (_I, [_P, _P, _P, _P]),
    "rts_serialize": (_I, [_P, _P, _P, _P, _P, _P]),
    "rts_bvh_stats": (_I, [_P, _P, _P, _P, _P]),
    "rts_generate": (_I, [_P, _I, _I, C.c_float]),
    "rts_load_obj": (_I, [_P, C.c_char_p, _P, _P, _I]),
    "rts_parse_obj": (_I, [_P, C.c_char_p, C.c_long, _P, _P, _I]),
    "rts_write_image": (_I, [C.c_char_p, _P, _I, _I, C.c_long, _I]),
    "rts_update_bvh": (_I, [_P, _I, _P, _I, _P, _I, _P, _I]),
}

# include/rt_host.h (librthost.so: the reference's render loop as a C++ host)
HOST_SYMBOLS = {
    "rth_render_loop": (_I, [_P, _P, _I, _P, _I, _I, _P, C.c_size_t, _I, _I, _P]),
    "rth_render_loop_anim": (_I, [_P, _P, _I, _P, _I, _I, _P, C.c_size_t, _I, _I, _P, _I, _I, _P]),
    "rth_upload_animated": (_I, [_P, _P, _I, _P, _P, _I, _P, _I, _P, _I]),
    "rth_group_upload_animated": (_I, [_P, _P, _I, _P, _P, _I, _P, _I, _P, _I]),
    "rth_render_rows_loop": (_I, [_P, _P, _I, _P, _I, _I, _I, _I, _I, _I, _I, _P, C.c_size_t, _I, _I, _P]),
    "rth_render_loop_ref": (_I, [_P, _P, _I, _P, _I, _I, _P, C.c_size_t, _I, _I, _P, _I, _P, _I, _P, _I, _P, _I,
                                 _P, _I, _P]),
}

RT_SYMBOLS = {
    "rt_create": (_I, [_P, _I]), "rt_destroy": (_I, [_P]), "rt_set_stream": (_I, [_P, _P]),
    "rt_upload_scene": (_I, [_P, _P, _I, _P, _I, _P, _I]),
    "rt_update_shapes": (_I, [_P, _I, _I, _P]),
    "rt_update_nodes": (_I, [_P, _P, _I]),
    "rt_set_animated": (_I, [_P, _P, _I]), "rt_animate": (_I, [_P, _P]),
    "rt_read_nodes": (_I, [_P, _P, _I]),
    "rt_set_camera": (_I, [_P, _P]), "rt_set_light": (_I, [_P, _P]),
    "rt_set_params": (_I, [_P, _P]), "rt_set_kernel": (_I, [_P, _I]),
    "rt_dispatch": (_I, [_P, _I, _I, _I, _I]),
    "rt_dispatch_rows": (_I, [_P, _I, _I, _I, _I, _I, _I, _P, C.c_size_t]),
    "rt_dispatch_rows_fmt": (_I, [_P, _I, _I, _I, _I, _I, _I, _P, C.c_size_t, _I]),
    "rt_dispatch_rows_ex": (_I, [_P, _I, _I, _I, _I, _I, _I, _P, C.c_size_t, _I]),
    "rt_sync": (_I, [_P]), "rt_sync_frame": (_I, [_P]), "rt_read_image": (_I, [_P, _P, C.c_size_t, _I, _I]),
    "rt_device_image": (_I, [_P, _P, _P]),
    "rt_collect_stats": (_I, [_P, _I, _I, _I, _I, _I, _I, _P]),
    "rt_collect_stats_ex": (_I, [_P, _I, _I, _I, _I, _I, _I, _P]),
    "rt_last_kernel_ms": (_I, [_P, _P]),
    "rt_kernel_times": (_I, [_P, _P, _I]),
    "rt_accel_info_get": (_I, [_P, _P]),
    "rt_set_launch": (_I, [_P, _I, _I]),
    "rt_set_walk": (_I, [_P, _I]),
    "rt_set_tree": (_I, [_P, _I]),
    "rt_build_lbvh": (_I, [_P, _P]),
    "rt_scene_size": (_I, [_P, _P, _P, _P]),
    "rt_read_indices": (_I, [_P, _P, _I]),
    "rt_set_schedule": (_I, [_P, _I]),
    "rt_set_latency_mode": (_I, [_P, _I]),
    "rt_set_kernel_timing": (_I, [_P, _I]),
    "rt_set_tail": (_I, [_P, _I]),
    "rt_status_string": (C.c_char_p, [_I]),
}

# include/rt_group.h (also in librtamd.so)
GROUP_SYMBOLS = {
    "rt_group_unique_id": (_I, [_P, C.c_size_t]),
    "rt_group_create": (_I, [_P, _P, _I, _I]),
    "rt_group_create_rank": (_I, [_P, _P, _I, _I, _I]),
    "rt_group_destroy": (_I, [_P]),
    "rt_group_info": (_I, [_P, _P, _P, _P]),
    "rt_group_member": (_I, [_P, _I, _P]),
    "rt_group_member_slot": (_I, [_P, _I, _I, _P]),
    "rt_group_set_frames": (_I, [_P, _I]),
    "rt_group_frames": (_I, [_P]),
    "rt_group_set_timeout": (_I, [_P, C.c_double]),
    "rt_group_set_phase_timing": (_I, [_P, _I]),
    "rt_group_set_sky_rows": (_I, [_P, _I]),
    "rt_group_sky_band": (_I, [_P, _P, _P]),
    "rt_group_check": (_I, [_P]),
    "rt_group_phase_times": (_I, [_P, _P]),
    "rt_group_upload_scene": (_I, [_P, _P, _I, _P, _I, _P, _I]),
    "rt_group_set_camera": (_I, [_P, _P]), "rt_group_set_light": (_I, [_P, _P]),
    "rt_group_set_params": (_I, [_P, _P]),
    "rt_group_update_shapes": (_I, [_P, _I, _I, _P]),
    "rt_group_update_nodes": (_I, [_P, _P, _I]),
    "rt_group_set_animated": (_I, [_P, _P, _I]), "rt_group_animate": (_I, [_P, _P]),
    "rt_group_dispatch": (_I, [_P, _I, _I, _I]),
    "rt_group_set_root_share": (_I, [_P, _I]),
    "rt_group_collect_stats": (_I, [_P, _I, _I, _I, _P]),
    "rt_group_sync": (_I, [_P]),
    "rt_group_read_image": (_I, [_P, _P, C.c_size_t, _I, _I]),
    "rt_group_device_image": (_I, [_P, _P, _P]),
}
GATHER_AUTO, GATHER_RCCL, GATHER_COPY = 0, 1, 2
FORMAT_RGBA32F, FORMAT_RGB32F, FORMAT_RGBA32F_IMAGE = 0, 1, 2  # rt_format
GROUP_ID_BYTES = 128


def _bind(lib, table, partial=False):
    """partial: skip symbols the library lacks (an older build compared by tools/ab.py)."""
    for name, (res, args) in table.items():
        if partial and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


def scene_lib():
    global _scene_lib
    if _scene_lib is None:
        _scene_lib = _bind(_load("librtscene.so"), SCENE_SYMBOLS)
    return _scene_lib


def rt_lib():
    global _rt_lib
    if _rt_lib is None:
        _rt_lib = _bind(_bind(_load("librtamd.so"), RT_SYMBOLS), GROUP_SYMBOLS)
    return _rt_lib


_host_lib = None


def host_lib():
    """librthost.so: rth_render_loop, the reference's render loop (src/main.cpp:290-462)
    as a C++ host over the C ABI (include/rt_host.h)."""
    global _host_lib
    if _host_lib is None:
        rt_lib()  # librtamd.so first: librthost.so links it
        _host_lib = _bind(_load("librthost.so"), HOST_SYMBOLS)
    return _host_lib


def update_bvh(fs, ids):
    """updateBVH (src/main.cpp:1068-1077) on the scene's arrays in place (librtscene.so
    rts_update_bvh): every node listing one of the shapes `ids` grows to hold its
    current record in fs.shapes."""
    ids = np.ascontiguousarray(ids, np.int32)
    rc = scene_lib().rts_update_bvh(_ptr(fs.shapes), len(fs.shapes), _ptr(fs.nodes), len(fs.nodes),
                                    _ptr(fs.indices), len(fs.indices), _ptr(ids), len(ids))
    if rc != 0:
        raise RTError("rts_update_bvh", rc)


class ReferenceUpload:
    """A host that keeps the reference's own per-frame upload of an animated scene
    (src/main.cpp:336-346): its own copies of the shape and node arrays, moved
    frame by frame; upload() is one rth_upload_animated (librthost.so): one
    rt_update_shapes per animated index, updateBVH on the host's nodes, one
    rt_update_nodes."""

    def __init__(self, fs, ids):
        self.shapes = as_records(fs.shapes, SHAPE_DTYPE).copy()
        self.nodes = as_records(fs.nodes, NODE_DTYPE).copy()
        self.indices = np.ascontiguousarray(fs.indices, np.int32)
        self.ids = np.ascontiguousarray(ids, np.int32)

    def upload(self, ctx, recs):
        """ctx: a ComputeShader (rth_upload_animated) or a Group (rth_group_upload_animated:
        every member and frame slot is given the calls)."""
        recs = as_records(np.asarray(recs).reshape(-1), SHAPE_DTYPE)
        fn = host_lib().rth_group_upload_animated if isinstance(ctx, Group) else host_lib().rth_upload_animated
        rc = fn(ctx._h, _ptr(self.shapes), len(self.shapes), _ptr(self.ids), _ptr(recs), len(self.ids),
                _ptr(self.nodes), len(self.nodes), _ptr(self.indices), len(self.indices))
        if rc != 0:
            raise RTError("rth_group_upload_animated" if isinstance(ctx, Group) else "rth_upload_animated", rc)

    def scene(self, fs):
        """The scene this host has uploaded (for the oracle)."""
        return FlatScene(self.shapes.copy(), self.nodes.copy(), self.indices, fs.camera, fs.light)


def render_loop(ctx, cams, light, width, height, dst_ptr, pitch, frames, wait_each=True, anim=None, ref=None):
    """rth_render_loop(_anim / _ref) on ComputeShader `ctx`: `frames` frames (camera cams[i % len]),
    each waited for (wait_each) or back to back; anim: a list of per-frame record
    arrays of the animated shapes, frame i animated with anim[i % len] first -- by
    rt_animate, or with `ref` (a ReferenceUpload) by the reference's own upload.
    Returns the host wall times in ms: one per frame, or [total] when not waiting."""
    cams = as_records(np.asarray(cams), CAMERA_DTYPE).reshape(-1)
    light = as_records(np.asarray(light), LIGHT_DTYPE).reshape(1)
    out = np.zeros(max(1, frames), np.float64)
    if ref is not None:
        recs = as_records(np.concatenate([np.asarray(f).reshape(-1) for f in anim]), SHAPE_DTYPE)
        rc = host_lib().rth_render_loop_ref(ctx._h, _ptr(cams), len(cams), _ptr(light), int(width), int(height),
                                            C.c_void_p(dst_ptr), int(pitch), int(frames), int(bool(wait_each)),
                                            _ptr(ref.shapes), len(ref.shapes), _ptr(ref.ids), len(ref.ids), _ptr(recs),
                                            len(anim), _ptr(ref.nodes), len(ref.nodes), _ptr(ref.indices),
                                            len(ref.indices), _ptr(out))
    elif anim is not None:
        recs = as_records(np.concatenate([np.asarray(f).reshape(-1) for f in anim]), SHAPE_DTYPE)
        per = len(np.asarray(anim[0]).reshape(-1))
        rc = host_lib().rth_render_loop_anim(ctx._h, _ptr(cams), len(cams), _ptr(light), int(width), int(height),
                                             C.c_void_p(dst_ptr), int(pitch), int(frames), int(bool(wait_each)),
                                             _ptr(recs), per, len(anim), _ptr(out))
    else:
        rc = host_lib().rth_render_loop(ctx._h, _ptr(cams), len(cams), _ptr(light), int(width), int(height),
                                        C.c_void_p(dst_ptr), int(pitch), int(frames), int(bool(wait_each)),
                                        _ptr(out))
    if rc != 0:
        raise RTError("rth_render_loop", rc)
    return out if wait_each else out[:1]


def render_rows_loop(ctx, cams, light, width, height, y0, stripe, period, out_rows, dst_ptr, pitch, frames,
                     wait_each=True, fmt=FORMAT_RGB32F):
    """rth_render_rows_loop: rth_render_loop over one rank's rows (rt_dispatch_rows_ex).
    Returns the host wall times in ms: one per frame, or [total] when not waiting."""
    cams = as_records(np.asarray(cams), CAMERA_DTYPE).reshape(-1)
    light = as_records(np.asarray(light), LIGHT_DTYPE).reshape(1)
    out = np.zeros(max(1, frames), np.float64)
    rc = host_lib().rth_render_rows_loop(ctx._h, _ptr(cams), len(cams), _ptr(light), int(width), int(height), int(y0),
                                         int(stripe), int(period), int(out_rows), int(fmt), C.c_void_p(dst_ptr),
                                         int(pitch), int(frames), int(bool(wait_each)), _ptr(out))
    if rc != 0:
        raise RTError("rth_render_rows_loop", rc)
    return out if wait_each else out[:1]


def _f3(v):
    return (C.c_float * 3)(*[float(x) for x in v])


def material(color=(1, 1, 1), fresnel=1.0, ambient=0.4, diffuse=1.0, specular=0.5, shininess=32):
    """Material(c, fresnel, ambient, diffuse, specular, shine) (src/material.hpp:23)."""
    m = np.zeros(1, MATERIAL_DTYPE)
    m["color"] = color
    m["fresnelStrength"] = fresnel
    m["ambientStrength"] = ambient
    m["diffuseStrength"] = diffuse
    m["specularStrength"] = specular
    m["shininess"] = shininess
    return m


# ---------------------------------------------------------------------------
@dataclass
class FlatScene:
    """serializeScene output: the five SSBO images (src/flatStructures.hpp:80-108)."""
    shapes: np.ndarray
    nodes: np.ndarray
    indices: np.ndarray
    camera: np.ndarray
    light: np.ndarray

    def __post_init__(self):
        self.shapes = as_records(self.shapes, SHAPE_DTYPE)
        self.nodes = as_records(self.nodes, NODE_DTYPE)
        self.indices = np.ascontiguousarray(self.indices, np.int32)
        self.camera = as_records(self.camera, CAMERA_DTYPE).reshape(1)
        self.light = as_records(self.light, LIGHT_DTYPE).reshape(1)


class Scene:
    """The reference's `Scene` (src/main.cpp:92-100) on the host scene library."""

    def __init__(self):
        self._lib = scene_lib()
        self._h = self._lib.rts_new()
        if not self._h:
            raise MemoryError("rts_new")

    def __del__(self):
        if getattr(self, "_h", None):
            self._lib.rts_free(self._h)
            self._h = None

    def _chk(self, rc, what):
        if rc < 0:
            raise RTError(what, rc)
        return rc

    @staticmethod
    def _mat(m):
        return _ptr(m) if m is not None else None

    def add_sphere(self, center, radius, mat=None):
        return self._chk(self._lib.rts_add_sphere(self._h, _f3(center), radius, self._mat(mat)), "add_sphere")

    def add_plane(self, normal, point, mat=None):
        return self._chk(self._lib.rts_add_plane(self._h, _f3(normal), _f3(point), self._mat(mat)), "add_plane")

    def add_wall(self, start, width, height, normal, mat=None):
        return self._chk(self._lib.rts_add_wall(self._h, _f3(start), width, height, _f3(normal), self._mat(mat)),
                         "add_wall")

    def add_triangle(self, a, b, c, invert=False, mat=None):
        return self._chk(self._lib.rts_add_triangle(self._h, _f3(a), _f3(b), _f3(c), int(invert), self._mat(mat)),
                         "add_triangle")

    def add_mesh(self, vertices, indices, origin=(0, 0, 0), mat=None, oriented=False):
        v = np.ascontiguousarray(vertices, np.float32).reshape(-1, 3)
        i = np.ascontiguousarray(indices, np.uint32).reshape(-1)
        fn = self._lib.rts_add_mesh_oriented if oriented else self._lib.rts_add_mesh
        return self._chk(fn(self._h, _ptr(v), len(v), _ptr(i), len(i), _f3(origin), self._mat(mat)), "add_mesh")

    def load_obj(self, path, origin=(0, 0, 0), mat=None, oriented=False):
        """Wavefront OBJ file -> triangles (rts_load_obj); returns the triangle count."""
        return self._chk(self._lib.rts_load_obj(self._h, os.fsencode(path), _f3(origin), self._mat(mat),
                                                int(bool(oriented))), "load_obj")

    def parse_obj(self, text, origin=(0, 0, 0), mat=None, oriented=False):
        b = text.encode() if isinstance(text, str) else bytes(text)
        return self._chk(self._lib.rts_parse_obj(self._h, b, len(b), _f3(origin), self._mat(mat),
                                                 int(bool(oriented))), "parse_obj")

    def set_camera(self, position, fov=60.0, aspect=1.0):
        self._chk(self._lib.rts_set_camera(self._h, _f3(position), fov, aspect), "set_camera")

    def LookAt(self, target):
        self._chk(self._lib.rts_camera_look_at(self._h, _f3(target)), "LookAt")

    def set_light(self, position, color=(1, 1, 1), intensity=1.0):
        self._chk(self._lib.rts_set_light(self._h, _f3(position), _f3(color), intensity), "set_light")

    def camera(self):
        """serializeCamera (src/main.cpp:806-816) alone."""
        cam = np.zeros(1, CAMERA_DTYPE)
        self._chk(self._lib.rts_serialize(self._h, None, None, None, _ptr(cam), None), "serializeCamera")
        return cam

    def orbit(self, target, degrees):
        """Turn the camera `degrees` about the vertical axis through `target` and
        look at `target` again (the weak bench mode's per-rank frames of an orbit).
        The rotation is done in float64 on the serialised position."""
        cam = self.camera()
        p = cam["Position"][0].astype(np.float64) - np.asarray(target, np.float64)
        ang = np.radians(float(degrees))
        q = (p[0] * np.cos(ang) + p[2] * np.sin(ang), p[1], -p[0] * np.sin(ang) + p[2] * np.cos(ang))
        self.set_camera(np.asarray(q) + np.asarray(target, np.float64), float(cam["fov"][0]),
                        float(cam["aspectRatio"][0]))
        self.LookAt(target)

    def buildBVH(self, maxDepth=15):
        self._chk(self._lib.rts_build_bvh(self._h, maxDepth), "buildBVH")

    def generate(self, config, variant=0, aspect=16 / 9):
        self._chk(self._lib.rts_generate(self._h, config, variant, aspect), "generate")
        return self

    def counts(self):
        s, n, i = C.c_int(), C.c_int(), C.c_int()
        self._chk(self._lib.rts_counts(self._h, C.byref(s), C.byref(n), C.byref(i)), "counts")
        return s.value, n.value, i.value

    def bvh_stats(self):
        v = [C.c_int() for _ in range(4)]
        self._chk(self._lib.rts_bvh_stats(self._h, *[C.byref(x) for x in v]), "bvh_stats")
        return dict(zip(["leaves", "max_leaf", "depth", "max_stack"], [x.value for x in v]))

    def serializeScene(self) -> FlatScene:
        s, n, i = self.counts()
        shapes = np.zeros(s, SHAPE_DTYPE)
        nodes = np.zeros(n, NODE_DTYPE)
        idx = np.zeros(i, np.int32)
        cam = np.zeros(1, CAMERA_DTYPE)
        light = np.zeros(1, LIGHT_DTYPE)
        self._chk(self._lib.rts_serialize(self._h, _ptr(shapes), _ptr(nodes), _ptr(idx), _ptr(cam), _ptr(light)),
                  "serializeScene")
        return FlatScene(shapes, nodes, idx, cam, light)


IMAGE_PPM, IMAGE_PFM = 0, 1


def write_image(path, img, fmt=IMAGE_PPM):
    """[H, W, 4] float32 image (row 0 = NDC y +1) -> binary PPM (clamped, 8-bit) or PFM (exact)."""
    a = np.ascontiguousarray(img, np.float32)
    if a.ndim != 3 or a.shape[2] != 4:
        raise ValueError("write_image expects [H, W, 4] float32")
    rc = scene_lib().rts_write_image(os.fsencode(path), _ptr(a), a.shape[1], a.shape[0], a.shape[1] * 16, int(fmt))
    if rc != 0:
        raise RTError("rts_write_image", rc)


def generate(config, variant=0, width=1920, height=1080) -> FlatScene:
    """One of the BASELINE configurations as serialised arrays."""
    sc = Scene().generate(config, variant, float(width) / float(height))
    return sc.serializeScene()


# ---------------------------------------------------------------------------
class ComputeShader:
    """The GPU operator: ComputeShader("gpu_shader.comp") + its SSBOs + uniforms
    (src/computeShader.hpp, src/main.cpp:238-370) on one HIP device."""

    def __init__(self, device=0, lib_path=None):
        # lib_path: another build of librtamd.so (A/B of two builds in one process, tools/ab.py)
        self._lib = rt_lib() if lib_path is None else _bind(C.CDLL(os.path.abspath(lib_path)), RT_SYMBOLS, partial=True)
        h = C.c_void_p()
        self._chk(self._lib.rt_create(C.byref(h), device), "rt_create")
        self._h = h
        self.device = device

    def close(self):
        if getattr(self, "_h", None):
            self._lib.rt_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    @staticmethod
    def _chk(rc, what):
        if rc != 0:
            raise RTError(what, rc)

    def set_stream(self, stream_handle):
        self._chk(self._lib.rt_set_stream(self._h, C.c_void_p(stream_handle) if stream_handle else None),
                  "rt_set_stream")

    def upload(self, fs: FlatScene):
        self._keep = fs
        self._chk(self._lib.rt_upload_scene(self._h, _ptr(fs.shapes), len(fs.shapes), _ptr(fs.nodes), len(fs.nodes),
                                            _ptr(fs.indices), len(fs.indices)), "rt_upload_scene")
        self.set_camera(fs.camera)
        self.set_light(fs.light)

    def update_shapes(self, first, shapes):
        shapes = as_records(shapes, SHAPE_DTYPE)
        self._chk(self._lib.rt_update_shapes(self._h, first, len(shapes), _ptr(shapes)), "rt_update_shapes")

    def update_nodes(self, nodes):
        nodes = as_records(nodes, NODE_DTYPE)
        self._chk(self._lib.rt_update_nodes(self._h, _ptr(nodes), len(nodes)), "rt_update_nodes")

    def set_animated(self, ids):
        """Marks the animated shapes (animatedIndices, src/main.cpp:120,706-708)."""
        ids = np.ascontiguousarray(ids, np.int32)
        self._n_animated = len(ids)
        self._chk(self._lib.rt_set_animated(self._h, _ptr(ids), len(ids)), "rt_set_animated")

    def animate(self, shapes):
        """New records of the animated shapes, in set_animated order: updateScene +
        updateBVH + serializeBVH + upload (src/main.cpp:336-346), on the device."""
        shapes = as_records(shapes, SHAPE_DTYPE)
        if len(shapes) != getattr(self, "_n_animated", -1):
            raise ValueError("animate: one record per animated shape")
        self._chk(self._lib.rt_animate(self._h, _ptr(shapes)), "rt_animate")

    def read_nodes(self, num_nodes):
        """The current node records (boxes grown by animate)."""
        out = np.zeros(num_nodes, NODE_DTYPE)
        self._chk(self._lib.rt_read_nodes(self._h, _ptr(out), num_nodes), "rt_read_nodes")
        return out

    def set_camera(self, cam):
        cam = as_records(cam, CAMERA_DTYPE)
        self._chk(self._lib.rt_set_camera(self._h, _ptr(cam)), "rt_set_camera")

    def set_light(self, light):
        light = as_records(light, LIGHT_DTYPE)
        self._chk(self._lib.rt_set_light(self._h, _ptr(light)), "rt_set_light")

    def set_params(self, resX, resY, maxBounces=3, useBVH=True, useFresnel=False, useMollerTrumbore=False):
        p = rt_params(float(resX), float(resY), int(maxBounces), int(bool(useBVH)), int(bool(useFresnel)),
                      int(bool(useMollerTrumbore)))
        self._chk(self._lib.rt_set_params(self._h, C.byref(p)), "rt_set_params")

    def set_kernel(self, kernel):
        self._chk(self._lib.rt_set_kernel(self._h, int(kernel)), "rt_set_kernel")

    def dispatch(self, width, height, y0=0, y1=None):
        self._chk(self._lib.rt_dispatch(self._h, width, height, y0, height if y1 is None else y1), "rt_dispatch")

    def dispatch_rows(self, width, height, y0, stripe, step, out_rows, dst_ptr, pitch):
        self._chk(self._lib.rt_dispatch_rows(self._h, width, height, y0, stripe, step, out_rows,
                                             C.c_void_p(dst_ptr), pitch), "rt_dispatch_rows")

    def dispatch_rows_rgb(self, width, height, y0, stripe, step, out_rows, dst_ptr, pitch):
        """rt_dispatch_rows_fmt with RT_FORMAT_RGB32F: packed 12-byte pixels."""
        self._chk(self._lib.rt_dispatch_rows_fmt(self._h, width, height, y0, stripe, step, out_rows,
                                                 C.c_void_p(dst_ptr), pitch, 1), "rt_dispatch_rows_fmt")

    def dispatch_rows_ex(self, width, height, y0, stripe, period, out_rows, dst_ptr, pitch, rgb=False, fmt=None):
        """rt_dispatch_rows_ex: stripes of `stripe` rows from y0, one every `period` rows.
        fmt: FORMAT_RGBA32F / FORMAT_RGB32F / FORMAT_RGBA32F_IMAGE (default: RGB32F if rgb)."""
        f = int(fmt) if fmt is not None else int(bool(rgb))
        self._chk(self._lib.rt_dispatch_rows_ex(self._h, width, height, y0, stripe, period, out_rows,
                                                C.c_void_p(dst_ptr), pitch, f), "rt_dispatch_rows_ex")

    def sync(self):
        self._chk(self._lib.rt_sync(self._h), "rt_sync")

    def sync_frame(self):
        """Waits for the last dispatch's frame (rt_sync_frame), not the renderer's order work behind it."""
        self._chk(self._lib.rt_sync_frame(self._h), "rt_sync_frame")

    def read_image(self, width, height):
        out = np.empty((height, width, 4), np.float32)
        self._chk(self._lib.rt_read_image(self._h, _ptr(out), width * 16, width, height), "rt_read_image")
        return out

    def render(self, width, height, y0=0, y1=None):
        """dispatch + barrier + readback of the full surface."""
        self.dispatch(width, height, y0, y1)
        self.sync()
        return self.read_image(width, height)

    def collect_stats(self, width, height, y0=0, stripe=1, step=1, out_rows=None):
        st = rt_stats()
        rows = height - y0 if out_rows is None else out_rows
        self._chk(self._lib.rt_collect_stats(self._h, width, height, y0, stripe, step, rows, C.byref(st)),
                  "rt_collect_stats")
        return st.as_dict()

    def kernel_times(self, cap=1024):
        """Device ms of each render dispatch since the last call (HIP events on the ctx stream)."""
        buf = np.zeros(cap, np.float32)
        n = self._lib.rt_kernel_times(self._h, _ptr(buf), cap)
        if n < 0:
            raise RTError("rt_kernel_times", n)
        return buf[:min(n, cap)].copy()

    def set_launch(self, waves_per_block=4, persistent=False):
        self._chk(self._lib.rt_set_launch(self._h, int(waves_per_block), int(bool(persistent))), "rt_set_launch")

    def set_walk(self, lane_from_depth):
        self._chk(self._lib.rt_set_walk(self._h, int(lane_from_depth)), "rt_set_walk")

    def build_lbvh(self):
        """Device LBVH over the current shapes (rt_build_lbvh); returns the build's device ms."""
        ms = C.c_float()
        self._chk(self._lib.rt_build_lbvh(self._h, C.byref(ms)), "rt_build_lbvh")
        return ms.value

    def scene_size(self):
        s, n, i = C.c_int(), C.c_int(), C.c_int()
        self._chk(self._lib.rt_scene_size(self._h, C.byref(s), C.byref(n), C.byref(i)), "rt_scene_size")
        return s.value, n.value, i.value

    def read_tree(self):
        """(nodes, indices) of the current scene tree as FlatNode records and int32."""
        _, n, i = self.scene_size()
        nodes = np.zeros(n, NODE_DTYPE)
        idx = np.zeros(i, np.int32)
        if n:
            self._chk(self._lib.rt_read_nodes(self._h, _ptr(nodes), n), "rt_read_nodes")
        self._chk(self._lib.rt_read_indices(self._h, _ptr(idx) if i else None, i), "rt_read_indices")
        return nodes, idx

    def set_tree(self, mode):
        """TREE_SCENE (default): one SAH tree over the reference leaves where exact; TREE_REFERENCE: the reference tree."""
        self._chk(self._lib.rt_set_tree(self._h, int(mode)), "rt_set_tree")

    def set_tail(self, from_bounce):
        """Bounces >= from_bounce of the rays still alive run compacted in a second kernel; 0 = off."""
        self._chk(self._lib.rt_set_tail(self._h, int(from_bounce)), "rt_set_tail")

    def debug_shadow_walk(self, from_bounce):
        fn = self._lib.rt_debug_shadow_walk
        fn.argtypes = [_P, _I]
        self._chk(fn(self._h, int(from_bounce)), "rt_debug_shadow_walk")

    def debug_tail_lanes(self, lanes):
        fn = self._lib.rt_debug_tail_lanes
        fn.argtypes = [_P, _I]
        self._chk(fn(self._h, int(lanes)), "rt_debug_tail_lanes")

    def set_kernel_timing(self, on):
        """rt_set_kernel_timing: record the device-time events around each dispatch (default on)."""
        self._chk(self._lib.rt_set_kernel_timing(self._h, int(bool(on))), "rt_set_kernel_timing")

    def set_latency_mode(self, on):
        """rt_set_latency_mode: tune for one frame at a time (split walks, heaviest tiles as 2 waves)."""
        self._chk(self._lib.rt_set_latency_mode(self._h, int(bool(on))), "rt_set_latency_mode")

    def set_schedule(self, mode):
        """SCHED_COST (default): tiles start longest-first by their last work; SCHED_COST_XCD: the same
        order dealt to the 8 XCDs as screen bands; SCHED_ROWS: row-major."""
        self._chk(self._lib.rt_set_schedule(self._h, int(mode)), "rt_set_schedule")

    def debug_scene_stack(self, n):
        """Diagnostics: cap the stack a scene-tree walk may use (0 = no cap); exact at any value."""
        fn = self._lib.rt_debug_scene_stack
        fn.argtypes = [C.c_void_p, C.c_int]
        self._chk(fn(self._h, int(n)), "rt_debug_scene_stack")

    def debug_sched_period(self, period):
        fn = self._lib.rt_debug_sched_period
        fn.argtypes = [_P, _I]
        self._chk(fn(self._h, int(period)), "rt_debug_sched_period")

    def debug_lane_stack(self, n):
        fn = self._lib.rt_debug_lane_stack
        fn.argtypes = [_P, _I]
        self._chk(fn(self._h, int(n)), "rt_debug_lane_stack")

    def debug_tile_order(self, order):
        fn = self._lib.rt_debug_tile_order
        fn.argtypes = [_P, _P, _I]
        o = np.ascontiguousarray(order if order is not None else [], np.int32)
        self._chk(fn(self._h, _ptr(o) if o.size else None, int(o.size)), "rt_debug_tile_order")

    def debug_anim_rebuilds(self):
        """Host rebuilds rt_animate fell back to since the context was made."""
        fn = self._lib.rt_debug_anim_rebuilds
        fn.argtypes = [_P]
        fn.restype = _I
        return int(fn(self._h))

    def debug_refit(self, mode):
        """rt_debug_refit: 0 one launch (box roles wait, by tickets), 1 two launches, 2 one launch
        (direct), 3 one launch (box roles wait, in start order), 4 as 2 from a device copy;
        -1 (the default) 2 for few records, else 1."""
        fn = self._lib.rt_debug_refit
        fn.argtypes = [_P, _I]
        fn.restype = _I
        self._chk(fn(self._h, int(mode)), "rt_debug_refit")

    def debug_refits(self):
        """Device refits that applied rt_update_shapes / rt_update_nodes / rt_animate
        without a host rebuild, since the context was made."""
        fn = self._lib.rt_debug_refits
        fn.argtypes = [_P]
        fn.restype = _I
        return int(fn(self._h))

    def debug_spec(self, mode):
        fn = self._lib.rt_debug_spec
        fn.argtypes = [_P, _I]
        self._chk(fn(self._h, int(mode)), "rt_debug_spec")

    def debug_split(self, max_rays, group=8):
        """Split per-lane walks of waves with <= max_rays rays over groups of <= group lanes (0: off)."""
        fn = self._lib.rt_debug_split
        fn.argtypes = [_P, _I, _I]
        self._chk(fn(self._h, int(max_rays), int(group)), "rt_debug_split")

    def debug_heavy(self, k, parts):
        """Run the k heaviest tiles of the cost order as `parts` waves each (parts 1: off)."""
        fn = self._lib.rt_debug_heavy
        fn.argtypes = [_P, _I, _I]
        self._chk(fn(self._h, int(k), int(parts)), "rt_debug_heavy")

    def debug_sched_order(self, n):
        """The current cost order's first n tiles (longest first); empty before one exists."""
        fn = self._lib.rt_debug_sched_order
        fn.argtypes = [_P, _P, _I]
        buf = np.zeros(max(n, 1), np.int32)
        k = fn(self._h, _ptr(buf), int(n))
        if k < 0:
            raise RTError("rt_debug_sched_order", k)
        return buf[:k].copy()

    def debug_refit_stats(self):
        """The refit's shape: dirty slots, largest / total prim range, nodes, entries."""
        fn = self._lib.rt_debug_refit_stats
        fn.argtypes = [_P, C.c_void_p]
        out = np.zeros(7, np.int64)
        self._chk(fn(self._h, out.ctypes.data), "rt_debug_refit_stats")
        return dict(zip(["dirty_slots", "max_range", "sum_range", "nodes", "entries", "flush_bytes", "compactions"],
                        out.tolist()))

    def debug_moving(self, period, dilate, split):
        """Cost order of dispatches whose camera moved: re-derived every `period` frames
        (0: as still frames), over costs dilated by `dilate` tiles, split tiles kept on
        its cost frames (`split`)."""
        fn = self._lib.rt_debug_moving
        fn.argtypes = [_P, _I, _I, _I]
        self._chk(fn(self._h, int(period), int(dilate), int(split)), "rt_debug_moving")

    def debug_order_stream(self, mode):
        """Where the cost order's kernels run: 0 the context's stream after the render,
        1 an order stream in latency-mode dispatches, 2 the order stream always."""
        fn = self._lib.rt_debug_order_stream
        fn.argtypes = [_P, _I]
        self._chk(fn(self._h, int(mode)), "rt_debug_order_stream")

    def debug_frame_event(self, on):
        """Latency-mode cost frames record the event rt_sync_frame waits for (1) or not (0)."""
        fn = self._lib.rt_debug_frame_event
        fn.argtypes = [_P, _I]
        self._chk(fn(self._h, int(on)), "rt_debug_frame_event")

    def debug_cost_dilate(self, r):
        """Cost order over each tile's largest cost within r tiles (0: off)."""
        fn = self._lib.rt_debug_cost_dilate
        fn.argtypes = [_P, _I]
        self._chk(fn(self._h, int(r)), "rt_debug_cost_dilate")

    def debug_cost_time(self, mode):
        """Cost-order measure: 1 the tiles' wave wall time, 0 their lanes' steps + tests, -1 default."""
        fn = self._lib.rt_debug_cost_time
        fn.argtypes = [_P, _I]
        self._chk(fn(self._h, int(mode)), "rt_debug_cost_time")

    def debug_lane_k(self, k, mode):
        """The first k dispatch slots walk camera rays (bit 0) / their shadows (bit 1) per lane."""
        fn = self._lib.rt_debug_lane_k
        fn.argtypes = [_P, _I, _I]
        self._chk(fn(self._h, int(k), int(mode)), "rt_debug_lane_k")

    def debug_cone_cull(self, on):
        fn = self._lib.rt_debug_cone_cull
        fn.argtypes = [_P, _I]
        self._chk(fn(self._h, int(bool(on))), "rt_debug_cone_cull")

    def debug_tile_times(self, cap):
        """cap > 0: enable per-tile stamps (diagnostics); then tile_times(cap) reads them."""
        fn = self._lib.rt_debug_tile_times
        fn.argtypes = [_P, _I, _P]
        self._chk(fn(self._h, int(cap), None), "rt_debug_tile_times")

    def tile_times(self, cap):
        """[n, 24] per-tile records of k_accel (layout: kTileRec in rt_kernels.hip)."""
        buf = np.zeros((cap, 24), np.uint64)
        fn = self._lib.rt_debug_tile_times
        fn.argtypes = [_P, _I, _P]
        n = fn(self._h, int(cap), _ptr(buf))
        if n < 0:
            raise RTError("rt_debug_tile_times", n)
        return buf[:n]

    def accel_info(self):
        a = rt_accel_info()
        self._chk(self._lib.rt_accel_info_get(self._h, C.byref(a)), "rt_accel_info_get")
        return {n: getattr(a, n) for n, _ in rt_accel_info._fields_}

    def last_kernel_ms(self):
        ms = C.c_float()
        self._chk(self._lib.rt_last_kernel_ms(self._h, C.byref(ms)), "rt_last_kernel_ms")
        return ms.value


# ---------------------------------------------------------------------------
def group_unique_id() -> bytes:
    """ncclGetUniqueId for rt_group_create_rank (rank 0 makes it, the others receive it)."""
    buf = (C.c_char * GROUP_ID_BYTES)()
    rc = rt_lib().rt_group_unique_id(buf, GROUP_ID_BYTES)
    if rc != 0:
        raise RTError("rt_group_unique_id", rc)
    return bytes(buf)


class _Member(ComputeShader):
    """A group member's context: owned (and destroyed) by its Group."""

    def __init__(self, lib, handle, device):
        self._lib = lib
        self._h = handle
        self.device = device

    def close(self):
        self._h = None


class GroupPhases(C.Structure):
    _fields_ = [("frames", C.c_int), ("render_ms", C.c_float), ("fanin_ms", C.c_float),
                ("unstripe_ms", C.c_float), ("frame_ms", C.c_float)]


class Group:
    """One frame over several GPUs (include/rt_group.h): interleaved row stripes
    per rank (rank 0 may take `share` stripes per period, set_root_share), gathered
    to rank 0 by one grouped ncclSend/ncclRecv per frame over xGMI (RCCL) or by
    device copies, then unstriped on rank 0.

    Group(devices=[0, 1, ...])            one process drives every device
    Group(uid=..., nranks=P, rank=r, device=d)   one process per GPU
    frames=F: F frames in flight (slots), one communicator and one fan-in stream.
    `members` holds each local member's slot-0 context, `contexts` every slot's.
    """

    def __init__(self, devices=None, transport=GATHER_AUTO, uid=None, nranks=None, rank=None, device=None,
                 frames=1):
        self._lib = rt_lib()
        h = C.c_void_p()
        if uid is not None:
            idb = (C.c_char * GROUP_ID_BYTES).from_buffer_copy(uid)
            self._chk(self._lib.rt_group_create_rank(C.byref(h), idb, int(nranks), int(rank), int(device)),
                      "rt_group_create_rank")
        else:
            d = np.ascontiguousarray(devices, np.int32)
            self._chk(self._lib.rt_group_create(C.byref(h), _ptr(d), len(d), int(transport)), "rt_group_create")
        self._h = h
        n, nl, tr = C.c_int(), C.c_int(), C.c_int()
        self._chk(self._lib.rt_group_info(h, C.byref(n), C.byref(nl), C.byref(tr)), "rt_group_info")
        self.nranks, self.nlocal, self.transport = n.value, nl.value, tr.value
        if frames != 1:
            self._chk(self._lib.rt_group_set_frames(h, int(frames)), "rt_group_set_frames")
        self.frames = self._lib.rt_group_frames(h)
        self.members, self.contexts = [], []
        for k in range(self.nlocal):
            dev = device if uid is not None else int(devices[k])
            for j in range(self.frames):
                c = C.c_void_p()
                self._chk(self._lib.rt_group_member_slot(h, k, j, C.byref(c)), "rt_group_member_slot")
                self.contexts.append(_Member(self._lib, c, dev))
                if j == 0:
                    self.members.append(self.contexts[-1])

    @staticmethod
    def _chk(rc, what):
        if rc != 0:
            raise RTError(what, rc)

    def close(self):
        if getattr(self, "_h", None):
            for m in self.contexts:
                m.close()
            self._lib.rt_group_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def upload(self, fs: FlatScene):
        self._keep = fs
        self._chk(self._lib.rt_group_upload_scene(self._h, _ptr(fs.shapes), len(fs.shapes), _ptr(fs.nodes),
                                                  len(fs.nodes), _ptr(fs.indices), len(fs.indices)),
                  "rt_group_upload_scene")
        self.set_camera(fs.camera)
        self.set_light(fs.light)

    def set_camera(self, cam):
        cam = as_records(cam, CAMERA_DTYPE)
        self._chk(self._lib.rt_group_set_camera(self._h, _ptr(cam)), "rt_group_set_camera")

    def set_light(self, light):
        light = as_records(light, LIGHT_DTYPE)
        self._chk(self._lib.rt_group_set_light(self._h, _ptr(light)), "rt_group_set_light")

    def set_params(self, resX, resY, maxBounces=3, useBVH=True, useFresnel=False, useMollerTrumbore=False):
        p = rt_params(float(resX), float(resY), int(maxBounces), int(bool(useBVH)), int(bool(useFresnel)),
                      int(bool(useMollerTrumbore)))
        self._chk(self._lib.rt_group_set_params(self._h, C.byref(p)), "rt_group_set_params")

    def dispatch(self, width, height, stripe=8):
        self._chk(self._lib.rt_group_dispatch(self._h, width, height, stripe), "rt_group_dispatch")

    # the reference's animated-frame upload on every member and frame slot (rt_group.h)
    def update_shapes(self, first, shapes):
        shapes = as_records(shapes, SHAPE_DTYPE)
        self._chk(self._lib.rt_group_update_shapes(self._h, first, len(shapes), _ptr(shapes)),
                  "rt_group_update_shapes")

    def update_nodes(self, nodes):
        nodes = as_records(nodes, NODE_DTYPE)
        self._chk(self._lib.rt_group_update_nodes(self._h, _ptr(nodes), len(nodes)), "rt_group_update_nodes")

    def set_animated(self, ids):
        """animatedIndices (src/main.cpp:120,706-708) on every member and frame slot."""
        ids = np.ascontiguousarray(ids, np.int32)
        self._n_animated = len(ids)
        self._chk(self._lib.rt_group_set_animated(self._h, _ptr(ids), len(ids)), "rt_group_set_animated")

    def animate(self, shapes):
        """The animated shapes' new records, in set_animated order: updateScene +
        updateBVH + upload (src/main.cpp:336-346) on the device of every member and slot."""
        shapes = as_records(shapes, SHAPE_DTYPE)
        if len(shapes) != getattr(self, "_n_animated", -1):
            raise ValueError("animate: one record per animated shape")
        self._chk(self._lib.rt_group_animate(self._h, _ptr(shapes)), "rt_group_animate")

    def set_root_share(self, share):
        """Rank 0's stripes per period of share + P - 1 (rt_group_set_root_share)."""
        self._chk(self._lib.rt_group_set_root_share(self._h, int(share)), "rt_group_set_root_share")

    def collect_stats(self, width, height, stripe=8):
        """Reference-walk totals of this process's members' rows (rt_group_collect_stats)."""
        st = rt_stats()
        self._chk(self._lib.rt_group_collect_stats(self._h, width, height, stripe, C.byref(st)),
                  "rt_group_collect_stats")
        return st.as_dict()

    def sync(self):
        """Bounded wait (rt_group_set_timeout); RTError -8 / -7 with the communicator aborted."""
        self._chk(self._lib.rt_group_sync(self._h), "rt_group_sync")

    def set_timeout(self, ms):
        self._chk(self._lib.rt_group_set_timeout(self._h, float(ms)), "rt_group_set_timeout")

    def check(self):
        """Non-blocking RCCL asynchronous-error poll (rt_group_check)."""
        self._chk(self._lib.rt_group_check(self._h), "rt_group_check")

    def set_sky_rows(self, on):
        """rt_group_set_sky_rows: keep background-only rows off the links (default on)."""
        self._chk(self._lib.rt_group_set_sky_rows(self._h, int(bool(on))), "rt_group_set_sky_rows")

    def sky_band(self):
        """The image rows [y0, y1) the last dispatch sent over the links (rt_group_sky_band)."""
        y0, y1 = C.c_int(), C.c_int()
        self._chk(self._lib.rt_group_sky_band(self._h, C.byref(y0), C.byref(y1)), "rt_group_sky_band")
        return y0.value, y1.value

    def device_image(self):
        """(pointer, pitch) of rank 0's surface of the last dispatched frame (rt_group_device_image):
        the frame after sync(), until `frames` more dispatches reuse the slot."""
        p, pitch = C.c_void_p(), C.c_size_t()
        self._chk(self._lib.rt_group_device_image(self._h, C.byref(p), C.byref(pitch)), "rt_group_device_image")
        return p.value, pitch.value

    def set_phase_timing(self, on):
        """rt_group_set_phase_timing: record the render / fan-in / unstripe events (default on)."""
        self._chk(self._lib.rt_group_set_phase_timing(self._h, int(bool(on))), "rt_group_set_phase_timing")

    def phase_times(self):
        """Mean device ms of render / fan-in / unstripe / whole frame since the last call."""
        p = GroupPhases()
        self._chk(self._lib.rt_group_phase_times(self._h, C.byref(p)), "rt_group_phase_times")
        return {"frames": p.frames, "render_ms": p.render_ms, "fanin_ms": p.fanin_ms,
                "unstripe_ms": p.unstripe_ms, "frame_ms": p.frame_ms}

    def read_image(self, width, height):
        out = np.empty((height, width, 4), np.float32)
        self._chk(self._lib.rt_group_read_image(self._h, _ptr(out), width * 16, width, height),
                  "rt_group_read_image")
        return out

    def render(self, width, height, stripe=8):
        self.dispatch(width, height, stripe)
        self.sync()
        return self.read_image(width, height)
