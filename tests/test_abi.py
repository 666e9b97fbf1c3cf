"""The C-ABI libraries load and export every entry point include/*.h declares
(no compute calls: this runs without a GPU)."""
import ctypes as C
import os
import re
import subprocess

import pytest

import rtamd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DECL = re.compile(r"^\s*(?:const\s+)?(?:int|void|char|struct\s+\w+)\s*\*?\s*(r[a-z]*_\w+)\s*\(", re.M)


def declared(header):
    with open(os.path.join(ROOT, "include", header)) as f:
        text = re.sub(r"/\*.*?\*/", "", f.read(), flags=re.S)
    return sorted(set(DECL.findall(text)))


TABLES = {"rt_api.h": ("librtamd.so", rtamd.RT_SYMBOLS), "rt_group.h": ("librtamd.so", rtamd.GROUP_SYMBOLS),
          "rt_scene.h": ("librtscene.so", rtamd.SCENE_SYMBOLS), "rt_host.h": ("librthost.so", rtamd.HOST_SYMBOLS)}
MIN_ENTRIES = {"rt_host.h": 1}


@pytest.mark.parametrize("header", sorted(TABLES))
def test_exports(header):
    lib, table = TABLES[header]
    names = declared(header)
    assert len(names) >= MIN_ENTRIES.get(header, 12), names
    so = C.CDLL(os.path.join(rtamd.LIBDIR, lib))
    missing = [n for n in names if not hasattr(so, n)]
    assert not missing, missing
    assert sorted(table) == names, "binding table out of sync with the header"


def test_status_strings():
    lib = rtamd.rt_lib()
    for code in range(0, -9, -1):
        assert lib.rt_status_string(code).decode() == rtamd.STATUS[code]


def test_no_device_fails_loudly():
    """Without a HIP device rt_create must fail with a status, never crash."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(rtamd.RTError) as e:
        rtamd.ComputeShader(0)
    assert e.value.code in (-6, -2)


def test_kernel_is_gfx950():
    """The HIP code object inside librtamd.so targets gfx950."""
    with open(os.path.join(rtamd.LIBDIR, "librtamd.so"), "rb") as f:
        blob = f.read()
    assert b"gfx950" in blob


def test_group_wait_is_bounded():
    """rt_group_sync's poll loop (csrc/group_wait.h) on the CPU with fake queries:
    completion, a fan-in that never completes (the deadline fires instead of a
    hang), an RCCL asynchronous error and a device error (tests/native/wait_check.cpp)."""
    exe = os.path.join(ROOT, "tests", "native", "build", "wait_check")
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "native"), "build/wait_check"], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "wait_check ok" in r.stdout


def test_sky_rows_band_is_conservative():
    """rt_group's sky-row band (csrc/sky_rows.h): over 3,000 random cameras and root
    boxes, every pixel of every row it calls background has a camera ray (getRay in
    float, as the kernels) that misses the box under the GLSL slab test
    (tests/native/sky_check.cpp)."""
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "native"), "build/sky_check"], check=True)
    r = subprocess.run([os.path.join(ROOT, "tests", "native", "build", "sky_check")], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "sky_check ok" in r.stdout and " 0 violations" in r.stdout
