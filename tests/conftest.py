"""Shared test setup: the `gpu` marker, import paths, in-tree builds.

CPU tests (-m "not gpu") cover the oracle against the reference's golden
vectors, the host scene library, the C-ABI exports and the sharding logic;
-m gpu tests are the HIP parity tests and call through the C ABI.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "opengl-ray-tracer_amd")
sys.path.insert(0, PKG)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


# bench.py runs F = 3 frames in flight at 1080p on 2F hardware queues
# (bench.plan_inflight); the GPU tests that mirror it need the same, and HIP reads
# the count once, when the runtime starts (before any test touches the GPU).
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 6:
    os.environ["GPU_MAX_HW_QUEUES"] = "6"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


def _ensure_built():
    need = [os.path.join(PKG, "lib", "librtamd.so"), os.path.join(PKG, "lib", "librtscene.so"),
            os.path.join(ROOT, "oracle", "build", "liboracle.so")]
    if all(os.path.exists(p) for p in need):
        return
    subprocess.run(["make", "-s", "-j4", "-C", PKG], check=True)
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "build/liboracle.so"], check=True)


_ensure_built()


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(ROOT, "tests", "golden")
