"""Shared test setup. `-m gpu` tests need a real MI355X and the built HIP library;
everything else runs on the CPU (oracle, host logic, ABI exports)."""
import os
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "julia-raytracer_amd"))
sys.path.insert(0, str(ROOT / "oracle"))
sys.path.insert(0, str(ROOT))

CORNELL = str(ROOT / "assets" / "scenes" / "cornellbox" / "cornellbox.json")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD GPU (MI355X) and the built HIP library")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def abi():
    from jtrace import abi as _abi
    return _abi


@pytest.fixture(scope="session")
def lib(abi):
    return abi.load_library()


@pytest.fixture
def options(abi, lib):
    """Setter of the library's run-time options (jt_set_option) for contexts the test creates;
    every option is removed again when the test ends."""
    def set_(name, value):
        abi.set_option(lib, name, value)
    yield set_
    abi.set_option(lib, None, None)


@pytest.fixture(scope="session")
def oracle(abi):
    from oracle import Oracle
    return Oracle(abi)


@pytest.fixture(scope="session")
def cornell():
    from jtrace import sceneio
    return sceneio.load_scene(CORNELL)


@pytest.fixture(scope="session")
def cornell_abi(abi, cornell):
    return abi.SceneABI(cornell)


def make_params(abi, **kw):
    from jtrace.cli import Params
    # tests name the traversal the oracle restates: near unless a test asks for another
    # (the product default "auto" is resolved by the library; tests/test_gpu_traversal.py covers it)
    d = dict(scene="", resolution=64, samples=8, bounces=8, sampler=1, clamp=10, envhidden=False,
             tentfilter=False, nocaustics=False, batch=1, bvhstacksize=128, seed=0x5EED, traversal="near")
    d.update(kw)
    cam = d.pop("camera", 0)
    return abi.make_params(Params(**d), cam)


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu(lib):
    import ctypes as C
    n = C.c_int32()
    st = lib.jt_device_count(C.byref(n))
    if st != 0 or n.value < 1:
        pytest.fail("gpu test requested but no HIP device is visible")
    return n.value


def compare_images(a, b):
    """Per-pixel comparison statistics between two (H, W, C) float images."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    d = np.abs(a - b)
    scale = np.maximum(np.abs(a), np.abs(b))
    rel = np.where(scale > 0, d / np.maximum(scale, 1e-6), 0)
    pix_rel = rel.reshape(rel.shape[0] * rel.shape[1], -1).max(axis=1)
    return {
        "max_abs": float(d.max()),
        "mean_abs": float(d.mean()),
        "bitwise_frac": float(np.mean(np.all((a == b).reshape(pix_rel.shape[0], -1), axis=1))),
        "frac_pix_rel_le_1e-3": float(np.mean(pix_rel <= 1e-3)),
        "image_mean_rel": float(abs(a.mean() - b.mean()) / max(abs(b.mean()), 1e-12)),
    }
