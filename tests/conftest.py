"""Shared fixtures.  `-m gpu` tests need an MI355X; everything else runs on CPU."""
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TESTS = os.path.join(ROOT, "tests")
GOLDEN = os.path.join(TESTS, "golden")
REF_LIB = os.path.join(ROOT, "oracle", "_ref", "libvvref.so")
ORACLE_LIB = os.path.join(ROOT, "oracle", "liboracle.so")
AMD_DIR = os.path.join(ROOT, "vv-dsp_amd")
AMD_LIB = os.path.join(AMD_DIR, "lib", "libvvdsp_amd.so")

for p in (TESTS, AMD_DIR):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; run with -m gpu")


def tolerances(default_rtol=5e-5, default_atol=5e-5):
    """The reference harness convention (python/common.py:34-46): VV_PY_RTOL / VV_PY_ATOL."""
    def env(name, d):
        try:
            return float(os.environ.get(name, d))
        except ValueError:
            return d
    return env("VV_PY_RTOL", default_rtol), env("VV_PY_ATOL", default_atol)


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        manifest = json.load(f)

    def load(name):
        assert name in manifest, name
        with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
            return {k: z[k] for k in z.files}
    return load


@pytest.fixture(scope="session")
def orc():
    from vvapi import Oracle
    if not os.path.exists(ORACLE_LIB):
        pytest.fail("oracle/liboracle.so missing: run `make -C oracle`")
    return Oracle(ORACLE_LIB)


@pytest.fixture(scope="session")
def ref():
    from vvapi import VvDsp
    if not os.path.exists(REF_LIB):
        pytest.skip("oracle/_ref/libvvref.so not built (needs /root/reference)")
    return VvDsp(REF_LIB)


@pytest.fixture(scope="session")
def amd_lib_path():
    if not os.path.exists(AMD_LIB):
        pytest.fail("vv-dsp_amd/lib/libvvdsp_amd.so missing: run `make -C vv-dsp_amd`")
    return AMD_LIB


@pytest.fixture(scope="session")
def amd(amd_lib_path):
    """The product library through the reference's own C API (host pointers)."""
    import torch  # noqa: F401  -- one HIP runtime in the process (torch's)
    from vvapi import VvDsp
    lib = VvDsp(amd_lib_path)
    if lib.lib.vvhip_available() <= 0:
        pytest.fail("no HIP device visible to libvvdsp_amd.so")
    return lib


@pytest.fixture(scope="session")
def vdev(amd_lib_path):
    """Device-pointer API binding (vv-dsp_amd/vvdsp_amd.py)."""
    import torch
    import vvdsp_amd
    if not torch.cuda.is_available() or vvdsp_amd.device_count() <= 0:
        pytest.fail("GPU tests need an MI355X")
    return vvdsp_amd


@pytest.fixture
def knob():
    """knob("STFT_DYN", 0): select a launcher alternative of the product library
    (vvhip_debug_set, csrc/hip/debug.hip) for this test; every knob the test set
    is cleared at teardown.  "" / None clears at once."""
    import vvdsp_amd as vv
    touched = []

    def setter(name, value):
        name = name[6:] if name.startswith("VVHIP_") else name
        if value in ("", None):
            vv.debug_clear(name)
        else:
            vv.debug_set(name, int(value))
            touched.append(name)
    yield setter
    for n in touched:
        vv.debug_clear(n)
