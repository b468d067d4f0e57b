"""The HIP vtable as a slot in the REFERENCE's own dispatcher.

The reference's vv_dsp_fft_make_plan mallocs exactly sizeof(struct
vv_dsp_fft_plan) -- 32 bytes on LP64 (src/spectral/fft_backend.h:17-29,
src/spectral/fft.c:76-83) -- and hands it to vtable->make_plan.  These tests
allocate plans the same way, with the bytes past the struct poisoned, and drive
vv_dsp_fft_hip_vtable.make_plan / execute / free_plan directly:
  * the output matches the oracle (a single transform: a stray read of the
    poison as a batch count would copy ~10^18 transforms and fault),
  * device memory does not grow over 1,000 create / execute / destroy cycles
    (the reference's vv_dsp_fft_backend_free is a no-op, fft_kiss.c:211-216;
    INTEGRATION.md section 2 routes destroy through the slot's free_plan).
The CPU test pins the struct layout against the reference header itself.
"""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, tolerances
from vvapi import C2C, R2C, FWD, BWD, HIP, OK

REF = "/root/reference"

_MAKE = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_void_p))
_EXEC = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p)
_FREE = C.CFUNCTYPE(None, C.c_void_p)
_AVAIL = C.CFUNCTYPE(C.c_int)


class Vtable(C.Structure):      # fft_backend.h:32-38
    _fields_ = [("make_plan", _MAKE), ("execute", _EXEC), ("free_plan", _FREE),
                ("is_available", _AVAIL), ("name", C.c_char_p)]


PLAN_BYTES = 32                 # sizeof(struct vv_dsp_fft_plan), pinned by test_plan_layout_matches_reference
POISON = 0xAB


def _ref_plan(n, kind, direction):
    """A heap block laid out as fft.c:76-83 fills it, followed by 32 poisoned bytes."""
    buf = (C.c_uint8 * (2 * PLAN_BYTES))()
    C.memset(buf, POISON, 2 * PLAN_BYTES)
    C.c_size_t.from_buffer(buf, 0).value = n
    C.c_int.from_buffer(buf, 8).value = kind
    C.c_int.from_buffer(buf, 12).value = direction
    C.c_int.from_buffer(buf, 16).value = HIP
    C.c_void_p.from_buffer(buf, 24).value = None
    return buf


_LAYOUT_SRC = r"""
#include <stdio.h>
#include <stddef.h>
#include "fft_backend.h"
int main(void) {
    printf("%zu %zu %zu %zu %zu %zu\n", sizeof(struct vv_dsp_fft_plan),
           offsetof(struct vv_dsp_fft_plan, n), offsetof(struct vv_dsp_fft_plan, type),
           offsetof(struct vv_dsp_fft_plan, dir), offsetof(struct vv_dsp_fft_plan, backend),
           offsetof(struct vv_dsp_fft_plan, backend_plan));
    return 0;
}
"""


def _layout(tmp_path, tag, incs):
    src = tmp_path / f"{tag}.c"
    src.write_text(_LAYOUT_SRC)
    exe = tmp_path / tag
    subprocess.run(["gcc", "-std=gnu99", *[f"-I{i}" for i in incs], str(src), "-o", str(exe)], check=True)
    return subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()


def test_plan_layout_matches_reference(tmp_path):
    ours = _layout(tmp_path, "ours", [os.path.join(ROOT, "vv-dsp_amd", "csrc", "host"), os.path.join(ROOT, "include")])
    assert ours == [str(PLAN_BYTES), "0", "8", "12", "16", "24"], ours
    if not os.path.isdir(os.path.join(REF, "src", "spectral")):
        pytest.skip("reference tree absent (GPU box): layout pinned by the constants above")
    theirs = _layout(tmp_path, "theirs", [os.path.join(REF, "src", "spectral"), os.path.join(REF, "include")])
    assert ours == theirs


@pytest.fixture(scope="module")
def vtab(amd):
    return Vtable.in_dll(amd.lib, "vv_dsp_fft_hip_vtable")


@pytest.mark.gpu
@pytest.mark.parametrize("kind,direction", [(C2C, FWD), (C2C, BWD), (R2C, FWD)])
def test_vtable_on_reference_sized_plan(amd, orc, vtab, kind, direction):
    assert vtab.is_available() == 1 and vtab.name == b"HIP-gfx950"
    n = 1024
    rng = np.random.default_rng(11)
    if kind == C2C:
        x = (rng.uniform(-0.5, 0.5, n) + 1j * rng.uniform(-0.5, 0.5, n)).astype(np.complex64)
        xin = x.view(np.float32)
        out = np.full(2 * n + 64, np.float32(7.0), np.float32)    # tail sentinel: nothing past one transform
        nout = 2 * n
    else:
        x = rng.uniform(-1, 1, n).astype(np.float32)
        xin = x
        out = np.full(2 * (n // 2 + 1) + 64, np.float32(7.0), np.float32)
        nout = 2 * (n // 2 + 1)
    spec = _ref_plan(n, kind, direction)
    bd = C.c_void_p()
    assert vtab.make_plan(C.addressof(spec), C.byref(bd)) == OK
    assert bd.value
    assert bytes(spec)[PLAN_BYTES:] == bytes([POISON]) * PLAN_BYTES      # the vtable wrote nothing past the plan
    try:
        assert vtab.execute(C.addressof(spec), bd, xin.ctypes.data, out.ctypes.data) == OK
    finally:
        vtab.free_plan(bd)
    assert np.all(out[nout:] == np.float32(7.0))
    y = out[:nout].view(np.complex64)
    kiss = orc.fft(x, kind, direction)
    x64 = x.astype(np.complex128) if kind == C2C else x.astype(np.float64)
    f64 = np.fft.fft(x64) if direction == FWD else np.fft.ifft(x64)
    if kind == R2C:
        f64 = np.fft.rfft(x64)
    r, a = tolerances()
    np.testing.assert_allclose(y, f64, rtol=r, atol=a)
    np.testing.assert_allclose(y, kiss, rtol=2 * r, atol=2 * a)


@pytest.mark.gpu
def test_vtable_create_destroy_does_not_leak(amd, vtab):
    import torch
    n = 1024
    x = np.ones(2 * n, np.float32)
    out = np.zeros(2 * n, np.float32)

    def cycle():
        spec = _ref_plan(n, C2C, FWD)
        bd = C.c_void_p()
        assert vtab.make_plan(C.addressof(spec), C.byref(bd)) == OK
        assert vtab.execute(C.addressof(spec), bd, x.ctypes.data, out.ctypes.data) == OK
        vtab.free_plan(bd)

    for _ in range(10):
        cycle()                       # per-device tables are cached once
    torch.cuda.synchronize()
    free0 = torch.cuda.mem_get_info()[0]
    for _ in range(1000):
        cycle()
    torch.cuda.synchronize()
    free1 = torch.cuda.mem_get_info()[0]
    assert free0 - free1 < (4 << 20), (free0, free1)
    assert out[0] == np.float32(n) and out[1] == np.float32(n)    # the impulse-dual: DC of all-ones = n
    vtab.free_plan(None)              # NULL backend data is accepted, as Kiss's free is


@pytest.mark.gpu
def test_dispatcher_destroy_frees_device_memory(amd):
    """Our own dispatcher: make_plan_many(batch) -> destroy returns the staging."""
    import torch
    L = amd.lib
    L.vv_dsp_fft_make_plan_many.argtypes = [C.c_size_t, C.c_int, C.c_int, C.c_size_t, C.POINTER(C.c_void_p)]
    x = np.zeros(2 * 1024 * 4096, np.float32)
    x[0::2048] = 1.0
    y = np.empty_like(x)

    def cycle():
        p = C.c_void_p()
        assert L.vv_dsp_fft_make_plan_many(1024, C2C, FWD, 4096, C.byref(p)) == OK
        assert L.vv_dsp_fft_execute(p, x.ctypes.data, y.ctypes.data) == OK
        assert L.vv_dsp_fft_destroy(p) == OK

    for _ in range(3):
        cycle()                   # per-device tables and the host-path staging pool are cached once
    torch.cuda.synchronize()
    free0 = torch.cuda.mem_get_info()[0]
    for _ in range(200):          # a 32 MiB batch per plan: a per-plan leak would show as >= 6 GiB
        cycle()
    assert np.allclose(y.view(np.complex64).reshape(4096, 1024), 1.0)
    torch.cuda.synchronize()
    assert free0 - torch.cuda.mem_get_info()[0] < (4 << 20)
