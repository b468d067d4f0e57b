#!/usr/bin/env python3
"""Check that a timing-lab STFT variant (scripts/stftlab.hip, EXP bits that keep
the results exact) writes the same rows as the lab's EXP 0 (the library's kernel).
    python scripts/labcheck.py 8192 [nch] [seconds]"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vv-dsp_amd"))
import vvdsp_amd as vv  # noqa: E402

if sys.argv[1] == "firr32":   # python scripts/labcheck.py firr32 <EXP>: k_fir_r32 variant vs EXP 0 (every output)
    e = int(sys.argv[2])
    lib = ctypes.CDLL(os.path.join(ROOT, "scripts", "libstftlab.so"))
    lib.firr32lab_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                  ctypes.c_longlong, ctypes.c_longlong, ctypes.c_void_p]
    worst = 0.0
    for nch, n in ((3, (1 << 20) + 12346), (1, 768 * 6), (2, 700), (5, 1540), (7, 768 * 41 + 2)):
        x = torch.rand(nch, n, device="cuda") * 2 - 1
        H = torch.complex(torch.rand(1024, device="cuda"), torch.rand(1024, device="cuda"))
        s = torch.cuda.current_stream().cuda_stream
        ref = torch.full_like(x, -2.0)
        assert lib.firr32lab_run(0, H.data_ptr(), x.data_ptr(), ref.data_ptr(), n, nch, s) == 0
        for rep in range(2):
            out = torch.full_like(x, -1.0)
            assert lib.firr32lab_run(e, H.data_ptr(), x.data_ptr(), out.data_ptr(), n, nch, s) == 0
            torch.cuda.synchronize()
            ne = out != ref
            bad = ne.sum().item()
            d = (out - ref).abs().max().item()
            worst = max(worst, d / ref.abs().max().item())
            print(f"firr32lab{e} ({nch} x {n}) launch {rep}: {bad} of {out.numel()} values differ, max |diff| {d:.3g} "
                  f"(max |y| {ref.abs().max().item():.3g}), first at {ne.nonzero()[:5].tolist()}")
    assert worst <= 1e-5, worst
    sys.exit(0)

if sys.argv[1] == "fir":   # python scripts/labcheck.py fir <EXP>: k_fir_bulk_reg variant vs EXP 0
    e = int(sys.argv[2])
    lib = ctypes.CDLL(os.path.join(ROOT, "scripts", "libstftlab.so"))
    lib.firreglab_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                  ctypes.c_longlong, ctypes.c_longlong, ctypes.c_void_p]
    nch, n = 3, (1 << 20) + 12345
    x = torch.rand(nch, n, device="cuda") * 2 - 1
    H = torch.complex(torch.rand(1024, device="cuda"), torch.rand(1024, device="cuda"))
    s = torch.cuda.current_stream().cuda_stream
    ref = torch.full_like(x, -2.0)
    assert lib.firreglab_run(0, H.data_ptr(), x.data_ptr(), ref.data_ptr(), n, nch, s) == 0
    for rep in range(2):
        out = torch.full_like(x, -1.0)
        assert lib.firreglab_run(e, H.data_ptr(), x.data_ptr(), out.data_ptr(), n, nch, s) == 0
        torch.cuda.synchronize()
        # the lab launch covers the bulk pairs only (the edge pairs' outputs stay -2 / -1)
        ref_w = ref != -2.0
        out = torch.where(ref_w, out, ref)
        ne = out != ref
        bad = ne.sum().item()
        d = (out - ref).abs().max().item()
        idx = ne.nonzero()[:5].tolist()
        print(f"firreglab{e} launch {rep}: {bad} of {out.numel()} values differ, max |diff| {d:.3g} "
              f"(max |y| {ref.abs().max().item():.3g}), first at {idx}")
        assert d <= 1e-5 * ref.abs().max().item()   # same arithmetic, possibly other contractions
    sys.exit(0)
# python scripts/labcheck.py [pow|lab5] <EXP> [nch] [seconds]: the power-row (stftpowlab_run) or
# VAR 5 magnitude (stftlab5_run) lab launch instead of stftlab_run
fn, row = "stftlab_run", 1024
if sys.argv[1] in ("pow", "lab5"):
    fn, row = ("stftpowlab_run", 513) if sys.argv[1] == "pow" else ("stftlab5_run", 1024)
    sys.argv.pop(1)
e = int(sys.argv[1])
nch = int(sys.argv[2]) if len(sys.argv) > 2 else 4
sec = int(sys.argv[3]) if len(sys.argv) > 3 else 60
lib = ctypes.CDLL(os.path.join(ROOT, "scripts", "libstftlab.so"))
getattr(lib, fn).argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_longlong, ctypes.c_longlong,
                             ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
lib.stftlab_run = getattr(lib, fn)
n = sec * 48000
sig = torch.rand(nch, n, device="cuda") * 2 - 1
win = torch.hann_window(1024, periodic=False, device="cuda")
frames = (n - 1024 + 256) // 256 + 1
ref = torch.full((nch, frames, row), -2.0, device="cuda")
assert lib.stftlab_run(0, sig.data_ptr(), n, nch, win.data_ptr(), ref.data_ptr(),
                       torch.cuda.current_stream().cuda_stream) == 0
out = torch.full_like(ref, -1.0)
for rep in range(3):   # the counters must reset between launches
    out.fill_(-1.0)
    assert lib.stftlab_run(e, sig.data_ptr(), n, nch, win.data_ptr(), out.data_ptr(),
                           torch.cuda.current_stream().cuda_stream) == 0
    torch.cuda.synchronize()
    bad = (out != ref).sum().item()
    print(f"lab{e} launch {rep}: {bad} of {out.numel()} values differ")
    assert bad == 0
