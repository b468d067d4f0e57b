#!/usr/bin/env python3
"""A/B variants of the register STFT kernel (VVHIP_MIX_VAR) must write the
same rows as the default, bit for bit: magnitude and complex rows at every
register length, an odd frame count (a missing second frame) included.
    python scripts/sqcheck.py [var]"""
import os
import sys


import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vv-dsp_amd"))
import vvdsp_amd as vv  # noqa: E402

var = sys.argv[1] if len(sys.argv) > 1 else "1"
g = torch.Generator(device="cuda").manual_seed(5)
for nf in (320, 400, 441, 480, 600, 640, 720, 800, 900, 960):
    st = vv.Stft(nf, nf // 4)
    for n in (3 * 48000 + 77, 48000):
        sig = torch.rand(3, n, device="cuda", generator=g) * 2 - 1
        for cpx in (False, True):
            a = st.spectrogram(sig, complex_out=cpx).clone()
            with vv.knobs(MIX_VAR=int(var)):   # the registry knob (csrc/hip/debug.hip), set per call
                b = st.spectrogram(sig, complex_out=cpx)
            torch.cuda.synchronize()
            bad = (a != b).sum().item()
            print(f"nfft {nf} n {n} {'complex' if cpx else 'magnitude'} frames {a.shape[1]}: {bad} differ")
            assert bad == 0
print("sqcheck ok")
