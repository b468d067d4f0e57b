"""debug: which STFT output kind writes past the end of its rows (guard values)"""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "vv-dsp_amd"))
import vvdsp_amd as vv
for (nfft, hop, n) in [(1024, 256, 1280), (1024, 512, 20000), (1024, 256, 700), (1024, 256, 48333)]:
    nch = 3
    sig = torch.rand(nch, n, device="cuda") * 2 - 1
    st = vv.Stft(nfft, hop)
    fr = st.frames(n)
    for kind in ("pow", "mag", "cpx"):
        w = {"pow": nfft // 2 + 1, "mag": nfft, "cpx": 2 * nfft}[kind]
        buf = torch.full((nch * fr * w + 4096,), -7.0, device="cuda")
        o = buf[:nch * fr * w]
        if kind == "pow":
            st.power(sig, out=o.view(nch, fr, w))
        elif kind == "mag":
            st.spectrogram(sig, out=o.view(nch, fr, w))
        else:
            st.spectrogram(sig, out=o.view(torch.complex64).view(nch, fr, nfft), complex_out=True)
        torch.cuda.synchronize()
        t = buf[nch * fr * w:].cpu().numpy()
        bad = np.nonzero(t != -7.0)[0]
        print(nfft, hop, n, fr, kind, "overrun floats:", len(bad), bad[:3], bad[-3:] if len(bad) else "")
