#!/usr/bin/env python3
"""Config 3 (60 s mono STFT): how much of the per-call time is host overhead.
Prints the host time per call of the Python wrapper and of the bare C entry
(ctypes), the event-timed back-to-back rate of each, and the per-call device
rate of 100 calls captured in one HIP graph and replayed."""
import ctypes as C
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vv-dsp_amd"))
import vvdsp_amd as vv  # noqa: E402

n, nfft, hop, burst = 60 * 48000, 1024, 256, 100
sig = torch.rand(1, n, device="cuda") * 2 - 1
st = vv.Stft(nfft, hop)
fr = st.frames(n)
out = torch.empty(1, fr, nfft, device="cuda")
byts = n * 4 + nfft * 4 + fr * nfft * 4
L = vv.lib()
s = torch.cuda.current_stream()
sp = C.c_void_p(s.cuda_stream)
nf = C.c_size_t(0)
raw = lambda: L.vv_dsp_stft_spectrogram_device(st.h, C.c_void_p(sig.data_ptr()), n, 1, n,  # noqa: E731
                                               C.c_void_p(out.data_ptr()), fr * nfft, sp, C.byref(nf))
py = lambda: st.spectrogram(sig, out=out)  # noqa: E731


def host_and_b2b(fn, reps=2000):
    for _ in range(50):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    host = (time.perf_counter() - t0) / reps
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(burst):
        fn()
    b.record(s)
    torch.cuda.synchronize()
    return host * 1e6, a.elapsed_time(b) / burst * 1e3


res = {}
for name, fn in (("python_wrapper", py), ("c_entry_ctypes", raw)):
    h, g = host_and_b2b(fn)
    res[name] = {"host_us_per_call": round(h, 2), "b2b_us_per_call": round(g, 2)}
ref = out.clone()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    sp = C.c_void_p(torch.cuda.current_stream().cuda_stream)   # the capture stream
    for _ in range(burst):
        raw()
for _ in range(5):
    g.replay()
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(10):
    g.replay()
b.record()
torch.cuda.synchronize()
per = a.elapsed_time(b) / (10 * burst) * 1e3
res["graph_100_calls"] = {"us_per_call": round(per, 2), "frac": round(byts / (per * 1e-6) / 8e12, 4),
                          "rows_equal": bool(torch.equal(out, ref))}
# one call's device time: a spin kernel ahead of the start event keeps the GPU
# busy while the host enqueues the call, so no host time lands between the events
ms = []
for _ in range(50):
    torch.cuda._sleep(200000)
    a.record(s)
    py()
    b.record(s)
    torch.cuda.synchronize()
    ms.append(a.elapsed_time(b) * 1e3)
ms.sort()
res["single_call_device_us"] = {"median": round(ms[len(ms) // 2], 2), "min": round(ms[0], 2)}
print(json.dumps(res))
