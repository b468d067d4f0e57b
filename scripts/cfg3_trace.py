#!/usr/bin/env python3
"""Config 3 (60 s mono STFT, 11,248 frames) timed the bench's way -- HIP events
around each of 50 single calls, then 100 calls back to back -- for a rocprofv3
kernel trace of the same process (kernel duration vs event time)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vv-dsp_amd"))
import vvdsp_amd as vv  # noqa: E402

n = 60 * 48000
sig = torch.rand(1, n, device="cuda") * 2 - 1
st = vv.Stft(1024, 256)
out = torch.empty(1, st.frames(n), 1024, device="cuda")
s = torch.cuda.current_stream()
for _ in range(200):
    st.spectrogram(sig, out=out)
torch.cuda.synchronize()
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(50)]
for a, b in ev:
    a.record(s)
    st.spectrogram(sig, out=out)
    b.record(s)
torch.cuda.synchronize()
single = sorted(a.elapsed_time(b) * 1e3 for a, b in ev)
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record(s)
for _ in range(100):
    st.spectrogram(sig, out=out)
b.record(s)
torch.cuda.synchronize()
print({"single_us_median": round(single[25], 2), "single_us_min": round(single[0], 2),
       "b2b_us_per_call": round(a.elapsed_time(b) * 10, 2)})
