#!/usr/bin/env python3
"""Host-buffer (PCIe-inclusive) rates of the reference's own C API on one MI355X.

The reference API (fft.h, stft.h) takes host pointers, so a drop-in caller
pays the host<->device copies on every call.  This measures, through
libvvdsp_amd.so's vv_dsp_* symbols with NumPy host buffers:

  * the PCIe ceiling: torch pageable / pinned H2D and D2H of the same sizes;
  * vv_dsp_stft_spectrogram, 60 s mono @ 48 kHz, 1024 Hann, hop 256 (config 3):
    11.5 MB in, 46 MB out per call;
  * vv_dsp_fft_execute on a 65536 x 1024 c2c plan (vv_dsp_fft_make_plan_many,
    config 2 with host buffers): 512 MiB in, 512 MiB out;
  * vv_dsp_fft_execute, one 1024-pt c2c per call (the reference's call shape):
    per-call latency.

    python scripts/hostbench.py [--json out.json]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vv-dsp_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import vvdsp_amd as vv  # noqa: E402
from vvapi import VvDsp, StftParams, C2C, FWD  # noqa: E402


def timeit(fn, reps, warm=2):
    for _ in range(warm):
        fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)), float(np.min(ts))


def copy_rates(nbytes, reps=5):
    d = torch.empty(nbytes // 4, device="cuda")
    hp = torch.empty(nbytes // 4, pin_memory=True)
    hn = torch.from_numpy(np.ones(nbytes // 4, np.float32))
    r = {}
    for name, h in (("pageable", hn), ("pinned", hp)):
        def h2d():
            d.copy_(h, non_blocking=False)
            torch.cuda.synchronize()

        def d2h():
            h.copy_(d, non_blocking=False)
            torch.cuda.synchronize()
        r[f"h2d_{name}_GBs"] = round(nbytes / timeit(h2d, reps)[0] / 1e9, 2)
        r[f"d2h_{name}_GBs"] = round(nbytes / timeit(d2h, reps)[0] / 1e9, 2)
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--chunk-mb", default="", help="comma list: time the host rows at each HOST_CHUNK_MB knob value")
    a = ap.parse_args()
    if a.chunk_mb:
        for c in a.chunk_mb.split(","):
            with vv.knobs(HOST_CHUNK_MB=int(c)):   # the registry knob, read by each host call
                sub = run_rows(a, quick=True)
            for r in sub:
                r["chunk_mb"] = int(c)
                print(json.dumps(r), flush=True)
        return
    res = {"device": torch.cuda.get_device_name(0), "date": time.strftime("%Y-%m-%d"),
           "pcie_46MB": copy_rates(46071808), "rows": run_rows(a)}
    for r in res["rows"]:
        print(json.dumps(r), flush=True)
    print(json.dumps({"pcie_46MB": res["pcie_46MB"]}), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


def run_rows(a, quick=False):
    api = VvDsp(vv.LIB_PATH)
    L = api.lib
    L.vv_dsp_stft_spectrogram.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.POINTER(C.c_size_t)]
    L.vv_dsp_fft_execute.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    res = {"rows": []}

    # config 3 through the reference API with host buffers
    n = 60 * 48000
    x = np.random.default_rng(3).uniform(-1, 1, n).astype(np.float32)
    fr = 1 + (n - 1024 + 256) // 256
    out = np.empty(fr * 1024, np.float32)
    prm = StftParams(1024, 256, 1)
    h = C.c_void_p()
    assert L.vv_dsp_stft_create(C.byref(prm), C.byref(h)) == 0
    nfr = C.c_size_t(0)

    def stft():
        assert L.vv_dsp_stft_spectrogram(h, x.ctypes.data, n, out.ctypes.data, C.byref(nfr)) == 0
    med, best = timeit(stft, a.reps)
    byts = n * 4 + fr * 4096
    res["rows"].append({"row": "stft_spectrogram_host_60s", "api": "vv_dsp_stft_spectrogram (host in/out)",
                        "ms_median": round(med * 1e3, 3), "ms_min": round(best * 1e3, 3),
                        "frames_per_s": round(fr / med, 1), "host_bytes": byts,
                        "effective_GBs": round(byts / med / 1e9, 2)})
    L.vv_dsp_stft_destroy(h)

    # config 2 with host buffers through a batched plan
    B, N = 65536, 1024
    xin = (np.random.default_rng(1).random((B, 2 * N), dtype=np.float32) - 0.5)
    yout = np.empty_like(xin)
    L.vv_dsp_fft_make_plan_many.argtypes = [C.c_size_t, C.c_int, C.c_int, C.c_size_t, C.POINTER(C.c_void_p)]
    p = C.c_void_p()
    assert L.vv_dsp_fft_make_plan_many(N, C2C, FWD, B, C.byref(p)) == 0

    def fftb():
        assert L.vv_dsp_fft_execute(p, xin.ctypes.data, yout.ctypes.data) == 0
    med, best = timeit(fftb, max(3, a.reps // 2))
    byts = 2 * B * N * 8
    res["rows"].append({"row": "fft_c2c_1024_batch65536_host", "api": "vv_dsp_fft_make_plan_many + vv_dsp_fft_execute "
                        "(host in/out)", "ms_median": round(med * 1e3, 3), "ms_min": round(best * 1e3, 3),
                        "transforms_per_s": round(B / med, 1), "host_bytes": byts,
                        "effective_GBs": round(byts / med / 1e9, 2)})
    L.vv_dsp_fft_destroy(p)

    if quick:
        return res["rows"]
    # the reference's call shape: one 1024-pt transform per vv_dsp_fft_execute
    x1 = np.random.default_rng(0).random(2 * N).astype(np.float32)
    y1 = np.empty_like(x1)
    p1 = C.c_void_p()
    assert L.vv_dsp_fft_make_plan(N, C2C, FWD, C.byref(p1)) == 0

    def fft1():
        for _ in range(100):
            L.vv_dsp_fft_execute(p1, x1.ctypes.data, y1.ctypes.data)
    med, best = timeit(fft1, 5)
    res["rows"].append({"row": "fft_c2c_1024_single_host", "api": "vv_dsp_fft_execute, one 1024-pt transform per call",
                        "us_per_call": round(med / 100 * 1e6, 2), "transforms_per_s": round(100 / med, 1)})
    L.vv_dsp_fft_destroy(p1)
    return res["rows"]


if __name__ == "__main__":
    main()
