#!/usr/bin/env python3
"""Config 3's ceiling on the box (timing tool, not a test): the 60 s mono STFT's
57.6 MB (11.5 MB read, 46.1 MB written) moved by pure streaming kernels with no
FFT -- scripts/membench.hip k_rwc (1 KB read -> 4 KB written per wave item, the
STFT's per-frame shape) and k_rw (flat 1:4) -- and an empty kernel's launch
floor, each timed as bench.py times config 3: an event pair around each single
launch (median of 50) and one event pair around 100 back to back.  Prints one
JSON line per case beside the product kernel's own config-3 numbers.

    python scripts/cfg3_ceiling.py
"""
import ctypes as C
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

FRAMES = 11248
BYTES = 57595904   # SURVEY 8d row note 3 (with the 4 KB window)


def timed(f, reps=50, burst=100):
    s = torch.cuda.current_stream()
    for _ in range(10):
        f()
    torch.cuda.synchronize()
    one = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        f()
        e1.record(s)
        torch.cuda.synchronize()
        one.append(e0.elapsed_time(e1))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(burst):
        f()
    e1.record(s)
    torch.cuda.synchronize()
    return statistics.median(one), e0.elapsed_time(e1) / burst


def line(name, ms1, msb, extra=None):
    d = {"case": name, "ms_single": round(ms1, 5), "ms_back_to_back": round(msb, 5),
         "frac_single": round(BYTES / (ms1 * 1e-3) / 8e12, 4), "frac_back_to_back": round(BYTES / (msb * 1e-3) / 8e12, 4)}
    d.update(extra or {})
    print(json.dumps(d), flush=True)


def main():
    mb = C.CDLL(os.path.join(ROOT, "scripts", "libmembench.so"))
    mb.membench_rwc.argtypes = [C.c_void_p, C.c_void_p, C.c_longlong] + [C.c_int] * 5 + [C.c_void_p]
    mb.membench_rw.argtypes = [C.c_void_p, C.c_void_p, C.c_longlong, C.c_int, C.c_int, C.c_void_p]
    lab = C.CDLL(os.path.join(ROOT, "scripts", "libstftlab.so"))
    lab.emptylab_run.argtypes = [C.c_int, C.c_void_p]
    a = torch.rand(FRAMES * 256, device="cuda")
    b = torch.empty(FRAMES * 1024, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    for u in (1, 2):
        for blocks in (703, 1406, 2812):
            f = (lambda u=u, blocks=blocks: mb.membench_rwc(a.data_ptr(), b.data_ptr(), FRAMES, 4, u, 1, 1, blocks, s))
            assert f() == 0
            line("rwc", *timed(f), {"u": u, "blocks": blocks, "waves": 4 * blocks})
    n4 = FRAMES * 64
    for blocks in (703, 2812):
        f = (lambda blocks=blocks: mb.membench_rw(a.data_ptr(), b.data_ptr(), n4, 4, blocks, s))
        assert f() == 0
        line("rw_flat", *timed(f), {"blocks": blocks})
    for grid in (703, 2812):
        f = (lambda grid=grid: lab.emptylab_run(grid, s))
        assert f() == 0
        line("empty", *timed(f), {"grid": grid})
    d = bench.stft_config3()
    line("product_stft", d["ms_avg"], d["back_to_back_100"]["ms_per_call"])


if __name__ == "__main__":
    main()
