#!/usr/bin/env python3
"""bench.py -- MI355X benchmark of the vv-dsp spectral hot path.

Headline (BASELINE.json metric): STFT frames/sec, 1024-pt Hann, hop 256, on
config 5 itself -- 256 channels x 10 min @ 48 kHz (28,800,000 samples, 112,498
frames each; 28,799,488 frames, 29.5 GB in + 118 GB out), magnitude spectrogram
[ch][frame][1024] f32 (src/spectral/stft.c:112-144), computed by the fused gfx950
STFT kernel (one launch per step and rank).  Strong scaling: the 256 channels
are split over the N ranks (channel_shard: contiguous ranges, 32 per rank at
N = 8), so at N = 1 the whole job runs on one GPU (147 GB of its 288 GB HBM).
Inputs are synthetic (uniform[-1,1), seed = global channel id), generated on
the device and resident in HBM before timing.  Channels are independent: ranks
process disjoint channel shards with no collective in the timed region.

Also measured (same JSON line): the roofline of the dominant kernel (HIP events
on the launch stream), config 2 (65536 x 1024 c2c f32 FFT) and config 4 (FIR
overlap-save 257 taps, 8 ch x 2^24) GB/s, and the reference's own CPU STFT
(oracle/_ref, i.e. the reference sources compiled in the build container) timed
on this host's cores on a bounded sample.

    python bench.py [--gpus N] [--steps K] [--warmup W]     (N > 1: one process drives N GPUs)
    torchrun --nproc-per-node N bench.py --gpus N ...        (one rank per GPU)
Both N > 1 forms run through the library's plain-C RCCL layer
(include/vv_dsp/vv_dsp_dist.h): ncclCommInitAll in one process, or
ncclCommInitRank per torchrun rank; `--gpus N` on a box with fewer than N
visible GPUs exits non-zero.
"""
import argparse
import concurrent.futures as cf
import ctypes as C
import glob
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "vv-dsp_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import vvdsp_amd as vv  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
NFFT, HOP = 1024, 256
FS = 48000
CH_TOTAL = 256               # config 5: the whole job, split over the ranks
CH_SHARD = 32                # config 5 per-GPU shard at 8 GPUs (extra leg at N = 1)
SAMPLES = 10 * 60 * FS        # 10 min per channel
PUBLISHED_CPU_FPS = 24903.0   # BASELINE.md §1 STFT_size_1024 (CPU, 1 thread) -- informational only:
                              # BASELINE.json "published" is empty, so vs_baseline is null
# the newest round's committed PMC summary of this command (profiles/rNN_bench_pmc.json,
# or that round's rNN_final_pmc.json of its final tree, which sorts after it)
TRAFFIC_JSON = (sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_bench_pmc.json")) +
                       glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_final_pmc.json")),
                       key=lambda f: (os.path.basename(f)[:3], "_final_" in f)) or
                [os.path.join(ROOT, "profiles", "r01_bench_pmc.json")])[-1]
METRIC = "STFT frames/sec (1024-pt, hop 256) at 1/2/4/8 GPU; achieved HBM GB/s vs peak"
TIMING_NOTE = ("ms_avg: HIP events around the timed launches back to back / launches (the launch stream); "
               "ms_avg_isolated / ms_min: an event pair around each single launch")


def frames_of(n):
    return 1 if n < NFFT else 1 + (n - NFFT + HOP) // HOP


def timed_launches(fn, reps, warm=3, warm_s=0.25):
    """Average device time of fn() (one kernel launch each) with HIP events
    recorded on torch's current stream -- the stream the library launches on.
    Warm-up: at least `warm` launches AND `warm_s` seconds of back-to-back
    launches, so the GPU clock has left its idle state (a 0.2 ms kernel timed
    after ten warm-up launches reads up to 30 % slow: the clock ramp is tens of
    ms, measured on the FIR leg).
    Returns (avg, min, isolated_avg): avg = one event pair around `reps`
    back-to-back launches / reps -- the kernel's average launch duration, which
    rocprofv3's kernel trace of the same launches matches; min and isolated_avg
    from an event pair around each single launch (each then also carries an
    event's end-of-kernel wait and the next launch's dispatch, +2-3 % for a
    0.2 ms kernel)."""
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < warm_s:
        for _ in range(8):
            fn()
        torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record(s)
        fn()
        b.record(s)
    torch.cuda.synchronize()
    ms = [a.elapsed_time(b) for a, b in ev]
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(reps):
        fn()
    b.record(s)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps, float(np.min(ms)), float(np.mean(ms))


def fft_c2c_roofline(reps=50):
    """Config 2: 65536 x 1024-pt c2c f32 forward, device resident."""
    B, N = 65536, 1024
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.complex(torch.rand(B, N, device="cuda", generator=g) - 0.5,
                      torch.rand(B, N, device="cuda", generator=g) - 0.5)
    y = torch.empty_like(x)
    plan = vv.FftPlan(N, vv.C2C, vv.FWD, batch=B)
    avg, best, iso = timed_launches(lambda: plan(x, out=y), reps, warm=10)
    planb = vv.FftPlan(N, vv.C2C, vv.BWD, batch=B)
    bavg, bbest, biso = timed_launches(lambda: planb(x, out=y), reps, warm=10)
    byts = 2 * B * N * 8
    del x, y
    return {"workload": "config2: 65536 x 1024-pt c2c f32 forward", "bytes_per_launch": byts,
            "ms_avg": round(avg, 4), "ms_min": round(best, 4), "ms_avg_isolated": round(iso, 4),
            "timing": TIMING_NOTE,
            "achieved_GBs": round(byts / (avg * 1e-3) / 1e9, 1), "peak_GBs": HBM_PEAK_GBS,
            "frac": round(byts / (avg * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "ffts_per_s": round(B / (avg * 1e-3), 1),
            "kernel": "vvh::k_c2c<1024, true> (one launch)",
            **dict(zip(("traffic", "traffic_source"), kernel_traffic(["vvh::k_c2c<1024, true>", "vvh::k_c2c<1024, true,"]))),
            "backward": {"ms_avg": round(bavg, 4), "ms_min": round(bbest, 4), "ms_avg_isolated": round(biso, 4),
                         "frac": round(byts / (bavg * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}}


def stft_config3(reps=50, burst=100):
    """Config 3: STFT magnitude of 60 s mono @ 48 kHz (11,248 frames), one call,
    and `burst` calls back to back between one pair of events."""
    n = 60 * 48000
    g = torch.Generator(device="cuda").manual_seed(3)
    sig = torch.rand(1, n, device="cuda", generator=g) * 2 - 1
    st = vv.Stft(NFFT, HOP)
    fr = st.frames(n)
    out = torch.empty(1, fr, NFFT, device="cuda")
    fn = lambda: st.spectrogram(sig, out=out)  # noqa: E731
    _, best, avg = timed_launches(fn, reps)   # one call: events around each single call (isolated)
    s = torch.cuda.current_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(burst):
        fn()
    b.record(s)
    torch.cuda.synchronize()
    per = a.elapsed_time(b) / burst
    byts = n * 4 + NFFT * 4 + fr * NFFT * 4
    del sig, out
    ceil = copy_ceiling(fr)
    extra = {}
    if ceil is not None:
        cbyts = fr * HOP * 4 + fr * NFFT * 4
        extra = {"copy_ceiling": {
            "what": "the same job's bytes (1 KB in -> 4 KB out per frame) moved by a streaming copy with no FFT "
                    "(scripts/membench.hip k_rwc, best of u in {1,2} x {703, 2812} workgroups), timed in this run "
                    "exactly as the product: the box's ceiling for a 57.6 MB single launch",
            "ms_avg": round(ceil["ms_avg"], 4), "ms_back_to_back": round(ceil["ms_back_to_back"], 4),
            "frac": round(cbyts / (ceil["ms_avg"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "frac_back_to_back": round(cbyts / (ceil["ms_back_to_back"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "shape": {"u": ceil["u"], "blocks": ceil["blocks"]}},
            "frac_of_ceiling": round(ceil["ms_avg"] / avg, 4),
            "frac_of_ceiling_back_to_back": round(ceil["ms_back_to_back"] / per, 4)}
    return {"workload": "config3: STFT 60 s mono @ 48 kHz, 1024 Hann, hop 256 (11,248 frames)",
            "bytes_per_call": byts, "ms_avg": round(avg, 4), "ms_min": round(best, 4),
            "timing": "ms_avg: an event pair around each single call (isolated); back_to_back: one event pair "
                      "around the burst",
            "frames_per_s": round(fr / (avg * 1e-3), 1),
            "frac": round(byts / (avg * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            f"back_to_back_{burst}": {"ms_per_call": round(per, 4), "frames_per_s": round(fr / (per * 1e-3), 1),
                                      "frac": round(byts / (per * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
            **extra}


def _membench():
    """scripts/libmembench.so (built by __graft_entry__.build(): `make -C vv-dsp_amd membench`): streaming
    kernels with no FFT, the box's own ceiling for a job's bytes (measurement only, not the product)"""
    path = os.path.join(ROOT, "scripts", "libmembench.so")
    if not os.path.exists(path):
        return None
    mb = C.CDLL(path)
    mb.membench_rwc.argtypes = [C.c_void_p, C.c_void_p, C.c_longlong] + [C.c_int] * 5 + [C.c_void_p]
    return mb


def copy_ceiling(frames, reps=50, burst=100):
    """Config 3's bytes (1 KB of new samples in, one 4 KB row out per frame) moved
    by a pure streaming kernel with no FFT (membench k_rwc: one 1 KB -> 4 KB item
    per wave step, u items in flight per wave), timed exactly as stft_config3 times
    the product: the best of four launch shapes, single call and back to back."""
    mb = _membench()
    if mb is None:
        return None
    a = torch.rand(frames * HOP, device="cuda")
    b = torch.empty(frames * NFFT, device="cuda")
    s = torch.cuda.current_stream()
    best = None
    for u in (1, 2):
        for blocks in (703, 2812):
            fn = (lambda u=u, blocks=blocks: mb.membench_rwc(a.data_ptr(), b.data_ptr(), frames, 4, u, 1, 1, blocks,
                                                             s.cuda_stream))
            assert fn() == 0
            _, mn, avg = timed_launches(fn, reps)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(burst):
                fn()
            e1.record(s)
            torch.cuda.synchronize()
            b2b = e0.elapsed_time(e1) / burst
            if best is None or avg < best["ms_avg"]:
                best = {"ms_avg": avg, "ms_back_to_back": b2b, "u": u, "blocks": blocks}
    del a, b
    return best


def fir_roofline(reps=50):
    """Config 4: 257-tap lowpass (Hann, fc 0.25) overlap-save, 8 ch x 2^24 f32."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    nch, n = 8, 1 << 24
    # taps designed by the library's host setup code (fir.c:47-73 arithmetic)
    L = vv.lib()
    L.vv_dsp_fir_design_lowpass.argtypes = [C.c_void_p, C.c_size_t, C.c_float, C.c_int]
    h = np.zeros(257, np.float32)
    assert L.vv_dsp_fir_design_lowpass(h.ctypes.data, 257, 0.25, 2) == 0
    g = torch.Generator(device="cuda").manual_seed(4)
    x = torch.rand(nch, n, device="cuda", generator=g) * 2 - 1
    y = torch.empty_like(x)
    plan = vv.FirPlan(torch.from_numpy(h))
    avg, best, iso = timed_launches(lambda: plan(x, out=y), reps, warm=10)
    byts = 2 * nch * n * 4
    del x, y
    return {"workload": "config4: FIR overlap-save 257 taps, 8 ch x 2^24 f32", "bytes_per_launch": byts,
            "ms_avg": round(avg, 4), "ms_min": round(best, 4), "ms_avg_isolated": round(iso, 4),
            "timing": TIMING_NOTE,
            "achieved_GBs": round(byts / (avg * 1e-3) / 1e9, 1), "peak_GBs": HBM_PEAK_GBS,
            "frac": round(byts / (avg * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "samples_per_s": round(nch * n / (avg * 1e-3), 1),
            "kernel": "vvh::k_fir_r32<true> (1024-point blocks as 32 x 32 on half-waves: one LDS transpose per "
                      "FFT, radix 4 x 8 DFT_32; samples moved as 8 B per lane re-laid by v_permlane16_swap; two blocks "
                      "per complex FFT, two pairs per wave, every pair of every channel in one persistent launch, the "
                      "edge pairs bounds-checked in the same loop), one step",
            **dict(zip(("traffic", "traffic_source"), kernel_traffic(["vvh::k_fir_r32"])))}


def host_cpu_share():
    """Threads for the CPU baseline: this process's CPU affinity, capped by the
    cgroup CPU quota and by OMP_NUM_THREADS when either is set (the GPU box
    exposes every core of the host but grants one GPU's job a share of them),
    and the CPU model from /proc/cpuinfo."""
    cands = {"affinity": len(os.sched_getaffinity(0))}
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            cands["cgroup_quota"] = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    try:
        cands["OMP_NUM_THREADS"] = max(1, int(os.environ["OMP_NUM_THREADS"]))
    except (KeyError, ValueError):
        pass
    model = "?"
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return min(cands.values()), cands, model, os.cpu_count()


def _threaded(threads, seconds, work):
    """Run work(i, t_end) on `threads` threads until `seconds` pass; ctypes
    releases the GIL inside the reference's C calls."""
    t_end = time.perf_counter() + seconds
    t0 = time.perf_counter()
    with cf.ThreadPoolExecutor(threads) as ex:
        done = sum(ex.map(lambda i: work(i, t_end), range(threads)))
    return done, time.perf_counter() - t0


def _repeats(threads, seconds, work, reps):
    """`reps` back-to-back samples of _threaded; each sample's rate (units/s)."""
    rates, units, secs = [], 0, 0.0
    for _ in range(reps):
        n, dt = _threaded(threads, seconds, work)
        rates.append(n / dt)
        units += n
        secs += dt
    return rates, units, secs


def _spread(rates):
    med = float(np.median(rates))
    return {"value": round(med, 1), "repeats": [round(r, 1) for r in rates],
            "spread_pct": round(100.0 * (max(rates) - min(rates)) / med, 2) if med > 0 else None}


def cpu_baseline(threads=None, seconds=5.0, reps=3):
    """The reference's own code (oracle/_ref = the reference sources compiled in
    the build container, KissFFT backend) on this host's CPU share, on bounded
    samples of three BASELINE workloads, each timed as `reps` back-to-back
    samples (value = the median, spread = (max - min) / median):
      * headline: vv_dsp_stft_spectrogram of 60 s mono (stft.c:112-144) back to
        back on every thread, 3 x 5 s (frames/s; the bench line's cpu_baseline value);
      * config 2: 1024-pt C2C transforms through vv_dsp_fft_execute
        (fft_kiss.c:27-74), 4096-transform chunks of a 65,536 x 1024 batch, 3 x 3 s;
      * config 4: vv_dsp_fir_apply direct form (fir.c:160-196), 257 taps, 2^22-
        sample quarter channels (fresh state each) back to back, 3 x 2 s (the
        reference's fir_apply_fft is O(n^2) there)."""
    from vvapi import VvDsp, FirState
    path = os.path.join(ROOT, "oracle", "_ref", "libvvref.so")
    bpath = os.path.join(ROOT, "oracle", "_ref", "librefbench.so")
    if not os.path.exists(path):
        return {"value": None, "unit": "frames/s", "cores": 0, "kind": "reference",
                "sample": "oracle/_ref/libvvref.so missing"}
    ref = VvDsp(path)
    share, cands, model, ncpu = host_cpu_share()
    threads = threads or share
    n = 60 * FS
    rng = np.random.default_rng(3)
    sigs = [rng.uniform(-1, 1, n).astype(np.float32) for _ in range(threads)]

    def stft_work(i, t_end):
        done = 0
        while time.perf_counter() < t_end:
            ref.spectrogram(sigs[i], NFFT, HOP)
            done += frames_of(n)
        return done

    rates, frames, dt = _repeats(threads, seconds, stft_work, reps)
    t1 = time.perf_counter()
    ref.spectrogram(sigs[0], NFFT, HOP)
    d1 = time.perf_counter() - t1
    del sigs
    res = {**_spread(rates), "unit": "frames/s", "cores": threads, "kind": "reference",
           "sample": f"{threads} threads x vv_dsp_stft_spectrogram(60 s @ 48 kHz mono, 1024 Hann, hop 256) "
                     f"back to back, {reps} samples of {seconds:.0f} s: {frames} frames in {dt:.2f} s; "
                     f"value = median of the samples",
           "single_thread_frames_per_s": round(frames_of(n) / d1, 1),
           "cpu_model": model, "host_cpus": ncpu, "thread_caps": cands}

    if os.path.exists(bpath):      # config 2
        rb = C.CDLL(bpath)
        rb.refbench_fft_rows.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_size_t, C.c_int]
        B, N, chunk = 65536, 1024, 4096
        x = np.random.default_rng(1).uniform(-0.5, 0.5, (B, 2 * N)).astype(np.float32)
        ys = [np.empty((chunk, 2 * N), np.float32) for _ in range(threads)]

        def fft_work(i, t_end):
            done = 0
            while time.perf_counter() < t_end:
                r0 = (done * chunk + i * 977 * chunk) % B
                r0 -= r0 % chunk
                assert rb.refbench_fft_rows(x[r0:].ctypes.data, ys[i].ctypes.data, N, chunk, 1) == 0
                done += chunk
            return done

        rates2, cnt, dt2 = _repeats(threads, 3.0, fft_work, reps)
        sp = _spread(rates2)
        res["config2_fft_c2c_1024"] = {
            **sp, "unit": "transforms/s", "cores": threads,
            "batch_65536_s": round(B / sp["value"], 4),
            "sample": f"{threads} threads x vv_dsp_fft_execute (Kiss radix-2, one plan per thread) over rows of a "
                      f"65536 x 1024 uniform[-0.5,0.5) batch, {reps} samples of 3 s: {cnt} transforms in {dt2:.2f} s"}
        del x, ys

    # the reference's other STFT sizes (bench/bench_stft.c:165), 60 s mono per call, hop nfft/4
    sigs = [np.random.default_rng(3 + i).uniform(-1, 1, n).astype(np.float32) for i in range(threads)]
    sizes = {}
    for nfft in STFT_SIZES:
        hop = nfft // 4
        per = 1 if n < nfft else 1 + (n - nfft + hop) // hop

        def size_work(i, t_end, nfft=nfft, hop=hop, per=per):
            done = 0
            while time.perf_counter() < t_end:
                ref.spectrogram(sigs[i], nfft, hop)
                done += per
            return done

        r, cnt, dts = _repeats(threads, 2.0, size_work, 1)
        sizes[str(nfft)] = {"value": round(r[0], 1), "unit": "frames/s", "hop": hop,
                            "sample": f"{threads} threads x vv_dsp_stft_spectrogram(60 s mono, nfft {nfft}, hop {hop}) "
                                      f"back to back for 2 s: {cnt} frames in {dts:.2f} s"}
    res["stft_sizes"] = sizes
    del sigs

    h = np.zeros(257, np.float32)          # config 4
    ref.lib.vv_dsp_fir_design_lowpass(h.ctypes.data_as(C.POINTER(C.c_float)), 257, 0.25, 2)
    ns = 1 << 22
    xs = [np.random.default_rng(4 + i).uniform(-1, 1, ns).astype(np.float32) for i in range(threads)]
    ys = [np.empty(ns, np.float32) for _ in range(threads)]

    def fir_work(i, t_end):
        done = 0
        fp = C.POINTER(C.c_float)
        while time.perf_counter() < t_end:
            st = FirState()
            assert ref.lib.vv_dsp_fir_state_init(C.byref(st), 257) == 0
            r = ref.lib.vv_dsp_fir_apply(C.byref(st), h.ctypes.data_as(fp), xs[i].ctypes.data_as(fp),
                                         ys[i].ctypes.data_as(fp), ns)
            ref.lib.vv_dsp_fir_state_free(C.byref(st))
            assert r == 0
            done += ns
        return done

    rates4, cnt, dt4 = _repeats(threads, 2.0, fir_work, reps)
    sp = _spread(rates4)
    res["config4_fir_direct_257"] = {
        **sp, "unit": "samples/s", "cores": threads,
        "config4_s": round(8 * (1 << 24) / sp["value"], 3),
        "sample": f"{threads} threads x vv_dsp_fir_apply (direct form, fresh state per 2^22-sample block) on "
                  f"uniform[-1,1) samples, {reps} samples of >= 2 s: {cnt} samples in {dt4:.2f} s"}
    return res


def _load_pmc():
    try:
        with open(TRAFFIC_JSON) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def kernel_traffic(prefixes, per_step_calls=None, channels=None):
    """HBM bytes per launch of one leg from the committed rocprofv3 PMC summary
    of this command (scripts/gpu_bench_prof.sh + scripts/pmc_summary.py --json):
    FETCH_SIZE x 2 (gfx950 tallies 128-B reads at 64 B, MI355X_MICROARCH.md
    §HBM) + WRITE_SIZE, both in KiB, per dispatch, summed over the kernels of
    one launch (names starting with one of `prefixes`)."""
    prof = _load_pmc()
    if prof is None:
        return None, "no PMC summary committed"
    if channels is not None and prof.get("channels_per_gpu") != channels:
        return None, f"PMC summary is for {prof.get('channels_per_gpu')} channels per GPU"
    tot, names = 0.0, []
    for k, c in prof["kernels"].items():
        if k.startswith(tuple(prefixes)) and "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            tot += (2.0 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024.0
            names.append(f"{k} ({c.get('avg_us')} us avg)")
    if not names:
        return None, f"PMC summary has no {'/'.join(prefixes)} entries"
    return round(tot), f"{os.path.relpath(TRAFFIC_JSON, ROOT)} ({prof.get('box', '?')}): " \
                       f"(2*FETCH_SIZE + WRITE_SIZE) KiB x 1024 per dispatch over {', '.join(names)}"


def hbm_traffic(channels):
    return kernel_traffic(["vvh::k_stft_pair<1024, 0, 5"], channels=channels)


def shard_leg(ch=CH_SHARD, steps=20, warm=10):
    """Config 5's per-GPU shard at 8 GPUs -- 32 ch x 10 min @ 48 kHz, 18.4 GB in
    + out -- on one GPU: what each rank of the driver's N = 8 run computes.  Same
    kernel, walk and output layout as the headline."""
    nfr = frames_of(SAMPLES)
    try:
        sig = torch.empty(ch, SAMPLES, device="cuda")
        for c in range(ch):
            g = torch.Generator(device="cuda").manual_seed(c)
            sig[c].uniform_(-1.0, 1.0, generator=g)
        out = torch.empty(ch, nfr, NFFT, device="cuda")
    except torch.OutOfMemoryError as e:
        return {"error": repr(e)[:200]}
    st = vv.Stft(NFFT, HOP, vv.WIN_HANN)
    avg, best, iso = timed_launches(lambda: st.spectrogram(sig, out=out), steps, warm=warm)
    fr = 12345
    x0 = sig[ch - 1, fr * HOP: fr * HOP + NFFT].double().cpu().numpy()
    ok = np.allclose(out[ch - 1, fr].cpu().numpy(), np.abs(np.fft.fft(x0 * hann64())), rtol=5e-5, atol=5e-5)
    byts = ch * SAMPLES * 4 + ch * nfr * NFFT * 4 + NFFT * 4
    del sig, out, st
    torch.cuda.empty_cache()
    return {"workload": f"config5 per-GPU shard at 8 GPUs: {ch} ch x 10 min @ 48 kHz, 1024 Hann, hop 256 "
                        f"({ch * nfr:,} frames; 3.7 GB in, 14.7 GB out)",
            "steps": steps, "ms_avg": round(avg, 4), "ms_min": round(best, 4),
            "frames_per_s": round(ch * nfr / (avg * 1e-3), 1),
            "bytes_per_launch": byts, "frac": round(byts / (avg * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "check_row_vs_numpy_f64": bool(ok)}


def hann64(nfft=NFFT):
    """The reference's symmetric Hann (window.c:25-36, float arithmetic) in f64."""
    return np.array([0.5 - 0.5 * np.cos(np.float32(2 * np.pi) / np.float32(nfft - 1) * np.float32(i))
                     for i in range(nfft)], np.float64)


STFT_SIZES = (256, 512, 2048, 4096)   # the reference's own STFT sizes besides 1024 (bench/bench_stft.c:165)


def stft_sizes_leg(ch=CH_SHARD, reps=20, sizes=STFT_SIZES):
    """The reference's benchmarked STFT sizes (bench/bench_stft.c:163-227, docs/profiles/stft_profile.json:17-46:
    nfft 256 / 512 / 2048 / 4096 at hop nfft/4) on config 5's per-GPU shard (32 ch x 10 min @ 48 kHz),
    magnitude rows [ch][frame][nfft]: frames/s, HBM fraction and one row per size against NumPy f64."""
    try:
        sig = torch.empty(ch, SAMPLES, device="cuda")
        for c in range(ch):
            g = torch.Generator(device="cuda").manual_seed(c)
            sig[c].uniform_(-1.0, 1.0, generator=g)
    except torch.OutOfMemoryError as e:
        return {"error": repr(e)[:200]}
    res = {"workload": f"{ch} ch x 10 min @ 48 kHz per size, Hann, hop nfft/4, magnitude rows (stft.c:112-144)"}
    for nfft in sizes:
        hop = nfft // 4
        nfr = 1 if SAMPLES < nfft else 1 + (SAMPLES - nfft + hop) // hop
        out = torch.empty(ch, nfr, nfft, device="cuda")
        st = vv.Stft(nfft, hop, vv.WIN_HANN)
        avg, best, iso = timed_launches(lambda: st.spectrogram(sig, out=out), reps, warm=10)
        byts = ch * SAMPLES * 4 + ch * nfr * nfft * 4 + nfft * 4
        fr = nfr // 3
        x0 = sig[ch - 1, fr * hop: fr * hop + nfft].double().cpu().numpy()
        ok = np.allclose(out[ch - 1, fr].cpu().numpy(), np.abs(np.fft.fft(x0 * hann64(nfft))), rtol=5e-5, atol=5e-5)
        res[str(nfft)] = {"hop": hop, "frames": ch * nfr, "ms_avg": round(avg, 4), "ms_min": round(best, 4),
                          "frames_per_s": round(ch * nfr / (avg * 1e-3), 1), "bytes_per_launch": byts,
                          "frac": round(byts / (avg * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                          "check_row_vs_numpy_f64": bool(ok)}
        del out, st
        torch.cuda.empty_cache()
    del sig
    torch.cuda.empty_cache()
    return res


def features_leg(ch=CH_SHARD, reps=20, n_mels=40, n_coeffs=13):
    """SURVEY §8 f1 / f3 on config 5's per-GPU shard (32 ch x 10 min @ 48 kHz, 1024 Hann, hop 256): power rows
    [ch][frame][513] (|X|^2 of bins 0..nfft/2, the mel stage's input), and signal -> log-mel (40 bands) / MFCC
    (13 coefficients, lifter 22) rows in one launch each (src/features/mel.c:204-330 after stft.c:112-144).
    Checks: one power row against NumPy f64; one log-mel and one MFCC row bit for bit against the two-step
    device pipeline (power rows, then vv_dsp_log_mel_device / vv_dsp_mfcc_process_device)."""
    nfr = frames_of(SAMPLES)
    nb = NFFT // 2 + 1
    try:
        sig = torch.empty(ch, SAMPLES, device="cuda")
        for c in range(ch):
            g = torch.Generator(device="cuda").manual_seed(c)
            sig[c].uniform_(-1.0, 1.0, generator=g)
        pw = torch.empty(ch, nfr, nb, device="cuda")
    except torch.OutOfMemoryError as e:
        return {"error": repr(e)[:200]}
    st = vv.Stft(NFFT, HOP, vv.WIN_HANN)
    mf = vv.Mfcc(NFFT, n_mels, n_coeffs, float(FS), 20.0, 20000.0, lifter=22.0)
    res = {"workload": f"{ch} ch x 10 min @ 48 kHz, 1024 Hann, hop 256 ({ch * nfr:,} frames): power rows, "
                       f"log-mel ({n_mels} bands) and MFCC ({n_coeffs} coefficients) from the signal"}
    avg, best, _ = timed_launches(lambda: st.power(sig, out=pw), reps, warm=10)
    byts = ch * SAMPLES * 4 + ch * nfr * nb * 4
    fr = nfr // 3
    x0 = sig[ch - 1, fr * HOP: fr * HOP + NFFT].double().cpu().numpy()
    want = np.abs(np.fft.fft(x0 * hann64())[:nb]) ** 2
    ok = np.allclose(pw[ch - 1, fr].cpu().numpy(), want, rtol=1e-4, atol=1e-4 * NFFT)
    res["power_rows"] = {"ms_avg": round(avg, 4), "ms_min": round(best, 4), "bytes_per_launch": byts,
                         "frac": round(byts / (avg * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                         "check_row_vs_numpy_f64": bool(ok)}
    row = pw[ch - 1, fr:fr + 1].clone()
    for name, log_mel, width in (("log_mel", True, n_mels), ("mfcc", False, n_coeffs)):
        out = torch.empty(ch, nfr, width, device="cuda")
        avg, best, _ = timed_launches(lambda: mf.from_signal(st, sig, log_mel=log_mel, out=out), reps, warm=10)
        ref = mf.log_mel(row) if log_mel else mf(row)
        torch.cuda.synchronize()
        res[name] = {"ms_avg": round(avg, 4), "ms_min": round(best, 4),
                     "frames_per_s": round(ch * nfr / (avg * 1e-3), 1),
                     "bytes_per_launch": ch * SAMPLES * 4 + ch * nfr * width * 4,
                     "check_row_equals_two_step": bool(torch.equal(out[ch - 1, fr:fr + 1], ref))}
        del out
    del sig, pw, st, mf
    torch.cuda.empty_cache()
    return res


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs of this node (default 1).  Without torchrun (no WORLD_SIZE) N > 1 runs every GPU "
                         "from this one process over the library's plain-C RCCL layer (vv_dsp_dist_init_all); "
                         "under torchrun it must equal WORLD_SIZE (one rank per GPU, vv_dsp_dist_init_rank)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=25)
    ap.add_argument("--channels", type=int, default=CH_TOTAL,
                    help="channels of the whole job (config 5: 256), split over the ranks (strong scaling)")
    ap.add_argument("--no-extras", action="store_true", help="skip config 2/3/4, shard and CPU baseline legs")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg (profiling runs)")
    ap.add_argument("--legs", default="c2c,fir,config3,shard,sizes,features",
                    help="extra GPU legs: c2c (config 2), fir (config 4), config3, shard (config 5's 32-channel "
                         "per-GPU shard of the N = 8 run), sizes (the reference's STFT sizes 256/512/2048/4096 on "
                         "that shard), features (power rows, log-mel and MFCC on that shard); profiling runs "
                         "leave config3, shard, sizes and features out so the headline kernel's PMC average "
                         "covers the headline launches only")
    ap.add_argument("--gather-bins", choices=["half", "full"], default="half",
                    help="gather bins 0..512 and expand on rank 0 (half, default) or all 1024 bins (full)")
    ap.add_argument("--gather", choices=["auto", "on", "off"], default="auto",
                    help="after the timed steps, time one RCCL gather of all spectrogram rows to rank 0 "
                         "(config 5 'with gather'; auto = on when N > 1)")
    ap.add_argument("--dist-c", action="store_true",
                    help="run N = 1 through the multi-GPU layer too (vv_dsp_dist_init_all over one device): "
                         "the N > 1 code path on a one-GPU box")
    return ap.parse_args()


def launch_mode(args):
    """("plain", 1): today's single-GPU line; ("node", N): one process drives N
    GPUs (ncclCommInitAll); ("ranks", N): torchrun, one process per GPU.
    Never re-launches anything: a process that has touched the GPU must not exec."""
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None and (int(env_world) > 1 or args.dist_c):
        world = int(env_world)
        if args.gpus is not None and args.gpus != world:
            raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
        return "ranks", world
    n = 1 if args.gpus is None else args.gpus
    if n < 1:
        raise SystemExit(f"bench.py: --gpus {n}")
    visible = torch.cuda.device_count()   # counts devices without initialising them
    if visible < n:
        raise SystemExit(f"bench.py: --gpus {n} asks for {n} GPUs but this process sees {visible}; "
                         f"refusing to report an {n}-GPU number from fewer devices")
    return ("node", n) if (n > 1 or args.dist_c) else ("plain", 1)


def main():
    args = parse_args()
    mode, world = launch_mode(args)
    if mode == "plain":
        return main_plain(args)
    return main_dist(args, mode, world)


def result_line(args, value, world, elapsed, total_ch, per_gpu, nfr, parallelism, roofline, ok):
    return {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "published_cpu_reference": {"value": PUBLISHED_CPU_FPS, "unit": "frames/s",
                                    "what": "BASELINE.md §1 STFT_size_1024, Ryzen 9 7950X, 1 thread, KissFFT "
                                            "(informational; BASELINE.json publishes no number for this metric)"},
        "dtype": "f32",
        "data": "synthetic: uniform[-1,1) per channel, seed = global channel id, generated in HBM",
        "config": {
            "workload": f"config5: multi-channel STFT magnitude, {total_ch} ch x 10 min @ 48 kHz "
                        f"({total_ch * nfr:,} frames per step), nfft 1024 Hann, hop 256; strong scaling: "
                        + (f"{per_gpu} ch per GPU" if world > 1 else f"{per_gpu} ch on this rank")
                        + (" (the whole job on one GPU)" if world == 1 else ""),
            "channels_total": total_ch, "channels_per_gpu": per_gpu, "samples_per_channel": SAMPLES,
            "frames_per_channel": nfr, "frames_per_step": total_ch * nfr,
            "nfft": NFFT, "hop": HOP, "window": "hann (symmetric, window.c:25-36)",
            "output": "[ch][frame][1024] f32 magnitudes (stft.c:133-139)",
            "parallelism": parallelism},
        "roofline": roofline,
        "check_row_vs_numpy_f64": bool(ok),
    }


ROOFLINE_KERNEL = ("vvh::k_stft_pair<1024,0,5> (persistent dynamic band walk in runs of 2 pairs; LDS-DMA frame "
                   "spans kept as a ring of 256-float chunks + Hann + two frames per 1024-pt complex FFT + |X| rows "
                   "as full-line streaming stores; the zero-padded tail pairs run in the same launch)")


def check_rows(sig, out, channels):
    """one frame row of the given channels against NumPy f64, so a fast-but-wrong
    kernel cannot report"""
    fr, ok = 12345, True
    for c in channels:
        x0 = sig[c, fr * HOP: fr * HOP + NFFT].double().cpu().numpy()
        ok = ok and np.allclose(out[c, fr].cpu().numpy(), np.abs(np.fft.fft(x0 * hann64())), rtol=5e-5, atol=5e-5)
    return ok


def main_plain(args):
    """N = 1 (no torchrun): the whole job on cuda:0 through the single-GPU API."""
    torch.cuda.set_device(0)
    if vv.device_count() <= 0:
        raise SystemExit("libvvdsp_amd.so sees no HIP device")
    total_ch = args.channels
    C_ = total_ch
    nfr = frames_of(SAMPLES)
    sig = torch.empty(C_, SAMPLES, device="cuda")
    for c in range(C_):
        g = torch.Generator(device="cuda").manual_seed(c)
        sig[c].uniform_(-1.0, 1.0, generator=g)
    out = torch.empty(C_, nfr, NFFT, device="cuda")
    st = vv.Stft(NFFT, HOP, vv.WIN_HANN)

    def step():
        st.spectrogram(sig, out=out)

    for _ in range(args.warmup):
        step()
    # kernel duration for the roofline: events around each launch on the launch stream
    s = torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for a, b in ev:
        a.record(s)
        step()
        b.record(s)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))

    frames_total = total_ch * nfr * args.steps
    value = frames_total / elapsed
    bytes_per_launch = C_ * SAMPLES * 4 + C_ * nfr * NFFT * 4 + NFFT * 4
    achieved = bytes_per_launch / (kern_ms * 1e-3) / 1e9
    traffic, traffic_src = hbm_traffic(C_)
    ok = check_rows(sig, out, (0, C_ - 1))
    del sig, out, st
    torch.cuda.empty_cache()

    roof = {"kernel": ROOFLINE_KERNEL + "; kernel_ms = HIP events around "
                      f"each of the {args.steps} timed launches on the launch stream ({C_} channels per launch)",
            "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": traffic_src,
            "bytes_per_launch": bytes_per_launch, "kernel_ms": round(kern_ms, 4)}
    res = result_line(args, value, 1, elapsed, total_ch, C_, nfr,
                      "dp1 (channel shards, no data-path collective)", roof, ok)
    legs = set(args.legs.split(","))
    if not args.no_extras:
        if "shard" in legs:
            res["config5_shard_32ch"] = shard_leg()
            torch.cuda.empty_cache()
        if "c2c" in legs:
            res["fft_c2c_1024"] = fft_c2c_roofline()
            torch.cuda.empty_cache()
        if "fir" in legs:
            res["fir_ols_257"] = fir_roofline()
            torch.cuda.empty_cache()
        if "config3" in legs:
            res["stft_config3"] = stft_config3()
            torch.cuda.empty_cache()
        if "sizes" in legs:
            res["stft_sizes"] = stft_sizes_leg()
        if "features" in legs:
            try:   # an informational leg: its failure must not cost the bench line
                res["features"] = features_leg()
            except Exception as e:   # noqa: BLE001
                res["features"] = {"error": repr(e)[:200]}
            torch.cuda.empty_cache()
    if not args.no_extras and not args.no_cpu:
        res["cpu_baseline"] = cpu_baseline()
    print(json.dumps(res), flush=True)


def main_dist(args, mode, world):
    """N GPUs through the library's plain-C multi-GPU layer (vv_dsp_dist.h):
    mode "node": this one process drives all N GPUs (vv_dsp_dist_init_all =
    ncclCommInitAll), launching each rank's channel shard on its own device's
    stream (vv_dsp_dist_stft); mode "ranks": torchrun's one process per GPU,
    each a one-slot context of a communicator made by vv_dsp_dist_init_rank
    (ncclCommInitRank; the 128-byte id and the barriers / max-over-ranks go over
    torch.distributed's gloo group -- rendezvous only, no data).  The timed
    region is K steps of the sharded STFT (no data-path collective: channels are
    independent, stft.c:112-144 per channel); the gather of every rank's rows to
    rank 0 (ncclSend/ncclRecv slabs, half-spectrum rows) is timed after it as
    `with_gather`."""
    total_ch = args.channels
    nfr = frames_of(SAMPLES)
    if mode == "node":
        rank0, local = 0, 0
        devs = list(range(world))
        d = vv.Dist.all(devs)
        torch.cuda.set_device(0)
    else:
        rank0 = int(os.environ.get("RANK", "0"))
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        dist.init_process_group("gloo")
        uid = torch.zeros(128, dtype=torch.uint8)
        if rank0 == 0:
            uid.copy_(torch.frombuffer(bytearray(vv.Dist.unique_id()), dtype=torch.uint8))
        dist.broadcast(uid, src=0)
        d = vv.Dist.rank(world, rank0, bytes(uid.tolist()), local)
    if vv.device_count() <= 0:
        raise SystemExit("libvvdsp_amd.so sees no HIP device")
    rccl_ranks = d.comm_count(0)
    if rccl_ranks != world:
        raise SystemExit(f"bench.py: RCCL reports {rccl_ranks} ranks, expected {world}")

    # ---- every local slot's shard: channels [lo, lo + cnt) on its device ----
    slots = []
    root_slot = None
    full = None
    want_gather = world > 1 and args.gather in ("auto", "on") or args.gather == "on"
    for s in range(d.slots):
        r, w, dev = d.rank_info(s)
        lo, cnt = vv.shard_range(total_ch, w, r)
        with torch.cuda.device(dev):
            sig = torch.empty(cnt, SAMPLES, device=dev)
            for c in range(cnt):
                g = torch.Generator(device=torch.device("cuda", dev)).manual_seed(lo + c)
                sig[c].uniform_(-1.0, 1.0, generator=g)
            if r == 0 and want_gather:
                # the root's rows are written in place inside the gathered output
                full = torch.empty(total_ch, nfr, NFFT, device=dev)
                out = full[lo:lo + cnt]
                root_slot = s
            else:
                out = torch.empty(cnt, nfr, NFFT, device=dev)
            # an explicit stream per device for the launches, the events and the RCCL
            # send / receive of the gather (RCCL gets a real stream of the comm's device)
            stream = torch.cuda.Stream(device=dev)
        slots.append({"rank": r, "dev": dev, "lo": lo, "cnt": cnt, "sig": sig, "out": out, "stream": stream})
    st = vv.Stft(NFFT, HOP, vv.WIN_HANN)
    for x in slots:   # inputs generated on each device's default stream: complete before the launch streams read them
        torch.cuda.synchronize(x["dev"])

    def step():
        d.stft(st, [x["sig"] for x in slots], SAMPLES, total_ch, SAMPLES, [x["out"] for x in slots],
               streams=[x["stream"] for x in slots])

    def sync_all():
        for x in slots:
            torch.cuda.synchronize(x["dev"])

    def barrier():
        if mode == "ranks":
            dist.barrier()

    def max_over_ranks(v):
        if mode != "ranks":
            return v
        t = torch.tensor([v], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    for _ in range(args.warmup):
        step()
    ev = [[(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in slots]
          for _ in range(args.steps)]
    sync_all()
    barrier()
    t0 = time.perf_counter()
    for k in range(args.steps):
        for x, (a, _) in zip(slots, ev[k]):
            a.record(x["stream"])
        step()
        for x, (_, b) in zip(slots, ev[k]):
            b.record(x["stream"])
    sync_all()
    barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0)
    # per-device kernel time (HIP events on each device's launch stream); the
    # roofline is quoted on the slowest device of the job
    per_dev = []
    for i, x in enumerate(slots):
        ms = float(np.mean([ev[k][i][0].elapsed_time(ev[k][i][1]) for k in range(args.steps)]))
        byts = x["cnt"] * SAMPLES * 4 + x["cnt"] * nfr * NFFT * 4 + NFFT * 4
        per_dev.append((ms, byts, x["rank"], x["dev"], x["cnt"]))
    slow = max(per_dev)
    if mode == "ranks":
        t = torch.tensor([slow[0], slow[1], slow[2], slow[3], slow[4]], dtype=torch.float64)
        allt = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(allt, t)
        per_dev = [(float(a[0]), int(a[1]), int(a[2]), int(a[3]), int(a[4])) for a in allt]
        slow = max(per_dev)
    kern_ms, bytes_per_launch = slow[0], int(slow[1])
    achieved = bytes_per_launch / (kern_ms * 1e-3) / 1e9

    frames_per_step = total_ch * nfr
    value = frames_per_step * args.steps / elapsed
    ok = all(check_rows(x["sig"], x["out"], (0, x["cnt"] - 1)) for x in slots if x["cnt"])
    if mode == "ranks":
        t = torch.tensor([1.0 if ok else 0.0])
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        ok = bool(t.item() > 0.5)

    gather = None
    if want_gather:
        gather = dist_gather_leg(d, slots, root_slot, full, total_ch, nfr, elapsed / args.steps,
                                 frames_per_step, half=args.gather_bins == "half", sync_all=sync_all,
                                 barrier=barrier, max_over_ranks=max_over_ranks)
    per_gpu = max(x[4] for x in per_dev)
    roof = {"kernel": ROOFLINE_KERNEL + f"; kernel_ms = HIP events around each of the {args.steps} timed launches "
                                        "on every device's launch stream, the slowest device's average",
            "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
            "traffic_source": f"PMC summaries are taken on the one-GPU box ({TRAFFIC_JSON and os.path.basename(TRAFFIC_JSON)}, "
                              "256 channels per launch); not collected for this shard size",
            "bytes_per_launch": bytes_per_launch, "kernel_ms": round(kern_ms, 4),
            "per_device": [{"rank": int(r), "device": int(dv), "channels": int(c), "kernel_ms": round(m, 4),
                            "frac": round(b / (m * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
                           for (m, b, r, dv, c) in sorted(per_dev, key=lambda x: x[2])]}
    launch = (f"one process driving {world} GPUs (vv_dsp_dist_init_all = ncclCommInitAll; one launch per device "
              "per step, vv_dsp_dist_stft)" if mode == "node" else
              f"torchrun: {world} processes, one GPU each (vv_dsp_dist_init_rank = ncclCommInitRank; "
              "gloo for the id broadcast, barriers and max-over-ranks)")
    res = result_line(args, value, world, elapsed, total_ch, per_gpu, nfr,
                      f"dp{world} (channel shards, no data-path collective)", roof, ok)
    res["rccl_ranks"] = rccl_ranks
    res["launch"] = launch
    if gather is not None:
        res["with_gather"] = gather
    if rank0 == 0:
        print(json.dumps(res), flush=True)
    del slots, full
    del d
    if mode == "ranks":
        dist.barrier()
        dist.destroy_process_group()


def dist_gather_leg(d, slots, root_slot, full, total_ch, nfr, compute_s, frames_per_step, half, sync_all, barrier,
                    max_over_ranks):
    """One timed vv_dsp_dist_gather_rows of every rank's [ch][frame][1024] rows
    into rank 0's [256][frame][1024] output (grouped ncclSend / ncclRecv slabs over
    xGMI, each peer on its own link into the root).  `half`: each rank packs bins
    0..512 and the root expands them by mirror symmetry -- bit-identical rows for
    half the xGMI bytes (SURVEY 8e row note 1).  Checked afterwards: sampled rows
    of every rank equal the rank's own rows bit for bit."""
    try:
        sync_all()
        barrier()
        t0 = time.perf_counter()
        d.gather_rows([x["out"] for x in slots], total_ch, nfr, NFFT, full, root=0, half=half,
                      streams=[x["stream"] for x in slots])
        sync_all()
        barrier()
        g = max_over_ranks(time.perf_counter() - t0)
        row_bins = NFFT // 2 + 1 if half else NFFT
        root_ch = vv.shard_range(total_ch, d.rank_info(0)[1], 0)[1]
        gathered = (total_ch - root_ch) * nfr * row_bins * 4
        res = {"gather_s": round(g, 4), "bins_sent": row_bins, "bytes_into_rank0": gathered,
               "xgmi_GBs_into_rank0": round(gathered / g / 1e9, 1),
               "frames_per_s_with_gather": round(frames_per_step / (compute_s + g), 1),
               "note": "one step of compute + one vv_dsp_dist_gather_rows of every rank's magnitude rows to rank 0 "
                       + ("(bins 0..512 packed on each rank, expanded to 1024 on rank 0, bit-identical)"
                          if half else "(all 1024 bins)")}
        if full is not None and len(slots) > 1:   # one process holds every rank's rows: check them
            same = True
            for x in slots:
                if not x["cnt"]:      # fewer channels than ranks: this rank holds no rows
                    continue
                for c in sorted({0, x["cnt"] // 2, x["cnt"] - 1}):
                    for f in (0, 12345, nfr - 1):
                        a = full[x["lo"] + c, f].cpu()
                        b = x["out"][c, f].cpu()
                        same = same and torch.equal(a, b)
            res["rows_bit_identical_after_gather"] = bool(same)
        return res
    except Exception as e:  # report, do not lose the bench line
        return {"error": repr(e)[:300]}



if __name__ == "__main__":
    main()
