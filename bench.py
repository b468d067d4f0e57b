#!/usr/bin/env python3
"""bench.py -- MI355X benchmark of the vv-dsp spectral hot path.

Headline (BASELINE.json metric): STFT frames/sec, 1024-pt Hann, hop 256.
Workload per GPU (weak scaling): config 5's per-GPU shard -- 32 channels x
10 min @ 48 kHz (28,800,000 samples, 112,498 frames each; 256 channels at 8
GPUs = config 5), magnitude spectrogram [ch][frame][1024] f32, computed by the
fused gfx950 STFT kernel (one launch per step).  Inputs are synthetic
(uniform[-1,1), seed = global channel id), generated on the device and resident
in HBM before timing.  Channels are independent: ranks process disjoint
channel shards with no collective in the timed region.

Also measured (same JSON line): the roofline of the dominant kernel (HIP events
on the launch stream), config 2 (65536 x 1024 c2c f32 FFT) and config 4 (FIR
overlap-save 257 taps, 8 ch x 2^24) GB/s, and the reference's own CPU STFT
(oracle/_ref, i.e. the reference sources compiled in the build container) timed
on this host's cores on a bounded sample.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)
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
import vvdsp_dist  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
NFFT, HOP = 1024, 256
FS = 48000
CH_PER_GPU = 32
SAMPLES = 10 * 60 * FS        # 10 min per channel
PUBLISHED_CPU_FPS = 24903.0   # BASELINE.md §1 STFT_size_1024 (CPU, 1 thread) -- informational only:
                              # BASELINE.json "published" is empty, so vs_baseline is null
# the newest round's committed PMC summary of this command (profiles/rNN_bench_pmc.json)
TRAFFIC_JSON = (sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_bench_pmc.json"))) or
                [os.path.join(ROOT, "profiles", "r01_bench_pmc.json")])[-1]
METRIC = "STFT frames/sec (1024-pt, hop 256) at 1/2/4/8 GPU; achieved HBM GB/s vs peak"


def frames_of(n):
    return 1 if n < NFFT else 1 + (n - NFFT + HOP) // HOP


def timed_launches(fn, reps, warm=3, warm_s=0.25):
    """Average device time of fn() (one kernel launch each) with HIP events
    recorded on torch's current stream -- the stream the library launches on.
    Warm-up: at least `warm` launches AND `warm_s` seconds of back-to-back
    launches, so the GPU clock has left its idle state (a 0.2 ms kernel timed
    after ten warm-up launches reads up to 30 % slow: the clock ramp is tens of
    ms, measured on the FIR leg)."""
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
    return float(np.mean(ms)), float(np.min(ms))


def fft_c2c_roofline(reps=50):
    """Config 2: 65536 x 1024-pt c2c f32 forward, device resident."""
    B, N = 65536, 1024
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.complex(torch.rand(B, N, device="cuda", generator=g) - 0.5,
                      torch.rand(B, N, device="cuda", generator=g) - 0.5)
    y = torch.empty_like(x)
    plan = vv.FftPlan(N, vv.C2C, vv.FWD, batch=B)
    avg, best = timed_launches(lambda: plan(x, out=y), reps, warm=10)
    planb = vv.FftPlan(N, vv.C2C, vv.BWD, batch=B)
    bavg, bbest = timed_launches(lambda: planb(x, out=y), reps, warm=10)
    byts = 2 * B * N * 8
    del x, y
    return {"workload": "config2: 65536 x 1024-pt c2c f32 forward", "bytes_per_launch": byts,
            "ms_avg": round(avg, 4), "ms_min": round(best, 4),
            "achieved_GBs": round(byts / (avg * 1e-3) / 1e9, 1), "peak_GBs": HBM_PEAK_GBS,
            "frac": round(byts / (avg * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "ffts_per_s": round(B / (avg * 1e-3), 1),
            "backward": {"ms_avg": round(bavg, 4), "ms_min": round(bbest, 4),
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
    avg, best = timed_launches(fn, reps)
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
    return {"workload": "config3: STFT 60 s mono @ 48 kHz, 1024 Hann, hop 256 (11,248 frames)",
            "bytes_per_call": byts, "ms_avg": round(avg, 4), "ms_min": round(best, 4),
            "frames_per_s": round(fr / (avg * 1e-3), 1),
            "frac": round(byts / (avg * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            f"back_to_back_{burst}": {"ms_per_call": round(per, 4), "frames_per_s": round(fr / (per * 1e-3), 1),
                                      "frac": round(byts / (per * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}}


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
    avg, best = timed_launches(lambda: plan(x, out=y), reps, warm=10)
    byts = 2 * nch * n * 4
    del x, y
    return {"workload": "config4: FIR overlap-save 257 taps, 8 ch x 2^24 f32", "bytes_per_launch": byts,
            "ms_avg": round(avg, 4), "ms_min": round(best, 4),
            "achieved_GBs": round(byts / (avg * 1e-3) / 1e9, 1), "peak_GBs": HBM_PEAK_GBS,
            "frac": round(byts / (avg * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "samples_per_s": round(nch * n / (avg * 1e-3), 1)}


def cpu_baseline(threads=None, seconds=15.0):
    """The reference's own vv_dsp_stft_spectrogram (KissFFT, oracle/_ref = the
    reference sources compiled in the build container) on this host's cores:
    `threads` workers each run whole 60 s mono spectrograms back to back until
    `seconds` have passed (a bounded sample of the same per-channel workload)."""
    from vvapi import VvDsp
    path = os.path.join(ROOT, "oracle", "_ref", "libvvref.so")
    if not os.path.exists(path):
        return {"value": None, "unit": "frames/s", "cores": 0, "kind": "reference",
                "sample": "oracle/_ref/libvvref.so missing"}
    ref = VvDsp(path)
    threads = threads or max(1, min(16, len(os.sched_getaffinity(0))))
    n = 60 * FS
    rng = np.random.default_rng(3)
    sigs = [rng.uniform(-1, 1, n).astype(np.float32) for _ in range(threads)]
    t_end = time.perf_counter() + seconds

    def work(i):
        done = 0
        while time.perf_counter() < t_end:
            ref.spectrogram(sigs[i], NFFT, HOP)   # ctypes releases the GIL
            done += 1
        return done

    t0 = time.perf_counter()
    with cf.ThreadPoolExecutor(threads) as ex:
        runs = sum(ex.map(work, range(threads)))
    dt = time.perf_counter() - t0
    frames = runs * frames_of(n)
    t1 = time.perf_counter()
    ref.spectrogram(sigs[0], NFFT, HOP)
    d1 = time.perf_counter() - t1
    return {"value": round(frames / dt, 1), "unit": "frames/s", "cores": threads, "kind": "reference",
            "sample": f"{threads} threads x vv_dsp_stft_spectrogram(60 s @ 48 kHz mono, 1024 Hann, hop 256) "
                      f"back to back for {seconds:.0f} s: {runs} runs = {frames} frames in {dt:.2f} s",
            "single_thread_frames_per_s": round(frames_of(n) / d1, 1)}


def hbm_traffic(channels):
    """HBM bytes per launch from the committed rocprofv3 PMC summary of this
    command (scripts/gpu_prof.sh + scripts/pmc_summary.py --json): FETCH_SIZE x 2
    (gfx950 tallies 128-B reads at 64 B, MI355X_MICROARCH.md §HBM) + WRITE_SIZE,
    both in KiB, summed over the bulk and tail STFT launches of one step."""
    try:
        with open(TRAFFIC_JSON) as f:
            prof = json.load(f)
    except (OSError, ValueError):
        return None, "no PMC summary committed"
    if prof.get("channels_per_gpu") != channels:
        return None, f"PMC summary is for {prof.get('channels_per_gpu')} channels per GPU"
    tot, names = 0.0, []
    for k, c in prof["kernels"].items():
        if k.startswith("vvh::k_stft_pair<1024, 0"):
            tot += (2.0 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024.0
            names.append(k)
    if not names:
        return None, "PMC summary has no k_stft_pair<1024,0,*> entries"
    return round(tot), f"{os.path.relpath(TRAFFIC_JSON, ROOT)} ({prof.get('box', '?')}): " \
                       f"(2*FETCH_SIZE + WRITE_SIZE) KiB x 1024 per dispatch over {', '.join(names)}"


def gather_leg(out, total_ch, compute_s, frames_per_step, rank):
    """One timed RCCL gather (torch.distributed nccl backend = RCCL, point to
    point over xGMI) of every rank's [ch][frame][1024] rows to rank 0."""
    try:
        full = None
        if rank == 0:
            full = torch.empty((total_ch,) + tuple(out.shape[1:]), dtype=out.dtype, device=out.device)
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        vvdsp_dist.gather_rows(out, total_ch, dst=0, out=full)
        torch.cuda.synchronize()
        dist.barrier()
        g = time.perf_counter() - t0
        t = torch.tensor([g], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        g = float(t.item())
        gathered = (total_ch - out.shape[0]) * out[0].numel() * out.element_size()
        del full
        return {"gather_s": round(g, 4), "bytes_into_rank0": gathered,
                "xgmi_GBs_into_rank0": round(gathered / g / 1e9, 1),
                "frames_per_s_with_gather": round(frames_per_step / (compute_s + g), 1),
                "note": "one step of compute + one gather of the full magnitude rows to rank 0"}
    except Exception as e:  # report, do not lose the bench line
        return {"error": repr(e)[:300]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=25)
    ap.add_argument("--channels", type=int, default=CH_PER_GPU, help="channels per GPU")
    ap.add_argument("--no-extras", action="store_true", help="skip config 2/4 and CPU baseline legs")
    ap.add_argument("--gather", choices=["auto", "on", "off"], default="auto",
                    help="after the timed steps, time one RCCL gather of all spectrogram rows to rank 0 "
                         "(config 5 'with gather'; auto = on when N > 1)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    if vv.device_count() <= 0:
        raise SystemExit("libvvdsp_amd.so sees no HIP device")

    # ---- per-rank shard: channels [rank*C, rank*C + C) of the job ----
    C_ = args.channels
    nfr = frames_of(SAMPLES)
    sig = torch.empty(C_, SAMPLES, device="cuda")
    for c in range(C_):
        g = torch.Generator(device="cuda").manual_seed(rank * C_ + c)
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
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for a, b in ev:
        a.record(s)
        step()
        b.record(s)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))

    frames_total = world * C_ * nfr * args.steps
    value = frames_total / elapsed
    bytes_per_launch = C_ * SAMPLES * 4 + C_ * nfr * NFFT * 4 + NFFT * 4
    achieved = bytes_per_launch / (kern_ms * 1e-3) / 1e9

    traffic, traffic_src = hbm_traffic(C_)

    # spot-check one frame row against NumPy f64 so a fast-but-wrong kernel cannot report
    fr = 12345
    x0 = sig[0, fr * HOP: fr * HOP + NFFT].double().cpu().numpy()
    w = np.array([0.5 - 0.5 * np.cos(np.float32(2 * np.pi) / np.float32(NFFT - 1) * np.float32(i))
                  for i in range(NFFT)], np.float64)
    ok = np.allclose(out[0, fr].cpu().numpy(), np.abs(np.fft.fft(x0 * w)), rtol=5e-5, atol=5e-5)
    gather = None
    if world > 1 and (args.gather == "on" or args.gather == "auto"):
        gather = gather_leg(out, C_ * world, elapsed / args.steps, frames_total / args.steps, rank)
    del sig, out, st
    torch.cuda.empty_cache()

    res = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "published_cpu_reference": {"value": PUBLISHED_CPU_FPS, "unit": "frames/s",
                                    "what": "BASELINE.md §1 STFT_size_1024, Ryzen 9 7950X, 1 thread, KissFFT "
                                            "(informational; BASELINE.json publishes no number for this metric)"},
        "dtype": "f32",
        "data": "synthetic: uniform[-1,1) per channel, seed = global channel id, generated in HBM",
        "config": {
            "workload": f"config5 per-GPU shard: multi-channel STFT magnitude, {C_} ch x 10 min @ 48 kHz "
                        f"per GPU ({C_ * world} ch total; 256 ch = config 5 at 8 GPUs), nfft 1024 Hann, hop 256",
            "channels_per_gpu": C_, "samples_per_channel": SAMPLES, "frames_per_channel": nfr,
            "nfft": NFFT, "hop": HOP, "window": "hann (symmetric, window.c:25-36)",
            "output": "[ch][frame][1024] f32 magnitudes (stft.c:133-139)",
            "parallelism": f"dp{world} (channel shards, no data-path collective)"},
        "roofline": {"kernel": "vvh::k_stft_pair<1024,0,0> (LDS-DMA frame spans + Hann + two frames per "
                               "1024-pt complex FFT + |X| rows as full-line streaming stores; the zero-padded "
                               "tail pairs run in the same launch); kernel_ms = HIP events around the launch on "
                               "the launch stream",
                     "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "traffic_source": traffic_src,
                     "bytes_per_launch": bytes_per_launch, "kernel_ms": round(kern_ms, 4)},
        "check_row_vs_numpy_f64": bool(ok),
    }
    if gather is not None:
        res["with_gather"] = gather
    if rank == 0 and not args.no_extras and world == 1:
        res["fft_c2c_1024"] = fft_c2c_roofline()
        torch.cuda.empty_cache()
        res["fir_ols_257"] = fir_roofline()
        torch.cuda.empty_cache()
        res["stft_config3"] = stft_config3()
        torch.cuda.empty_cache()
    if rank == 0 and not args.no_extras and world == 1:
        res["cpu_baseline"] = cpu_baseline()
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
