"""Debug probe for k_fir_r32: which output positions (lane a = e % 32,
register b = e // 32 of block e = i + 256) differ from the 16x16x4 kernel."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vv-dsp_amd"))
import vvdsp_amd as vv  # noqa: E402

for name, taps in (("identity", np.eye(1, 257, 0, np.float32)[0]), ("random", np.random.default_rng(1).standard_normal(257).astype(np.float32) / 16)):
    plan = vv.FirPlan(torch.from_numpy(taps))
    for nch, n in ((1, 768 * 6), (1, 700), (2, 768 * 40)):
        x = torch.rand(nch, n, device="cuda") * 2 - 1
        y = plan(x)
        with vv.knobs(FIR_R32=0):
            yo = plan(x)
        torch.cuda.synchronize()
        d = (y - yo).abs().cpu().numpy()
        bad = np.argwhere(d > 1e-4)
        print(name, nch, n, "max", float(d.max()), "bad", len(bad), "of", d.size)
        if len(bad):
            idx = bad[:, 1]
            blk = idx // 768
            e = idx % 768 + 256
            lanes = sorted(set((e % 32).tolist()))
            regs = sorted(set((e // 32).tolist()))
            print("  lanes", lanes[:40])
            print("  regs", regs[:40])
            print("  blocks", sorted(set(blk.tolist()))[:20])
            print("  first", idx[:20].tolist())
