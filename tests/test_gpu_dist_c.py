"""The multi-GPU layer driven from plain C (vv-dsp_amd/tools/vv_dsp_dist_check.c,
no torch, no Python in the process): channel-sharded STFT over every visible
GPU through vv_dsp_dist_init_all (ncclCommInitAll) and vv_dsp_dist_stft, then
vv_dsp_dist_gather_rows of full and half-spectrum rows to roots 0 and N-1,
each gathered spectrogram bit-identical to the single-call rows
(stft.c:112-144 semantics).  On one GPU the RCCL context has one rank (no
send/receive); with two or more visible GPUs the same run crosses xGMI.  The
loopback run covers world 3 on one device."""
import json
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

BIN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "vv-dsp_amd", "bin",
                   "vv_dsp_dist_check")


def _run(args):
    if not os.path.exists(BIN):
        pytest.fail(f"{BIN} missing: run `make -C vv-dsp_amd`")
    p = subprocess.run([BIN] + args, capture_output=True, text=True, timeout=120)
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert line, (p.returncode, p.stdout[-500:], p.stderr[-500:])
    res = json.loads(line[-1])
    res["_stderr"] = p.stderr[-800:]
    res["_lines"] = line
    return p.returncode, res


def test_dist_from_c_all_devices():
    import torch
    rc, res = _run([])
    assert rc == 0 and res["ok"], res
    n = torch.cuda.device_count()
    assert res["world"] == n and res["rccl_ranks"] == n and res["gathers_bit_identical"] == "4/4"


def test_dist_from_c_loopback():
    rc, res = _run(["--loopback", "3"])
    assert rc == 0 and res["ok"] and res["world"] == 3, res
