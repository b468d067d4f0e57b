"""bench.py's N-GPU path on a small job: the one-process form
(vv_dsp_dist_init_all over the visible GPUs, one vv_dsp_dist_stft launch per
device and step, then vv_dsp_dist_gather_rows of half-spectrum rows into rank
0).  On the one-GPU box it runs at N = 1 (--dist-c: the same code with one
device); with two or more GPUs the N = 2 run crosses xGMI and the gathered
rows are compared bit for bit with each rank's own."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--channels", "8", "--steps", "2",
                        "--warmup", "1", "--no-extras"] + args, env=env, cwd=ROOT, capture_output=True, text=True,
                       timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    return json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])


def test_bench_node_mode_one_device():
    d = _bench(["--dist-c", "--gather", "on"])
    assert d["n_gpus"] == 1 and d["rccl_ranks"] == 1 and d["check_row_vs_numpy_f64"]
    assert d["config"]["channels_total"] == 8 and d["value"] > 0
    assert "error" not in d["with_gather"]


def _two():
    import torch
    return torch.cuda.device_count() >= 2


@pytest.mark.skipif(not _two(), reason="needs two visible GPUs")
def test_bench_node_mode_two_devices():
    d = _bench(["--gpus", "2"])
    assert d["n_gpus"] == 2 and d["rccl_ranks"] == 2 and d["check_row_vs_numpy_f64"]
    assert d["with_gather"]["rows_bit_identical_after_gather"] is True
    assert len(d["roofline"]["per_device"]) == 2
