"""bench.py's launch contract (no GPU needed): an N-GPU number is only ever
reported from N devices.  `--gpus N` with fewer visible GPUs, or a --gpus that
disagrees with torchrun's WORLD_SIZE, exits non-zero before any device is
touched (torch.cuda.device_count() does not initialise the GPU)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, **env):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        e.pop(k, None)
    e.update(env)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=e, cwd=ROOT,
                          capture_output=True, text=True, timeout=300)


def test_more_gpus_than_visible_exits_nonzero():
    p = _run(["--gpus", "999", "--steps", "1", "--warmup", "0", "--no-extras"])
    assert p.returncode != 0
    assert "999" in p.stderr and "refusing" in p.stderr
    assert '"metric"' not in p.stdout


def test_gpus_must_match_world_size():
    p = _run(["--gpus", "3", "--steps", "1", "--warmup", "0"], WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    assert p.returncode != 0 and "WORLD_SIZE=2" in p.stderr
