"""bench.py --gpus N started plainly (no torch.distributed.run around it): the launcher
that starts the N ranks itself (bench.py:launch_ranks).  CPU tests: the refusals and the
failure paths; the GPU test that runs config 5 through it is in test_gpu_dist.py."""
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _env():
    drop = ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")
    return {k: v for k, v in os.environ.items() if k not in drop}


def _run(args, timeout=120):
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, timeout=timeout, env=_env())
    return r, time.monotonic() - t0


def test_nccl_more_ranks_than_gpus_fails_fast():
    """--gpus 8 over RCCL with fewer than 8 visible GPUs (here: none) is refused before any
    rank starts"""
    r, secs = _run(["--gpus", "8", "--steps", "1"])
    assert r.returncode == 2, (r.returncode, r.stderr[-500:])
    assert "needs 8 GPUs" in r.stderr
    assert secs < 30


def test_failing_ranks_end_the_launch():
    """every rank fails (no GPU here): the launcher returns non-zero, prints no line"""
    import torch
    if torch.cuda.is_available():
        return  # the ranks would run; the GPU test covers that case
    r, secs = _run(["--gpus", "2", "--backend", "gloo", "--steps", "1", "--no-host-path"])
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert secs < 90


def test_launch_deadline_ends_the_ranks():
    """a deadline shorter than the ranks' start-up: the whole child tree is ended, exit 124"""
    r, secs = _run(["--gpus", "2", "--backend", "gloo", "--steps", "1", "--no-host-path", "--launch-timeout", "0.5"])
    assert r.returncode == 124, (r.returncode, r.stderr[-500:])
    assert "did not finish" in r.stderr
    assert secs < 30
