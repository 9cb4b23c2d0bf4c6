"""bench.py launch contract on the CPU box (no GPU here).

The driver runs `python bench.py --gpus N` (and under torchrun with
WORLD_SIZE = N); a run that cannot give every rank its own GPU must fail
loudly instead of timing fewer ranks (the reference's stage 4 runs N ranks on
N GPUs, stage4-mpi+cuda/poisson_mpi_cuda2.cu:986-990)."""

import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, **env):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "PE_COMM"):
        e.pop(k, None)
    e.update(env)
    return subprocess.run([sys.executable, BENCH, *args], cwd=ROOT, env=e, capture_output=True, text=True,
                          timeout=240)


def test_multi_gpu_without_enough_gpus_fails():
    r = _run(["--gpus", "2", "--steps", "2", "--warmup", "0"])
    assert r.returncode != 0
    assert "needs 2 visible GPUs" in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


def test_world_size_mismatch_fails():
    r = _run(["--gpus", "4", "--steps", "2", "--warmup", "0"], WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    assert r.returncode == 2
    assert "WORLD_SIZE=2" in r.stderr


def test_single_gpu_run_needs_a_device():
    r = _run(["--steps", "2", "--warmup", "0"])
    assert r.returncode == 2
    assert "no HIP device" in r.stderr
