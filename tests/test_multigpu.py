"""Multi-GPU jobs on REAL RCCL over xGMI (one process per GPU).

The reference's stage 4 runs N MPI ranks on N GPUs with halo traffic and
per-iteration allreduces between them (stage4-mpi+cuda/poisson_mpi_cuda2.cu:
331-500, :842-925) and publishes 2-GPU rows (Этап_4_1213.pdf p.11-12).  These
tests launch that path for N ∈ {2, 4, 8} with the default transport (the
halo path the construction times fastest — RCCL send/recv, the peer-put
kernel or the sweep's push, overlapped with the interior items or not — and
each path forced; the in-sweep P2P sum or ncclAllReduce for the scalars) and
compare the gathered
solution and the iteration count with the single-GPU solve.  Each case is
skipped unless the box has at least N GPUs (the gpurun boxes of this project
have one: the same code paths run there through the host-staged transport in
tests/test_gpu.py; the driver's 8-GPU node runs these)."""

import json
import os
import signal
import subprocess
import sys

import numpy as np
import pytest

from poisson_ellipse_openmp_mpi_cuda_amd import EllipseProblem, native, solve

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GRID = (600, 840)


def _ndev() -> int:
    try:
        return int(native().device_count())
    except Exception:
        return 0


def _need(n):
    if _ndev() < n:
        pytest.skip(f"needs {n} GPUs (this box has {_ndev()})")


def _run(cmd, env, timeout=240):
    p = subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                         start_new_session=True)
    try:
        out, err = p.communicate(timeout=timeout)
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, signal.SIGKILL)
        p.communicate()
        pytest.fail(f"multi-GPU job hung: {' '.join(cmd)}")
    assert p.returncode == 0, err[-4000:]
    return out


@pytest.fixture(scope="module")
def single():
    return solve(EllipseProblem(*GRID), backend="hip", return_w=True)


@pytest.mark.parametrize("nproc,decomp,allreduce,overlap,halo", [
    # the DEFAULT path (no PE_HALO / PE_OVERLAP): the construction times the
    # candidates on the real transport and keeps the fastest
    (2, "device", "p2p", None, None), (2, "2x1", "rccl", None, None), (2, "1x2", "p2p", None, None),
    (4, "2x2", "p2p", None, None), (4, "device", "rccl", None, None), (4, "2x2", "rccl", "0", None),
    (8, "device", "p2p", None, None), (8, "4x2", "p2p", None, None), (8, "4x2", "rccl", None, None),
    (8, "rows", "p2p", None, None),
    # each path forced: the sweep's push, the peer put, the comm's exchange
    (2, "rows", "p2p", "0", "push"), (8, "rows", "p2p", "0", "push"),
    (4, "rows", "p2p", None, "put"), (8, "4x2", "p2p", "1", "put"),
    (8, "rows", "p2p", "1", "exchange"),
])
def test_rccl_torchrun_matches_single(gpu, single, nproc, decomp, allreduce, overlap, halo, tmp_path):
    _need(nproc)
    from conftest import free_port

    env = dict(os.environ, PE_ALLREDUCE=allreduce, PE_P2P_TIMEOUT_S="30", PE_WATCHDOG_S="60")
    for k, v in (("PE_OVERLAP", overlap), ("PE_HALO", halo)):
        env.pop(k, None)
        if v is not None:
            env[k] = v
    env.pop("PE_COMM", None)
    outp = str(tmp_path / "w.npy")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "-m",
           "poisson_ellipse_openmp_mpi_cuda_amd", "--json", "--quiet", "--decomp", decomp, "--dump", outp,
           str(GRID[0]), str(GRID[1])]
    out = _run(cmd, env)
    d = json.loads([l for l in out.splitlines() if l.startswith("{")][0])
    assert d["ranks"] == nproc and d["Px"] * d["Py"] == nproc
    assert d["comm"].endswith("rccl")
    assert d["comm"].startswith("p2p-allreduce") == (allreduce == "p2p")
    # the halo path: forced, or the fastest candidate as timed (every candidate listed)
    path = d["halo_path"]
    assert d["halo_push"] == path.startswith("push") and d["halo_put"] == path.startswith("put"), d
    assert d["overlap"] == ("+overlap" in path)
    if halo:
        assert path.startswith(halo), path
    if overlap is not None:
        assert d["overlap"] == (overlap == "1"), path
    if allreduce == "rccl":  # no IPC-mapped P2P transport: neither the put nor the push
        assert path.startswith("exchange"), path
    if halo is None and overlap is None:
        names = [n for n, _ in d["halo_candidates"]]
        assert "exchange" in names and "exchange+overlap" in names, names
        if allreduce == "p2p":
            assert "put" in names and "put+overlap" in names, (names, d["put_status"])
            assert ("push" in names) == (d["Py"] == 1), names
    # first cross-device run labels (rank 0): distinct GPUs, peer access to each
    # (xGMI), every self-tested set-up passed, and the transports they chose
    assert len(d["peer_access"]) == nproc and d["peer_access"][0] == -1
    assert all(v == 1 for v in d["peer_access"][1:]), d["peer_access"]
    if allreduce == "p2p":
        assert d["p2p_sum_setup"] == "ok" and d["sums"] == "in-sweep P2P over xGMI"
        assert d["put_status"] == "available", d["put_status"]
    # every block of 600×840 keeps >= 12 rows and columns: three-step everywhere
    assert d["algo"] == "three-step", d["algo"]
    assert abs(d["iters"] - single.iters) <= 1
    np.testing.assert_allclose(np.load(outp), single.w, rtol=0, atol=1e-9)


def test_pe_launch_rccl(gpu):
    """The MPI-free launcher (`pe_launch -n N bin/pe_hip`, file bootstrap of
    the RCCL id) — the reference's `mpirun -np 2 poisson_mpi_cuda M N`."""
    _need(2)
    env = dict(os.environ, PE_WATCHDOG_S="60")
    env.pop("PE_COMM", None)
    out = _run([os.path.join(ROOT, "bin", "pe_launch"), "-n", "2", os.path.join(ROOT, "bin", "pe_hip"), "--json",
                "800", "1200"], env)
    d = json.loads([l for l in out.splitlines() if l.startswith("{")][0])
    assert d["iters"] == 989 and d["ranks"] == 2 and d["converged"]


@pytest.mark.parametrize("nproc", [2, 4, 8])
def test_bench_multi_gpu_contract(gpu, nproc):
    """bench.py under torchrun (the driver's scaling run, shortened): one JSON
    line, valid fixed-work steps, decomposition and transport reported."""
    _need(nproc)
    from conftest import free_port

    env = dict(os.environ)
    env.pop("PE_COMM", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", str(nproc), "--steps", "40", "--warmup", "5", "--grid", "2048", "2048"]
    out = _run(cmd, env, timeout=300)
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == nproc and d["valid"] and d["converged"] and d["iters_converged"] == 1730
    c = d["config"]
    assert c["decomposition"]["Px"] * c["decomposition"]["Py"] == nproc
    assert "rccl" in c["transport"]
    # 2047 rows: slabs while every rank keeps >= 32 rows (decomp.cpp: every N here); the
    # halo path is the construction's fastest candidate on the real transport
    names = [n for n, _ in c["halo_candidates_us_per_sweep"]]
    assert c["halo_path"] in names and "exchange" in names and "put" in names, c["halo_path"]
    assert ("push" in names) == (c["decomposition"]["Py"] == 1), names
    for r in c["ranks"]:  # per-rank diagnostics of the first cross-device run
        assert r["p2p_sum_setup"] == "ok" and r["sums"] == "in-sweep P2P over xGMI"
        assert r["halo_put"] == "available"
        assert r["halo_push"] == ("available" if c["decomposition"]["Py"] == 1 else "off: 2-D blocks")
        assert all(v == 1 for k, v in r["peer_access"].items() if int(k) != r["rank"])


@pytest.mark.parametrize("nproc", [2, 8])
def test_bench_self_launch_real_gpus(gpu, nproc):
    """`python bench.py --gpus N` with no launcher (how the driver may call it):
    N ranks on N distinct GPUs, RCCL saw N ranks, n_gpus == N."""
    _need(nproc)
    env = dict(os.environ)
    for k in ("PE_COMM", "WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    out = _run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(nproc), "--steps", "40", "--warmup",
                "5", "--grid", "2048", "2048", "--no-random-solve"], env, timeout=300)
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    c = d["config"]
    assert d["n_gpus"] == nproc and c["comm_ranks"] == nproc and c["distinct_gpus"] == nproc
    assert d["valid"] and d["converged"] and d["iters_converged"] == 1730
