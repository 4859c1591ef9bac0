"""Slab-decomposed step (pyrmt_amd/distributed.py, librmt rmt_slab_*).

CPU (gloo): every TorchComm collective against the in-process LocalComm on the same data,
world sizes 2 and 3 (uneven slabs).  GPU: the decomposed step over G virtual slabs is
bit-identical to the fused single-domain step (rmt_sim) when every slab holds 2^m rows at
a multiple of 2^m; with uneven slabs (N=129, G=3) it agrees to rounding; and two
processes sharing the GPU over gloo reproduce the single-domain step (the TorchComm path).
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _torchrun(nproc, script, *args, timeout=240, env=None):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={nproc}", "--master-addr=127.0.0.1", f"--master-port={_port()}",
           os.path.join(ROOT, "tests", "workers", script), *map(str, args)]
    e = dict(os.environ, OMP_NUM_THREADS="1", HSA_ENABLE_IPC_MODE_LEGACY="0", **(env or {}))
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=e)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r.stdout


def test_even_splits():
    from pyrmt_amd.distributed import even_splits
    assert even_splits(4096, 8, 12) == [512 * k for k in range(9)]
    s = even_splits(129, 3, 12)
    assert s[0] == 0 and s[-1] == 129 and all(x % 2 == 0 for x in s[:-1])
    assert all(b - a >= 12 for a, b in zip(s, s[1:]))
    with pytest.raises(ValueError):
        even_splits(20, 2, 12)


@pytest.mark.parametrize("G", [2, 3])
def test_torchcomm_gloo_matches_localcomm(G):
    out = _torchrun(G, "dist_comm.py")
    assert f"dist_comm ok {G}" in out


# ------------------------------------------------------------------------------ GPU --
def _fused(gpu, N, steps):
    from pyrmt_amd.simulation import soft_disc_in_lid_driven
    sim = soft_disc_in_lid_driven(N)
    sim.step(steps)
    return sim


@pytest.mark.gpu
@pytest.mark.parametrize("G", [1, 2, 4])
def test_slab_step_bitexact_vs_fused(gpu, G):
    """N=256: slabs of 256/G rows (aligned row-tree nodes) -> identical bits to rmt_sim."""
    from pyrmt_amd import distributed as D
    N, K = 256, 4
    ref = _fused(gpu, N, K)
    sim = D.soft_disc_in_lid_driven(N, D.LocalComm(G))
    sim.step(K)
    d, r = sim.diagnostics(), ref.diagnostics()
    np.testing.assert_array_equal(d["dt"], r["dt"])
    for f in ("u", "v", "p", "X1", "X2"):
        np.testing.assert_array_equal(sim.gather(f), ref.get(f), err_msg=f)
    np.testing.assert_array_equal(d["minJ"], r["minJ"])
    np.testing.assert_array_equal(d["maxJ"], r["maxJ"])
    np.testing.assert_allclose(d["cx"], r["cx"], rtol=1e-13)
    np.testing.assert_allclose(d["cy"], r["cy"], rtol=1e-13)
    assert d["fitted"][-1] > 0


@pytest.mark.gpu
def test_slab_step_uneven_slabs(gpu):
    """N=129 over 3 slabs (58/58/13-ish rows, not tree-aligned): the means differ in the
    last bits only, so fields agree to rounding and the centroid to 1e-12."""
    from pyrmt_amd import distributed as D
    N, K = 129, 5
    ref = _fused(gpu, N, K)
    sim = D.soft_disc_in_lid_driven(N, D.LocalComm(3))
    sim.step(K)
    d, r = sim.diagnostics(), ref.diagnostics()
    np.testing.assert_allclose(d["cx"], r["cx"], rtol=1e-12)
    np.testing.assert_allclose(d["cy"], r["cy"], rtol=1e-12)
    for f in ("u", "v", "X1", "X2"):
        np.testing.assert_allclose(sim.gather(f), ref.get(f), rtol=0, atol=1e-10, err_msg=f)


@pytest.mark.gpu
def test_slab_step_two_processes_gloo(gpu):
    """The TorchComm path: two processes on cuda:0 over gloo (host-staged collectives)
    match the fused single-domain step."""
    out = _torchrun(2, "dist_step.py", 129, 4, "gloo", timeout=300)
    assert "dist_step ok" in out


@pytest.mark.gpu
def test_slab_step_rccl_one_rank(gpu):
    """The TorchComm path over RCCL (backend "nccl": device tensors, no host staging) at one
    rank -- the one-GPU box cannot place two RCCL ranks on one device -- against the fused
    step."""
    out = _torchrun(1, "dist_step.py", 256, 4, "nccl", timeout=300)
    assert "dist_step ok" in out


@pytest.mark.gpu
def test_bench_multi_rank_path_rccl(gpu):
    """bench.py's N>1 code path (process group with device_id, TorchComm slabs, barriers, MAX
    over ranks) at one rank over RCCL (RMT_BENCH_DIST=1): one JSON line with the slab
    parallelism."""
    import json
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", os.path.join(ROOT, "bench.py"),
           "--gpus", "1", "--grid", "256", "--steps", "3", "--warmup", "1", "--no-cpu-baseline"]
    e = dict(os.environ, OMP_NUM_THREADS="1", HSA_ENABLE_IPC_MODE_LEGACY="0",
             RMT_BENCH_DIST="1")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=e)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["config"]["parallelism"] == "slab1 (row slabs, RCCL)"
    assert line["value"] > 0 and line["steps"] == 3


@pytest.mark.gpu
@pytest.mark.parametrize("G", [2, 4, 8])
def test_config4_slab_step_N4096(gpu, G):
    """Config 4 (soft_disc_in_lid_driven N=4096, 2->4->8 slabs) at its own size: G virtual
    slabs of 4096/G rows (tree-aligned) in one process, 2 steps, bit-identical to the fused
    single-domain step (rmt_sim) -- the rim capacity (~70k entries), halo and all-to-all
    paths at the bench size."""
    from pyrmt_amd import distributed as D
    N, K = 4096, 2
    ref = _fused(gpu, N, K)
    sim = D.soft_disc_in_lid_driven(N, D.LocalComm(G))
    sim.step(K)
    d, r = sim.diagnostics(), ref.diagnostics()
    np.testing.assert_array_equal(d["dt"], r["dt"])
    for f in ("u", "v", "p", "X1", "X2"):
        np.testing.assert_array_equal(sim.gather(f), ref.get(f), err_msg=f)
    np.testing.assert_array_equal(d["minJ"], r["minJ"])
    np.testing.assert_array_equal(d["maxJ"], r["maxJ"])
    np.testing.assert_allclose(d["cx"], r["cx"], rtol=1e-13)
    assert d["fitted"][-1] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("G", [4, 8])
def test_config4_slab_step_N4096_evicting_edge_lists(gpu, G):
    """As above with only 8 edge-tile lists kept on the context (edge_slots = 8): G slabs
    cycle 4 G + 4 (window, grid) keys per step, so lists are evicted, freed and re-uploaded
    every step while stage kernels of both streams are queued -- the configuration of the
    round-4 failure.  3 steps, bit-identical to the fused step."""
    from pyrmt_amd import distributed as D
    from pyrmt_amd import functions as F
    N, K = 4096, 3
    c = F.ctx_for(N, N)
    old = c.get_option("edge_slots")
    c.set_option("edge_slots", 8)
    try:
        ref = _fused(gpu, N, K)
        sim = D.soft_disc_in_lid_driven(N, D.LocalComm(G))
        sim.step(K)
        for f in ("u", "v", "p", "X1", "X2"):
            np.testing.assert_array_equal(sim.gather(f), ref.get(f), err_msg=f)
    finally:
        c.set_option("edge_slots", old)


@pytest.mark.gpu
def test_slab_step_two_processes_gloo_N4096(gpu):
    """The TorchComm path at config 4's own size (two processes on cuda:0 over gloo, 2 steps).
    (The slab step's LDS DCT-I needs 2(N-1) to factor into radices <= 23: N = 4096 and 256
    qualify, 1024 and 2048 do not.)"""
    out = _torchrun(2, "dist_step.py", 4096, 2, "gloo", timeout=400)
    assert "dist_step ok" in out


@pytest.mark.gpu
@pytest.mark.parametrize("G", [2, 4])
def test_slab_step_parallel_extrapolation(gpu, G):
    """The parallel extrapolation mode in the slab step (each rank solves the gathered band,
    extrap_par.hip): bit-identical to the fused step in the same mode."""
    from pyrmt_amd import distributed as D
    N, K = 256, 6
    gpu.extrapolation_parallel(True)
    try:
        ref = _fused(gpu, N, K)
        sim = D.soft_disc_in_lid_driven(N, D.LocalComm(G))
        sim.step(K)
    finally:
        gpu.extrapolation_parallel(False)
    d, r = sim.diagnostics(), ref.diagnostics()
    np.testing.assert_array_equal(d["dt"], r["dt"])
    for f in ("u", "v", "p", "X1", "X2"):
        np.testing.assert_array_equal(sim.gather(f), ref.get(f), err_msg=f)
    np.testing.assert_allclose(d["cx"], r["cx"], rtol=1e-13)


@pytest.mark.gpu
def test_slab_async_rim_overflow_reruns_window(gpu):
    """the asynchronous slab step moves a fixed rim capacity and sees an overflow
    only at the window's read-back.  The window then goes back to its snapshot and through the
    synchronous path (exact counts): forcing a capacity of one entry gives the bits of the
    fused step, with the rerun recorded."""
    from pyrmt_amd import distributed as D
    N, K = 256, 10
    ref = _fused(gpu, N, K)
    sim = D.soft_disc_in_lid_driven(N, D.LocalComm(2))
    sim.sync_every = 4
    sim.step(2)
    sim._rim_cap = 1            # far below the rim: every window overflows until raised
    sim.step(K - 2)
    assert getattr(sim, "reruns", 0) >= 1
    d, r = sim.diagnostics(), ref.diagnostics()
    assert len(d["t"]) == K
    np.testing.assert_array_equal(d["dt"], r["dt"])
    for f in ("u", "v", "p", "X1", "X2"):
        np.testing.assert_array_equal(sim.gather(f), ref.get(f), err_msg=f)
    np.testing.assert_array_equal(d["maxJ"], r["maxJ"])


@pytest.mark.gpu
def test_slab_rerun_after_late_dropped_geometry(gpu):
    """VERDICT r5 weak 3, hypothesis (a).  A window whose rim outgrows the capacity ends with
    the next step's extrapolation geometry queued on each slab's second stream; the rerun
    drops it and runs its first extrapolation in the same workspace.  test_delay_geo starts
    every slab geometry ~10 ms late, so the dropped one is still pending when the rerun begins:
    rmt_slab_drop_geometry makes the main stream wait for it, and the run stays bit-identical
    to the fused step (before that wait, nothing ordered the two)."""
    from pyrmt_amd import distributed as D
    N, K = 256, 10
    ref = _fused(gpu, N, K)
    sim = D.soft_disc_in_lid_driven(N, D.LocalComm(2), options={"test_delay_geo": 3000})
    sim.sync_every = 4
    sim.step(2)
    sim._rim_cap = 1            # the next window overflows and reruns
    sim.step(K - 2)
    assert getattr(sim, "reruns", 0) >= 1
    d, r = sim.diagnostics(), ref.diagnostics()
    np.testing.assert_array_equal(d["dt"], r["dt"])
    for f in ("u", "v", "p", "X1", "X2"):
        np.testing.assert_array_equal(sim.gather(f), ref.get(f), err_msg=f)
    np.testing.assert_array_equal(d["maxJ"], r["maxJ"])


def test_abort_word_detail():
    """The extrapolation's abort word (csrc/extrap.hpp EXA_*) decoded as the host reports it."""
    from pyrmt_amd.distributed import abort_detail
    code = (1 << 30) | (1 << 26) | (5 << 22) | 1234
    assert abort_detail(code) == "chain part 5, fit ordinal 1234"
    assert abort_detail((1 << 30) | (8 << 26)) == "fallback sweep part 0, fit ordinal 0"
    assert abort_detail(1) == "abort word 1"
