"""The config-5 MAC step decomposed into row slabs (librmt rmt_mac_slab_*, pyrmt_amd
distributed.MacDistributedSim) against the single-domain rmt_mac_sim step.

G virtual slabs on one GPU (LocalComm): with every slab holding 2^m rows at a multiple of
2^m the fields are bit-identical (same per-element code, row-tree means); uneven slabs
agree to rounding.  Two processes over gloo exercise the TorchComm path.
"""
import numpy as np
import pytest

from test_distributed import _torchrun

pytestmark = pytest.mark.gpu


def _ref(N, K):
    from pyrmt_amd.mac import MacMultiDisc
    ref = MacMultiDisc(N)
    ref.step(K)
    return ref


def _fields(sim):
    return ["u", "v", "p"] + [f"{a}:{k}" for k in range(sim.K) for a in ("X1", "X2", "phi")]


def _get(ref, f):
    base, _, k = f.partition(":")
    return ref.get(base, int(k or 0))


@pytest.mark.parametrize("N,G", [(64, 2), (64, 4), (128, 4)])
def test_mac_slab_bitexact_vs_fused(gpu, N, G):
    from pyrmt_amd import distributed as D
    K = 6
    ref = _ref(N, K)
    sim = D.mac_multi_disc_lid(N, D.LocalComm(G))
    sim.step(K)
    for f in _fields(sim):
        np.testing.assert_array_equal(sim.gather(f), _get(ref, f), err_msg=f)
    d, r = sim.diagnostics(), ref.diagnostics()
    for k in ("t", "dt", "minJ", "maxJ", "umax"):
        np.testing.assert_array_equal(d[k], r[k], err_msg=k)
    np.testing.assert_allclose(d["cx"], r["cx"], rtol=1e-13)
    np.testing.assert_allclose(d["cy"], r["cy"], rtol=1e-13)


def test_mac_slab_uneven(gpu):
    """N=96 over 3 slabs of 32 rows (not tree-aligned): fields to rounding."""
    from pyrmt_amd import distributed as D
    N, K = 96, 5
    ref = _ref(N, K)
    sim = D.mac_multi_disc_lid(N, D.LocalComm(3))
    sim.step(K)
    for f in _fields(sim):
        np.testing.assert_allclose(sim.gather(f), _get(ref, f), rtol=0, atol=1e-10, err_msg=f)


def test_mac_slab_extrapolation_fits(gpu):
    """at N=64 the discs' bands take extrapolated cells: the replicated chain path runs"""
    from pyrmt_amd import distributed as D
    sim = D.mac_multi_disc_lid(64, D.LocalComm(2))
    sim.step(3)
    d = sim.diagnostics()
    assert d["fitted"][-1] > 0 and d["identity_discs"][-1] < sim.K


def test_mac_slab_identity_path_bitexact(gpu):
    """N=8192 (config 5): no extrapolation target fits (det(Aw) ~ 1e-12 < 1e-10), the
    row-split no-op test proves it on every slab and the rim allgather / dense replica are
    skipped; the fields still match the single-domain step bit for bit"""
    from pyrmt_amd import distributed as D
    N, K = 8192, 1
    ref = _ref(N, K)
    sim = D.mac_multi_disc_lid(N, D.LocalComm(4))
    sim.step(K)
    d = sim.diagnostics()
    assert d["identity_discs"][-1] == sim.K and d["fitted"][-1] == 0
    for f in ("u", "v", "p", "X1:0", "X2:1", "phi:2"):
        np.testing.assert_array_equal(sim.gather(f), _get(ref, f), err_msg=f)


def test_mac_slab_config5_G8_two_steps_bitexact(gpu):
    """Config 5 at its own size and rank count (N=8192, mac_multi_disc_lid.py's 8 GPUs as 8
    virtual slabs of 1024 rows): two steps -- the second one from slab-advected, slab-solved
    fields -- match the single-domain step bit for bit on every field, and the per-step
    diagnostics (t, dt, minJ, maxJ, umax) exactly"""
    from pyrmt_amd import distributed as D
    N, K = 8192, 2
    ref = _ref(N, K)
    sim = D.mac_multi_disc_lid(N, D.LocalComm(8))
    sim.step(K)
    d, r = sim.diagnostics(), ref.diagnostics()
    assert len(d["t"]) == K
    for k in ("t", "dt", "minJ", "maxJ", "umax"):
        np.testing.assert_array_equal(d[k], r[k], err_msg=k)
    for f in _fields(sim):
        np.testing.assert_array_equal(sim.gather(f), _get(ref, f), err_msg=f)


def test_mac_slab_two_processes_gloo(gpu):
    out = _torchrun(2, "dist_step.py", 64, 4, "gloo", "mac", timeout=300)
    assert "dist_step ok" in out
