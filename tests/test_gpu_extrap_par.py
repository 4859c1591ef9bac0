"""The parallel extrapolation mode (pyrmt_amd/csrc/extrap_par.hip; opt-in, NOT bit-exact).

It evaluates the reference's fits (functions.py:95-161: same targets, acceptance, weights and
raster-order known sets) as the weighted least-squares plane in integer offsets from the
target, and solves each layer as one triangular system by segments.  Bars:
  * against oracle mode 2 (oracle/rmt_oracle.c: the same centred fits, evaluated serially in
    raster order) to rounding: 1e-12 absolute on maps of O(1);
  * against the reference's arithmetic (oracle mode 0): the same cells filled, values within
    the reference's own rounding of Cramer's rule on absolute coordinates (SURVEY.md App.
    A.2: up to 1.9e-6 at N = 4096);
  * whole loops in this mode against the oracle (the reference): the north-star bars
    (centroid / energy within 1e-6 relative), and bars set from the reference's own noise
    floor for 1-ulp weight noise (tools/noise_floor.py, profiles/r03/noise/).
"""
import os

import numpy as np
import pytest

from test_gpu_parity import _extrap_case

pytestmark = pytest.mark.gpu

CASES = ["disc1024", "slab", "discs3", "rect_l1", "rect_l6", "wide", "corner", "empty", "full",
         "tiny", "disc4096"]


@pytest.fixture
def par(gpu):
    gpu.extrapolation_parallel(True)
    yield gpu
    gpu.extrapolation_parallel(False)


@pytest.mark.parametrize("name", CASES)
def test_parallel_extrapolation_vs_oracle(par, oracle, name):
    X1, X2, phi, dx, dy, layers = _extrap_case(name)
    g1, g2 = par.extrapolate_reference_map(X1, X2, phi, dx, dy, layers)
    oracle.set_ex_mode(2)
    try:
        c1, c2 = oracle.extrapolate_reference_map(X1, X2, phi, dx, dy, layers)
    finally:
        oracle.set_ex_mode(0)
    r1, r2 = oracle.extrapolate_reference_map(X1, X2, phi, dx, dy, layers)
    # the same cells filled as the reference (acceptance is the reference's, exactly)
    filled_ref = (r1 != X1) | (r2 != X2)
    filled_gpu = (g1 != X1) | (g2 != X2)
    np.testing.assert_array_equal(filled_gpu, filled_ref)
    d_c = max(np.abs(g1 - c1).max(), np.abs(g2 - c2).max())
    d_r = max(np.abs(g1 - r1).max(), np.abs(g2 - r2).max())
    print(f"\n[extrap-par {name}] filled {int(filled_ref.sum())}: |gpu - centred oracle| {d_c:.3g}"
          f", |gpu - reference| {d_r:.3g}")
    assert d_c <= 1e-12
    assert d_r <= 1e-5


@pytest.fixture(scope="module")
def fast_oracle(oracle):
    oracle.set_threads(min(16, os.cpu_count() or 1))
    oracle.set_all_cores(True)
    yield oracle
    oracle.set_all_cores(False)


def test_config2_N256_parallel_mode(par, fast_oracle):
    """soft_disc_in_lid_driven N=256, 1000 steps in the parallel mode vs the reference."""
    from pyrmt_amd.simulation import soft_disc_in_lid_driven
    N, S = 256, 1000
    ref = fast_oracle.SoftDisc(N, "lid")
    rec = [ref.step() for _ in range(S)]
    sim = soft_disc_in_lid_driven(N)
    sim.step(S)
    d = sim.diagnostics()
    want = np.array([[r[k] for k in ("t", "cx", "cy", "minJ", "maxJ")] for r in rec])
    got = np.stack([d[k] for k in ("t", "cx", "cy", "minJ", "maxJ")], axis=1)
    rel = np.abs(got - want) / np.abs(want)
    print(f"\n[config2 N=256 x{S}, parallel extrapolation] max rel: t {rel[:, 0].max():.3g} "
          f"cx {rel[:, 1].max():.3g} cy {rel[:, 2].max():.3g} minJ {rel[:, 3].max():.3g} "
          f"maxJ {rel[:, 4].max():.3g}")
    np.testing.assert_allclose(got[:, 0], want[:, 0], rtol=1e-12)
    np.testing.assert_allclose(got[:, 1:3], want[:, 1:3], rtol=1e-6)     # north star
    np.testing.assert_allclose(got[:, 3:], want[:, 3:], rtol=1e-5)


def test_config3_N1024_parallel_mode(par, fast_oracle):
    """disc_in_taylor_green N=1024 WENO5, 20 steps in the parallel mode: the energies."""
    from pyrmt_amd.simulation import disc_in_taylor_green
    N, S = 1024, 20
    ref = fast_oracle.SoftDisc(N, "tg", "weno5")
    rec = [ref.step(energies=True) for _ in range(S)]
    sim = disc_in_taylor_green(N, "weno5")
    sim.step(S)
    d = sim.diagnostics()
    keys = ("t", "ke", "se", "diss", "integ")
    want = np.array([[r[k] for k in keys] + [r["E"]] for r in rec])
    got = np.stack([d[k] for k in keys] + [d["ke"] + d["se"] + d["integ"]], axis=1)
    rel = np.abs(got - want) / np.abs(want)
    print(f"\n[config3 N=1024 x{S}, parallel extrapolation] max rel {dict(zip(keys + ('E',), rel.max(0)))}")
    col = {k: i for i, k in enumerate(keys + ("E",))}
    for k in ("ke", "diss", "integ", "E"):        # north star
        np.testing.assert_allclose(got[:, col[k]], want[:, col[k]], rtol=1e-6)


def test_config4_N4096_parallel_mode(par, fast_oracle):
    """The bench workload, 10 steps in the parallel mode vs the reference."""
    from pyrmt_amd.simulation import soft_disc_in_lid_driven
    N, S = 4096, 10
    ref = fast_oracle.SoftDisc(N, "lid")
    rec = [ref.step() for _ in range(S)]
    sim = soft_disc_in_lid_driven(N)
    sim.step(S)
    d = sim.diagnostics()
    want = np.array([[r[k] for k in ("t", "cx", "cy", "minJ", "maxJ")] for r in rec])
    got = np.stack([d[k] for k in ("t", "cx", "cy", "minJ", "maxJ")], axis=1)
    rel = np.abs(got - want) / np.abs(want)
    print(f"\n[config4 N=4096 x{S}, parallel extrapolation] max rel: cx {rel[:, 1].max():.3g} "
          f"cy {rel[:, 2].max():.3g} minJ {rel[:, 3].max():.3g} maxJ {rel[:, 4].max():.3g}; "
          f"|dX1| {np.abs(sim.get('X1') - ref.X1).max():.3g}")
    np.testing.assert_allclose(got[:, 0], want[:, 0], rtol=1e-12)
    np.testing.assert_allclose(got[:, 1:3], want[:, 1:3], rtol=1e-6)     # north star
