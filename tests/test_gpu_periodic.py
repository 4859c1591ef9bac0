"""GPU parity of the periodic projection branch (functions.py:1177-1290)
against the reference's fixture (tests/golden/periodic.npz) and the reference's own tests
(tests/test_poisson.py:24-78).  Bars: bit-exact for the wrap-around divergence / gradient;
the FFT solve and the projection to 1e-12 of the field scale (rocFFT vs numpy's pocketfft);
the reference's roundtrip (< 1e-10) and divergence-free (< 1e-9) properties."""
import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu


def test_periodic_operators_bitwise(gpu):
    g = golden("periodic")
    dx, dy = float(g["dx"]), float(g["dy"])
    gx, gy = gpu._compute_pressure_gradient_periodic(g["p_true"], dx, dy)
    np.testing.assert_array_equal(gx, g["gx"])
    np.testing.assert_array_equal(gy, g["gy"])
    np.testing.assert_array_equal(gpu._compute_divergence_periodic(g["gx"], g["gy"], dx, dy),
                                  g["lap"])


def test_periodic_fft_solve(gpu):
    g = golden("periodic")
    dx, dy, N = float(g["dx"]), float(g["dy"]), int(g["N"])
    eig = gpu._precompute_poisson_eigenvalues_periodic(N, N, dx, dy)
    np.testing.assert_array_equal(eig[0], g["eig"])
    p = gpu._solve_poisson_fft(g["lap"], eig)
    np.testing.assert_allclose(p, g["p"], rtol=0, atol=1e-12 * np.abs(g["p"]).max())
    # tests/test_poisson.py:24-36: machine-precision roundtrip
    pt = g["p_true"] - g["p_true"].mean()
    assert np.max(np.abs((p - pt)[:-1, :-1])) < 1e-10


def test_periodic_projection(gpu):
    from pyrmt_amd.bc import Periodic

    def periodic_bc(u, v):   # the reference test's callable (tests/test_poisson.py:57-61)
        u = u.copy(); v = v.copy()
        u[:, -1] = u[:, 0]; v[:, -1] = v[:, 0]
        u[-1, :] = u[0, :]; v[-1, :] = v[0, :]
        return u, v
    g = golden("periodic")
    dx, dy, N = float(g["dx"]), float(g["dy"]), int(g["N"])
    eig = gpu._precompute_poisson_eigenvalues_periodic(N, N, dx, dy)
    for bc in (periodic_bc, Periodic()):
        an, bn, pn, _, _ = gpu.pressure_projection_amg(g["a"], g["b"], dx, dy, 1e-2, 1.0, bc,
                                                       p_prev=g["p_prev"], eigenvalues=eig,
                                                       bc_type="periodic")
        np.testing.assert_allclose(an, g["an"], rtol=0, atol=1e-12)
        np.testing.assert_allclose(bn, g["bn"], rtol=0, atol=1e-12)
        np.testing.assert_allclose(pn, g["pn"], rtol=0, atol=1e-12 * np.abs(g["pn"]).max())
        d1 = np.abs(gpu._compute_divergence_periodic(an, bn, dx, dy)[:-1, :-1]).max()
        assert d1 < 1e-9
