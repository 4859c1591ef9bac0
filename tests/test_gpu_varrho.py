"""Variable-density projection (functions.py:1016-1070, 1122-1168,
1296-1328) on the GPU against the oracle.

* the matrix-free operator div((1/rho) grad p) and the per-face Rhie-Chow divergence:
  bit-exact (NumPy restatements of the reference's own array operations);
* the DCT-preconditioned CG projection: the reference's CG does not converge on these
  problems (the mirror-ghost operator is not symmetric and the mean-removed rhs is not in
  its range), so it always runs its iteration cap.  Parity is checked
  iteration by iteration: with maxiter = 1, 2, 5 the GPU result equals the oracle's
  restatement of scipy.sparse.linalg.cg to rounding (dot products reduce in another order,
  the preconditioner's DCT is the LDS FFT vs pocketfft).  On the fixture made by the
  reference itself the run length (all 200 iterations) is reproduced.
"""
import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu


def _case(N=65, ratio=4.0, seed=21):
    from oracle import oracle as O
    X, Y, dx, dy = O.create_grid(N, N, 1.0, 1.0)
    rng = np.random.default_rng(seed)
    phi = np.sqrt((X - 0.5) ** 2 + (Y - 0.45) ** 2) - 0.25
    H = O.smoothed_heaviside(phi, 2 * dx)
    rho = (1 - H) * ratio + H * 1.0
    k = 2 * np.pi
    a = 0.5 * np.sin(k * X) * np.cos(k * Y) + 0.1 * rng.standard_normal((N, N))
    b = -0.5 * np.cos(k * X) * np.sin(k * Y) + 0.1 * rng.standard_normal((N, N))
    p_prev = 0.1 * rng.standard_normal((N, N))
    return dx, dy, rho, a, b, p_prev


def test_variable_operator_and_divergence_bitwise(gpu):
    from oracle import oracle as O
    from pyrmt_amd import functions as F
    dx, dy, rho, a, b, p_prev = _case()
    N = a.shape[0]
    p = np.random.default_rng(3).standard_normal((N, N))
    ir = 1.0 / rho
    np.testing.assert_array_equal(F._apply_variable_poisson(p.ravel(), N, N, dx, dy, ir),
                                  O._apply_variable_poisson(p.ravel(), N, N, dx, dy, ir))
    np.testing.assert_array_equal(F._compute_divergence_rc(a, b, p_prev, 1e-3, rho, dx, dy),
                                  O._compute_divergence_rc(a, b, p_prev, 1e-3, rho, dx, dy))


def test_variable_operator_fixture(gpu):
    from pyrmt_amd import functions as F
    g = golden("varrho")
    N = int(g["N"])
    np.testing.assert_array_equal(
        F._apply_variable_poisson(g["p"].ravel(), N, N, float(g["dx"]), float(g["dy"]),
                                  1.0 / g["rho"]), g["Ap"])
    np.testing.assert_array_equal(
        F._compute_divergence_rc(g["a"], g["b"], g["p_prev"], float(g["dt"]), g["rho"],
                                 float(g["dx"]), float(g["dy"])), g["divU"])


@pytest.mark.parametrize("N,ratio", [(65, 4.0), (128, 10.0)])
@pytest.mark.parametrize("maxiter", [1, 2, 5])
def test_variable_projection_iterations_vs_oracle(gpu, monkeypatch, N, ratio, maxiter):
    from oracle import oracle as O
    from pyrmt_amd import functions as F
    from pyrmt_amd.bc import FreeSlipBox
    dx, dy, rho, a, b, p_prev = _case(N, ratio)
    eig = O._precompute_poisson_eigenvalues(N, N, dx, dy)
    dt = 1e-3
    ra, rb, rp, iters = O.pressure_projection_variable(a, b, dx, dy, dt, rho, 2, 0.0, p_prev,
                                                       eig, maxiter=maxiter)
    monkeypatch.setattr(F, "CG_MAXITER", maxiter)
    ga, gb, gp, _, _ = F.pressure_projection_amg(a, b, dx, dy, dt, rho, FreeSlipBox(),
                                                 p_prev=p_prev, eigenvalues=eig)
    assert F.last_cg_iterations == iters == maxiter
    for got, ref in ((ga, ra), (gb, rb), (gp, rp)):
        np.testing.assert_allclose(got, ref, rtol=0, atol=1e-10 * max(np.abs(ref).max(), 1.0))


def test_variable_projection_reference_fixture(gpu):
    """The reference's own projection on the fixture runs all 200 CG iterations without
    converging (|p| ~ 1e8: the iteration amplifies the rhs component outside the operator's
    range).  What is amplified there is rounding-determined, so only the run length is a
    reproducible property; the iterates themselves are pinned by the maxiter = 1, 2, 5
    parity tests above."""
    from pyrmt_amd import functions as F
    from pyrmt_amd.bc import FreeSlipBox
    g = golden("varrho")
    ga, gb, gp, _, _ = F.pressure_projection_amg(g["a"], g["b"], float(g["dx"]),
                                                 float(g["dy"]), float(g["dt"]), g["rho"],
                                                 FreeSlipBox(), p_prev=g["p_prev"],
                                                 eigenvalues=g["eig"])
    assert F.last_cg_iterations == int(g["iters"]) == F.CG_MAXITER
    assert np.isfinite(gp).all() and np.isfinite(ga).all() and np.isfinite(gb).all()
