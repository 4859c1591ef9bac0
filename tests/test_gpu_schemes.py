"""GPU parity of the other advection schemes behind advect_reference_map:
semilagrangian_cubic (bicubic, functions.py:228-251, interpolators.py:64-156), central2 and
conservative (functions.py:420-498).  Bars: bit-exact against the oracle (Numba semantics)
and the reference fixture (central / conservative); the fused step with each scheme against
the oracle's driver loop at the north-star bar and tighter."""
import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu


def test_bicubic_and_sl_cubic_bitwise(gpu, oracle):
    g = golden("schemes")
    dx, dy, N = float(g["dx"]), float(g["dy"]), int(g["N"])
    np.testing.assert_array_equal(gpu.bicubic_interpolate(g["f"], g["xq"], g["yq"], dx, dy, N, N),
                                  oracle.bicubic_interpolate(g["f"], g["xq"], g["yq"], dx, dy, N, N))
    X, Y, _, _ = oracle.create_grid(N, N, 1.0, 1.0)
    dt = float(g["dt"])
    args = (g["X1"], g["a"], g["b"], X, Y, dt, dx, dy, g["phi"], 'semilagrangian_cubic')
    np.testing.assert_array_equal(gpu.advect_reference_map(*args),
                                  oracle.advect_reference_map(*args))


@pytest.mark.parametrize("name", ["central2", "conservative"])
def test_central_schemes_bitwise(gpu, name):
    g = golden("schemes")
    dx, dy, N = float(g["dx"]), float(g["dy"]), int(g["N"])
    X, Y, _, _ = gpu.create_grid(N, N, 1.0, 1.0)
    dt = float(g["dt"])
    for k, wc in enumerate((0.0, 2 * dx)):
        got = gpu.advect_reference_map(g["X1"], g["a"], g["b"], X, Y, dt, dx, dy, g["phi"], name, wc)
        np.testing.assert_array_equal(got, g[f"{name}_{k}"])
    np.testing.assert_array_equal(gpu._central2_rhs(g["X1"], g["a"], g["b"], dx, dy, g["phi"], 0.0),
                                  g["c2_rhs"])
    np.testing.assert_array_equal(
        gpu._conservative_rhs(g["X1"], g["a"], g["b"], dx, dy, g["phi"], 2 * dx), g["cons_rhs"])


@pytest.mark.parametrize("scheme", ["semilagrangian_cubic", "central2", "conservative"])
def test_fused_step_other_schemes(gpu, oracle, scheme):
    """The soft-disc loop body (configs 2/4 physics) with each scheme, 6 steps at N=65."""
    from pyrmt_amd.simulation import soft_disc_in_lid_driven
    sim = soft_disc_in_lid_driven(65, scheme=scheme)
    sim.step(6)
    d = sim.diagnostics()
    ref = oracle.SoftDisc(65, "lid", scheme=scheme)
    rec = [ref.step() for _ in range(6)]
    np.testing.assert_allclose(d["cx"], [r["cx"] for r in rec], rtol=1e-12)
    np.testing.assert_allclose(d["cy"], [r["cy"] for r in rec], rtol=1e-12)
    np.testing.assert_allclose(sim.get("X1"), ref.X1, rtol=0, atol=1e-11)
    np.testing.assert_allclose(sim.get("u"), ref.a, rtol=0, atol=1e-10)
