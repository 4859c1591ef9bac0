"""GPU parity of the MAC IMEX tier (mac.py:243-369): pyrmt_amd.mac
(librmt rmt_mac_lap_lid_hom / rmt_mac_helmholtz / rmt_mac_momentum_predictor_lid_imex)
against the reference's fixture (tests/golden/imex.npz, made by gen_golden.py gen_imex) and
the oracle (oracle/mac_oracle.py, pinned bit-exact to the same fixture).

Bars: the ghost-cell Laplacians bit-exact; the CG / PCG solves and the IMEX predictor to
1e-12 of the solution's scale, with the PCG iteration counts equal (dot products are
deterministic two-pass reductions here, BLAS-ordered in NumPy: rounding-level differences;
the DST goes through rocFFT, scipy's through pocketfft).  The reference's own tests of the
tier (tests/test_imex_wall.py:15-49) are restated: the CG solution satisfies the system to
1e-8, PCG agrees with CG to 1e-6 in <= 12 iterations at N = 64 and 128.
"""
import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def M(gpu):
    from pyrmt_amd import mac
    return mac


@pytest.fixture(scope="module")
def MO():
    from oracle import mac_oracle
    return mac_oracle


def _close(a, b, rel=1e-12):
    a, b = np.asarray(a), np.asarray(b)
    scale = max(np.abs(b).max(), 1e-300)
    assert np.abs(a - b).max() <= rel * scale, np.abs(a - b).max() / scale


def test_lap_lid_hom_bitwise(M):
    g = golden("imex")
    dx, dy = float(g["dx"]), float(g["dy"])
    np.testing.assert_array_equal(M._lap_u_lid_hom(g["u"], dx, dy), g["lap_u"])
    np.testing.assert_array_equal(M._lap_v_lid_hom(g["v"], dx, dy), g["lap_v"])
    np.testing.assert_array_equal(M._dst_helmholtz_eigs(g["rhs_u"].shape, dx, dy), g["eig_u"])


def test_cg_pcg_helmholtz_vs_reference(M):
    g = golden("imex")
    dx, dy, coef = float(g["dx"]), float(g["dy"]), float(g["coef"])
    emb_u = lambda x: np.pad(x, ((0, 0), (1, 1)))
    emb_v = lambda x: np.pad(x, ((1, 1), (0, 0)))
    lu = lambda w: M._lap_u_lid_hom(w, dx, dy)
    lv = lambda w: M._lap_v_lid_hom(w, dx, dy)
    _close(M._cg_helmholtz(g["rhs_u"], lu, emb_u, coef), g["cg_u"])
    cu, cv = [], []
    _close(M._pcg_helmholtz(g["rhs_u"], lu, emb_u, coef, dx, dy, rtol=1e-8, count=cu), g["pcg_u"])
    _close(M._pcg_helmholtz(g["rhs_v"], lv, emb_v, coef, dx, dy, rtol=1e-8, count=cv), g["pcg_v"])
    assert (cu[0], cv[0]) == (int(g["cnt_u"]), int(g["cnt_v"]))


def test_imex_predictor_vs_reference(M):
    g = golden("imex")
    dx, dy = float(g["dx"]), float(g["dy"])
    args = (g["u"], g["v"], float(g["nu"]), dx, dy, float(g["dt"]), float(g["U_lid"]))
    us, vs = M.momentum_predictor_lid_imex(*args)
    _close(us, g["us0"]); _close(vs, g["vs0"])
    us, vs = M.momentum_predictor_lid_imex(*args, fu=g["fu"], fv=g["fv"], rho=1.3, cs2=4.0)
    _close(us, g["us1"]); _close(vs, g["vs1"])
    # the adaptive predictor takes the IMEX branch at this CFL (mac.py:387-390)
    us2, vs2 = M.momentum_predictor_lid_semilag(*args)
    _close(us2, g["us0"]); _close(vs2, g["vs0"])


def test_imex_predictor_one_force_vs_oracle(M, MO):
    """mac.py:345 / :361 apply fu and fv independently: only one of them given (the other
    face kind gets no force) against the oracle's restatement."""
    g = golden("imex")
    dx, dy = float(g["dx"]), float(g["dy"])
    args = (g["u"], g["v"], float(g["nu"]), dx, dy, float(g["dt"]), float(g["U_lid"]))
    for kw in (dict(fu=g["fu"]), dict(fv=g["fv"])):
        us, vs = M.momentum_predictor_lid_imex(*args, rho=1.3, **kw)
        uo, vo = MO.momentum_predictor_lid_imex(*args, rho=1.3, **kw)
        _close(us, uo); _close(vs, vo)


@pytest.mark.parametrize("N", [64, 128, 256])
def test_pcg_vs_oracle_sizes(M, MO, N):
    """Odd interior extents (N - 1 = 63, 127 (prime), 255) through the rocFFT DST."""
    dx = dy = 1.0 / N
    rng = np.random.default_rng(N)
    coef = 2.0e-3 * 0.01
    for kind, shp in ((0, (N, N - 1)), (1, (N - 1, N))):
        rhs = rng.standard_normal(shp)
        emb = (lambda x: np.pad(x, ((0, 0), (1, 1)))) if kind == 0 else \
              (lambda x: np.pad(x, ((1, 1), (0, 0))))
        lap = (lambda w: M._lap_u_lid_hom(w, dx, dy)) if kind == 0 else \
              (lambda w: M._lap_v_lid_hom(w, dx, dy))
        cnt = []
        x = M._pcg_helmholtz(rhs, lap, emb, coef, dx, dy, rtol=1e-8, count=cnt)
        xo, ito = MO.helmholtz(rhs, kind, coef, dx, dy, 1e-8)
        _close(x, xo, 1e-11)
        assert cnt[0] == ito


def test_reference_imex_wall_semantics(M):
    """tests/test_imex_wall.py:15-49 of the reference, on the device path."""
    N = 24; dx = dy = 1.0 / N
    rhs = np.random.default_rng(2).standard_normal((N, N - 1))
    embed = lambda x: np.pad(x, ((0, 0), (1, 1)))
    c = 0.5
    x = M._cg_helmholtz(rhs, lambda w: M._lap_u_lid_hom(w, dx, dy), embed, c)
    resid = x - c * M._lap_u_lid_hom(embed(x), dx, dy) - rhs
    assert np.abs(resid).max() < 1e-8
    for N in (64, 128):
        dx = dy = 1.0 / N
        rhs = np.random.default_rng(4).standard_normal((N, N - 1))
        lap = lambda w: M._lap_u_lid_hom(w, dx, dy)
        coef = 2.0e-3 * 0.01
        x_cg = M._cg_helmholtz(rhs, lap, embed, coef, rtol=1e-8)
        cnt = []
        x_pcg = M._pcg_helmholtz(rhs, lap, embed, coef, dx, dy, rtol=1e-8, count=cnt)
        assert np.abs(x_cg - x_pcg).max() < 1e-6
        assert cnt[0] <= 12


def test_helmholtz_rejects_unknown_operator(M):
    N = 16; dx = dy = 1.0 / N
    rhs = np.ones((N, N - 1))
    with pytest.raises(NotImplementedError):
        M._cg_helmholtz(rhs, lambda w: w[:, 1:-1], lambda x: np.pad(x, ((0, 0), (1, 1))), 0.1)


def test_semilag_branch_vs_reference(M):
    """mac.py:381-442 at CFL 1.76 (> cfl_switch): the cubic-spline midpoint backtrace
    (map_coordinates order 3, 'nearest': prefilter + 16-tap sums here, scipy's C there) and
    the PCG viscosity, with and without forces / the elastic term, to 1e-12 of scale."""
    g = golden("imex_sl")
    args = (g["u"], g["v"], float(g["nu"]), float(g["dx"]), float(g["dy"]), float(g["dt"]),
            float(g["U_lid"]))
    us, vs = M.momentum_predictor_lid_semilag(*args)
    _close(us, g["us0"]); _close(vs, g["vs0"])
    us, vs = M.momentum_predictor_lid_semilag(*args, fu=g["fu"], fv=g["fv"], rho=1.3, cs2=4.0)
    _close(us, g["us1"]); _close(vs, g["vs1"])


@pytest.mark.parametrize("N", [48, 96])
def test_semilag_vs_oracle_sizes(M, MO, N):
    rng = np.random.default_rng(N + 1)
    dx = dy = 1.0 / N
    u = rng.standard_normal((N, N + 1)); u[:, 0] = 0.0; u[:, -1] = 0.0
    v = rng.standard_normal((N + 1, N)); v[0, :] = 0.0; v[-1, :] = 0.0
    args = (u, v, 0.01, dx, dy, 4.0 * dx, 1.0)          # CFL ~ 4 x max|u|: backtraces leave
    us, vs = M.momentum_predictor_lid_semilag(*args)     # the grid (clamped taps)
    uo, vo = MO.momentum_predictor_lid_semilag(*args)
    _close(us, uo, 1e-11); _close(vs, vo, 1e-11)
