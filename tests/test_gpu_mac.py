"""GPU parity of the MAC path (config 5): pyrmt_amd.mac (librmt rmt_mac_*) against the
reference's fixtures (tests/golden/mac_ops.npz, mac_trace.npz) and the oracle.

Bars: bit-exact for the predictor, divergence, face gradients and contact stress (IEEE
arithmetic in the reference's order); the DCT-II projection to 1e-12 relative (FFT
rounding differs from pocketfft's) and machine-zero divergence (tests/test_mac.py:97-113);
the 8-step multi-disc loop at N=64 to 1e-9 (centroids, J range, fields).
"""
import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def M(gpu):
    from pyrmt_amd import mac
    return mac


def test_mac_predictor_bitwise(M):
    g = golden("mac_ops")
    dx, dy = float(g["dx"]), float(g["dy"])
    us, vs = M.momentum_predictor(g["u"], g["v"], 0.01, dx, dy, 1e-3, 1.0, fu=g["fu"],
                                  fv=g["fv"], rho=1.0)
    np.testing.assert_array_equal(us, g["us"])
    np.testing.assert_array_equal(vs, g["vs"])


def test_mac_contact_stress_bitwise(M):
    g = golden("mac_ops")
    dx, dy = float(g["dx"]), float(g["dy"])
    for a, b in zip(M.contact_stress(g["pa"], g["pb"], 2.0, 0.6, 3 * dx, dx, dy),
                    (g["txx"], g["txy"], g["tyy"])):
        np.testing.assert_array_equal(a, b)


def test_mac_divergence_gradient_bitwise(M, oracle):
    from oracle import mac_oracle as MO
    g = golden("mac_ops")
    dx, dy = float(g["dx"]), float(g["dy"])
    np.testing.assert_array_equal(M.divergence(g["us"], g["vs"], dx, dy),
                                  MO.divergence(g["us"], g["vs"], dx, dy))
    np.testing.assert_array_equal(M.gradient_p_u(g["pp"], dx), MO.gradient_p_u(g["pp"], dx))
    np.testing.assert_array_equal(M.gradient_p_v(g["pp"], dy), MO.gradient_p_v(g["pp"], dy))


def test_mac_projection(M):
    g = golden("mac_ops")
    N, dx, dy = int(g["N"]), float(g["dx"]), float(g["dy"])
    eig = M.poisson_eigs_neumann(N, N, dx, dy)
    u, v, phi = M.project(g["us"], g["vs"], dx, dy, 1e-3, 1.0, eig)
    sc = np.abs(g["pp"]).max()
    np.testing.assert_allclose(phi, g["pp"], rtol=0, atol=1e-12 * sc)
    np.testing.assert_allclose(u, g["pu"], rtol=0, atol=1e-12)
    np.testing.assert_allclose(v, g["pv"], rtol=0, atol=1e-12)
    # the headline property of mac.py: machine-zero divergence after the projection
    assert np.abs(M.divergence(u, v, dx, dy)).max() < 1e-9


@pytest.mark.parametrize("N", [64, 256, 1024])
def test_mac_poisson_roundtrip(M, N):
    """tests/test_mac.py:82-95: solve(lap(p)) == p - mean(p), through the DCT-II solve."""
    from oracle import mac_oracle as MO
    dx = dy = 1.0 / N
    rng = np.random.default_rng(N)
    p = rng.standard_normal((N, N))
    eig = M.poisson_eigs_neumann(N, N, dx, dy)
    rhs = MO.divergence(MO.gradient_p_u(p, dx), MO.gradient_p_v(p, dy), dx, dy)
    got = M.solve_poisson_neumann(rhs, eig)
    np.testing.assert_allclose(got, p - p.mean(), rtol=0, atol=1e-9)
    ref = MO.solve_poisson_neumann(rhs, eig)
    np.testing.assert_allclose(got, ref, rtol=0, atol=1e-11)


def test_mac_multi_disc_trace(M):
    """mac_multi_disc_lid.py loop body, N=64, 3 discs (seed 3), 8 steps vs the reference."""
    g = golden("mac_trace")
    N, K = int(g["N"]), int(g["nsteps"])
    sim = M.MacMultiDisc(N, n_discs=3, seed=3)
    np.testing.assert_array_equal(np.array(sim.specs), g["specs"])
    assert sim.dt == float(g["dt"])
    np.testing.assert_array_equal(sim.get("X1", 0), g["X1_0"])
    sim.step(K)
    d = sim.diagnostics()
    np.testing.assert_allclose(d["cx"], g["cx"], rtol=1e-10)
    np.testing.assert_allclose(d["cy"], g["cy"], rtol=1e-10)
    np.testing.assert_allclose(d["minJ"], g["minJ"], rtol=1e-9)
    np.testing.assert_allclose(d["maxJ"], g["maxJ"], rtol=1e-9)
    np.testing.assert_allclose(sim.get("u"), g["u"], rtol=0, atol=1e-9)
    np.testing.assert_allclose(sim.get("v"), g["v"], rtol=0, atol=1e-9)
    for k in range(3):
        np.testing.assert_allclose(sim.get("X1", k), g[f"X1_{k}_end"], rtol=0, atol=1e-9)
        np.testing.assert_allclose(sim.get("X2", k), g[f"X2_{k}_end"], rtol=0, atol=1e-9)


@pytest.mark.parametrize("N,calls", [(64, (3, 1, 4)), (256, (5, 5))])
def test_mac_box_mode_is_bit_identical(M, N, calls):
    """The per-disc passes on each map's support box (mac_boxes, default on) against the
    full-grid passes: every field and diagnostic bit for bit, over several calls (each call
    starts from a full pass; the boxes then come back with the per-step diagnostics).  Also
    the no-op verdict kept on the device (mac_noop_host = 0: every extrapolation pass launched
    and exiting on the device flag) against the default host read-back, and the advection
    through the cell-centre planes (mac_face_sl = 0) against its default face sampling, and
    the SL certificate's exact max |u_c|^2 pass (mac_m2_bound = 0) against the face-maxima
    bound the correction leaves."""
    out = []
    for opts in ({"mac_boxes": 0}, {"mac_boxes": 1}, {"mac_boxes": 1, "mac_noop_host": 0},
                 {"mac_boxes": 1, "mac_face_sl": 0}, {"mac_boxes": 0, "mac_face_sl": 0},
                 {"mac_boxes": 1, "mac_m2_bound": 0}):
        sim = M.MacMultiDisc(N, n_discs=3, seed=3, options=opts)
        for c in calls:
            sim.step(c)
        d = sim.diagnostics()
        f = {f"{n}{k}": sim.get(n, k) for n in ("X1", "X2", "phi") for k in range(3)}
        f.update({n: sim.get(n) for n in ("u", "v", "p")})
        out.append((d, f))
    d0, f0 = out[0]
    for d1, f1 in out[1:]:
        for k in d0:
            np.testing.assert_array_equal(d1[k], d0[k], err_msg=k)
        for k in f0:
            np.testing.assert_array_equal(f1[k], f0[k], err_msg=k)


def test_mac_sim_stops_on_divergence(M):
    """mac_multi_disc_lid.py:100-103: the loop stops after a step with J < 0 (a folded map);
    the record of that step is kept and flagged, later steps are not run."""
    sim = M.MacMultiDisc(64, n_discs=3, seed=3)
    R, cx, cy = sim.specs[0]
    X1 = sim.get("X1", 0)
    sim.field("X1", 0).copy_(sim.torch.as_tensor(2 * cx - X1))   # mirrored map: det G < 0
    sim.step(5)
    d = sim.diagnostics()
    assert len(d["t"]) == 1 and d["diverged"][0] == 1 and d["minJ"][0] < 0
    sim.step(3)
    assert len(sim.diagnostics()["t"]) == 1


def test_mac_sim_raises_on_extrapolation_abort(M, gpu):
    """An aborted extrapolation is an error (RMTError), not a silently unfinished band."""
    from pyrmt_amd import _lib as L
    sim = M.MacMultiDisc(64, n_discs=3, seed=3)
    gpu.functions.extrapolation_mode(3)
    try:
        with pytest.raises(L.RMTError):
            sim.step(1)
    finally:
        gpu.functions.extrapolation_mode(0)


def test_extrapolate_reference_map_raises_on_abort(gpu):
    from pyrmt_amd import _lib as L
    N = 65
    X, Y, dx, dy = gpu.create_grid(N, N, 1.0, 1.0)
    phi = np.sqrt((X - 0.5) ** 2 + (Y - 0.5) ** 2) - 0.2
    m = (phi <= 0).astype(float)
    gpu.functions.extrapolation_mode(3)
    try:
        with pytest.raises(L.RMTError):
            gpu.extrapolate_reference_map(X * m, Y * m, phi, dx, dy, 3)
    finally:
        gpu.functions.extrapolation_mode(0)
    gpu.extrapolate_reference_map(X * m, Y * m, phi, dx, dy, 3)   # mode 0 again: no error
