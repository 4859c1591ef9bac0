"""oracle -- CPU restatement of the pyRMT RMT time step (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module, and only as the checker or the timed CPU baseline.  The product path
(pyrmt_amd) never imports it.

Structure mirrors what the reference compiles vs. what it runs as NumPy:
  * the reference's Numba @njit kernels are restated in C (rmt_oracle.c, loaded here
    with ctypes): FD gradients, 3rd-order upwind, bilinear interpolation, SL-RK4
    advection, narrow-band extrapolation, WENO5, solid stress; plus the per-cell
    arithmetic of the momentum RHS, BCs, Rhie-Chow divergence and pressure gradient;
  * what the reference does with NumPy/SciPy calls (DCT-I via scipy.fft.dctn, means,
    reductions, the time-step formula, energies, MAC operators) is restated with the
    same NumPy/SciPy calls, so it matches the reference bit for bit.
Pinned against the reference's own outputs in tests/golden/ (tests/test_oracle_golden.py).

Velocity BCs cross this boundary as descriptors (pyrmt_amd.bc) rather than Python
callables; ``bc_kind`` below: 0 identity, 1 no-slip lid (speed ``lid``), 2 free-slip box.
"""
import ctypes
import math
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "librmt_oracle.so")


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def _load():
    if not os.path.exists(_SO):
        build()
    lib = ctypes.CDLL(_SO)
    D, I, L, P = ctypes.c_double, ctypes.c_int, ctypes.c_long, ctypes.c_void_p
    sig = {
        "rmto_set_threads": (None, [I]),
        "rmto_set_all_cores": (None, [I]),
        "rmto_grad_x_2nd": (None, [P, I, I, D, P]),
        "rmto_grad_y_2nd": (None, [P, I, I, D, P]),
        "rmto_diff_upwind_3rd": (None, [P, P, I, I, D, I, P]),
        "rmto_fast_solve_3x3": (None, [P, P, P]),
        "rmto_bilinear": (None, [P, P, P, L, D, D, I, I, P]),
        "rmto_advect_sl_rk4": (None, [P, P, P, P, P, I, I, D, D, D, P]),
        "rmto_extrapolate": (L, [P, P, P, I, I, D, D, I, P, P]),
        "rmto_weno5_rhs": (None, [P, P, P, I, I, D, D, P, D, P]),
        "rmto_advect_weno5_rk3": (None, [P, P, P, I, I, D, D, D, P, D, P]),
        "rmto_solid_stress": (None, [P, P, I, I, D, D, D, D, P, D, D, I, P, P, P, P]),
        "rmto_heaviside": (None, [P, L, D, P]),
        "rmto_apply_bc": (None, [I, D, P, P, I, I]),
        "rmto_momentum_rk4": (None, [P, P, P, P, P, I, D, D, D, D, D, D, D, D, D, P, D, D, I, D,
                                     I, I, P, P, P, P, P, P]),
        "rmto_divergence_rc": (None, [P, P, P, D, I, I, D, D, P]),
        "rmto_velocity_rhs_blended": (None, [P, P, P, P, P, P, P, P, P, P, I, I, D, D, D, P, P]),
        "rmto_divergence_central": (None, [P, P, I, I, D, D, P]),
        "rmto_pressure_gradient": (None, [P, I, I, D, D, P, P]),
        "rmto_pairwise_sum": (D, [P, L]),
        "rmto_bicubic": (None, [P, P, P, L, D, D, I, I, P]),
        "rmto_set_pow_mode": (None, [I]),
        "rmto_set_ex_mode": (None, [I]),
        "rmto_advect_sl_cubic_rk4": (None, [P, P, P, P, P, I, I, D, D, D, P]),
        "rmto_central_rhs": (None, [P, P, P, I, I, D, D, P, D, I, P]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


_lib = _load()


def set_threads(n):
    """OpenMP threads for the kernels the reference runs with Numba parallel=True."""
    _lib.rmto_set_threads(int(n))


def set_all_cores(on):
    """All-cores mode: OpenMP also on the per-cell loops the reference runs serially (same
    results bit for bit; the extrapolation sweep stays serial).  Off = faithful threading."""
    _lib.rmto_set_all_cores(int(bool(on)))


def set_ex_mode(m):
    """Extrapolation fit arithmetic: 0 the reference's; 1 weights nudged +1 ulp (noise-floor
    experiment); 2 the centred restatement librmt's parallel mode computes (rmt_oracle.c)."""
    _lib.rmto_set_ex_mode(int(m))


def _c(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _e(shape):
    return np.empty(shape, dtype=np.float64)


# ── FD helpers / interpolation (utils.py, interpolators.py) ──────────────────────
def grad_central_x_2nd(f, dx):
    f = _c(f); out = _e(f.shape)
    _lib.rmto_grad_x_2nd(_p(f), f.shape[0], f.shape[1], dx, _p(out)); return out


def grad_central_y_2nd(f, dy):
    f = _c(f); out = _e(f.shape)
    _lib.rmto_grad_y_2nd(_p(f), f.shape[0], f.shape[1], dy, _p(out)); return out


def diff_upwind_3rd(f, u, h, axis):
    f = _c(f); u = _c(u); out = _e(f.shape)
    _lib.rmto_diff_upwind_3rd(_p(f), _p(u), f.shape[0], f.shape[1], h, int(axis), _p(out))
    return out


def fast_solve_3x3(A, b):
    A = _c(A); b = _c(b); x = _e(3)
    _lib.rmto_fast_solve_3x3(_p(A), _p(b), _p(x)); return x


def bilinear_interpolate(u, xq, yq, dx, dy, Nx, Ny):
    u = _c(u); xq = _c(xq); yq = _c(yq); out = _e(xq.shape)
    _lib.rmto_bilinear(_p(u), _p(xq), _p(yq), xq.size, dx, dy, int(Nx), int(Ny), _p(out))
    return out


# ── reference-map transport (functions.py:48-542) ─────────────────────────────────
def advect_semilagrangian_rk4(q, a, b, X, Y, dt, dx, dy):
    q, a, b, X, Y = map(_c, (q, a, b, X, Y)); out = _e(q.shape)
    _lib.rmto_advect_sl_rk4(_p(q), _p(a), _p(b), _p(X), _p(Y), q.shape[0], q.shape[1],
                            dt, dx, dy, _p(out))
    return out


def extrapolate_reference_map(X1, X2, phi, dx, dy, max_layers):
    X1, X2, phi = map(_c, (X1, X2, phi)); o1 = _e(X1.shape); o2 = _e(X1.shape)
    _lib.rmto_extrapolate(_p(X1), _p(X2), _p(phi), X1.shape[0], X1.shape[1], dx, dy,
                          int(max_layers), _p(o1), _p(o2))
    return o1, o2


def _weno5_rhs(q, a, b, dx, dy, phi, w_cut):
    q, a, b, phi = map(_c, (q, a, b, phi)); out = _e(q.shape)
    _lib.rmto_weno5_rhs(_p(q), _p(a), _p(b), q.shape[0], q.shape[1], dx, dy, _p(phi), w_cut,
                        _p(out))
    return out


def advect_weno5_rk3(q, a, b, dx, dy, dt, phi, w_cut=0.0):
    q, a, b, phi = map(_c, (q, a, b, phi)); out = _e(q.shape)
    _lib.rmto_advect_weno5_rk3(_p(q), _p(a), _p(b), q.shape[0], q.shape[1], dx, dy, dt,
                               _p(phi), w_cut, _p(out))
    return out


def set_pow_mode(on):
    """Pure-Python semantics for cubic_convolution's x**2 / x**3 (libm pow, as the golden
    generator runs it) instead of Numba's multiplications (the default)."""
    _lib.rmto_set_pow_mode(int(bool(on)))


def bicubic_interpolate(u, xq, yq, dx, dy, Nx, Ny):
    """interpolators.py:64-142."""
    u, xq, yq = map(_c, (u, xq, yq)); out = _e(xq.shape)
    _lib.rmto_bicubic(_p(u), _p(xq), _p(yq), xq.size, dx, dy, Nx, Ny, _p(out)); return out


def advect_semilagrangian_cubic_rk4(q, a, b, X, Y, dt, dx, dy):
    """functions.py:228-251."""
    q, a, b, X, Y = map(_c, (q, a, b, X, Y)); out = _e(q.shape)
    _lib.rmto_advect_sl_cubic_rk4(_p(q), _p(a), _p(b), _p(X), _p(Y), q.shape[0], q.shape[1], dt,
                                  dx, dy, _p(out))
    return out


def _central_rhs(q, a, b, dx, dy, phi, w_cut, mode):
    q, a, b, phi = map(_c, (q, a, b, phi)); out = _e(q.shape)
    _lib.rmto_central_rhs(_p(q), _p(a), _p(b), q.shape[0], q.shape[1], dx, dy, _p(phi), w_cut,
                          mode, _p(out))
    return out


def _central2_rhs(q, a, b, dx, dy, phi, w_cut):
    return _central_rhs(q, a, b, dx, dy, phi, w_cut, 0)


def _conservative_rhs(q, a, b, dx, dy, phi, w_cut):
    return _central_rhs(q, a, b, dx, dy, phi, w_cut, 1)


def _ssprk3(q, dt, rhs):
    """functions.py:447-463 / 492-498: Shu-Osher SSP-RK3 with NumPy combinations."""
    q1 = q + dt * rhs(q)
    q2 = 0.75 * q + 0.25 * (q1 + dt * rhs(q1))
    return (1.0 / 3.0) * q + (2.0 / 3.0) * (q2 + dt * rhs(q2))


def advect_central2_rk3(q, a, b, dx, dy, dt, phi, w_cut=0.0):
    return _ssprk3(_c(q), dt, lambda s: _central2_rhs(s, a, b, dx, dy, phi, w_cut))


def advect_conservative_rk3(q, a, b, dx, dy, dt, phi, w_cut=0.0):
    return _ssprk3(_c(q), dt, lambda s: _conservative_rhs(s, a, b, dx, dy, phi, w_cut))


def advect_reference_map(q, a, b, X, Y, dt, dx, dy, phi, scheme='semilagrangian', w_cut=0.0):
    """functions.py:501-542 dispatcher (the two schemes on the hot path)."""
    if not (np.all(np.isfinite(a)) and np.all(np.isfinite(b))):
        raise FloatingPointError("advect_reference_map: non-finite velocity")
    if scheme == 'semilagrangian':
        return advect_semilagrangian_rk4(q, a, b, X, Y, dt, dx, dy)
    if scheme == 'weno5':
        return advect_weno5_rk3(q, a, b, dx, dy, dt, phi, w_cut)
    if scheme == 'semilagrangian_cubic':
        return advect_semilagrangian_cubic_rk4(q, a, b, X, Y, dt, dx, dy)
    if scheme == 'central2':
        return advect_central2_rk3(q, a, b, dx, dy, dt, phi, w_cut)
    if scheme == 'conservative':
        return advect_conservative_rk3(q, a, b, dx, dy, dt, phi, w_cut)
    raise ValueError("Unknown advection scheme %r" % (scheme,))


def rebuild_phi_disc(X1, X2, x0, y0, R):
    """functions.py:1366 + benchmarks/common.py:55-57 (disc signed distance)."""
    return np.sqrt((X1 - x0) ** 2 + (X2 - y0) ** 2) - R


# ── stress / momentum (functions.py:545-944) ──────────────────────────────────────
def solid_cauchy_stress(X1, X2, dx, dy, mu_s, kappa, phi, w_cut=0.0, detg_clamp=0.0,
                        isochoric=False):
    X1, X2, phi = map(_c, (X1, X2, phi))
    outs = [_e(X1.shape) for _ in range(4)]
    _lib.rmto_solid_stress(_p(X1), _p(X2), X1.shape[0], X1.shape[1], dx, dy, mu_s, kappa,
                           _p(phi), w_cut, detg_clamp, int(bool(isochoric)), *map(_p, outs))
    return tuple(outs)


def smoothed_heaviside(x, w_t):
    x = _c(x); out = _e(x.shape)
    _lib.rmto_heaviside(_p(x), x.size, w_t, _p(out)); return out


def apply_bc(bc_kind, lid, u, v):
    u = _c(u).copy(); v = _c(v).copy()
    _lib.rmto_apply_bc(int(bc_kind), float(lid), _p(u), _p(v), u.shape[0], u.shape[1])
    return u, v


def momentum_step_rk4(u, v, p, X1, X2, bc_kind, lid, mu_s, kappa, eta_s, dx, dy, dt, rho_s,
                      rho_f, phi, mu_f, w_t, stress_band=False, detg_clamp=3.0):
    u, v, p, X1, X2, phi = map(_c, (u, v, p, X1, X2, phi))
    outs = [_e(u.shape) for _ in range(6)]
    _lib.rmto_momentum_rk4(_p(u), _p(v), _p(p), _p(X1), _p(X2), int(bc_kind), float(lid),
                           mu_s, kappa, eta_s, dx, dy, dt, rho_s, rho_f, _p(phi), mu_f, w_t,
                           int(bool(stress_band)), detg_clamp, u.shape[0], u.shape[1],
                           *map(_p, outs))
    return tuple(outs)


def velocity_rhs_blended_optimized(u, v, p, sxx, sxy, syy, dx, dy, phi, mu_f, H, dH_dx, dH_dy,
                                   rho_local, st_force_x, st_force_y):
    """functions.py:897-944 (phi, dH_dx, dH_dy unused, as in the reference)."""
    shp = np.shape(u)
    u, v, p, sxx, sxy, syy = map(_c, (u, v, p, sxx, sxy, syy))
    H = _c(np.broadcast_to(H, shp)); rho = _c(np.broadcast_to(rho_local, shp))
    scalar0 = np.ndim(st_force_x) == 0 and np.ndim(st_force_y) == 0 and \
        float(st_force_x) == 0.0 and float(st_force_y) == 0.0
    fx = None if scalar0 else _c(np.broadcast_to(st_force_x, shp))
    fy = None if scalar0 else _c(np.broadcast_to(st_force_y, shp))
    ru = _e(shp); rv = _e(shp)
    _lib.rmto_velocity_rhs_blended(_p(u), _p(v), _p(p), _p(sxx), _p(sxy), _p(syy), _p(H),
                                   _p(rho), fx.ctypes.data if fx is not None else None,
                                   fy.ctypes.data if fy is not None else None, shp[0], shp[1],
                                   dx, dy, mu_f, _p(ru), _p(rv))
    return ru, rv


# ── projection (functions.py:1005-1364) ──────────────────────────────────────────
def _precompute_poisson_eigenvalues(Nx, Ny, dx, dy):
    """functions.py:1091-1104: DCT-I symbol of the ghost-mirrored Neumann Laplacian."""
    lx = -2.0 * (1.0 - np.cos(np.pi * np.arange(Nx) / (Nx - 1))) / dx ** 2
    ly = -2.0 * (1.0 - np.cos(np.pi * np.arange(Ny) / (Ny - 1))) / dy ** 2
    eig = lx[np.newaxis, :] + ly[:, np.newaxis]
    eig[0, 0] = 1.0
    return eig


def _solve_poisson_dct(rhs, eig):
    """functions.py:1107-1119: unnormalised DCT-I both ways (scipy/pocketfft, as the
    reference), (0,0) mode divided by 1 and removed with the mean."""
    from scipy.fft import dctn, idctn
    p = idctn(dctn(rhs, type=1) / eig, type=1)
    p -= np.mean(p)
    return p


def _is_variable_rho(rho):
    return isinstance(rho, np.ndarray) and rho.ndim == 2 and np.ptp(rho) > 1e-10


def _compute_divergence_rc_variable(a_star, b_star, p_prev, dt, rho, dx, dy):
    """functions.py:1016-1070 with a variable rho array (NumPy, the reference's operations
    in its order): per-face d_f = dt * 0.5 * (1/rho_l + 1/rho_r)."""
    Ny, Nx = a_star.shape
    divU = np.zeros((Ny, Nx))
    dpdx_cc = np.zeros((Ny, Nx)); dpdy_cc = np.zeros((Ny, Nx))
    dpdx_cc[:, 1:-1] = (p_prev[:, 2:] - p_prev[:, :-2]) / (2.0 * dx)
    dpdx_cc[:, 0] = (-3.0 * p_prev[:, 0] + 4.0 * p_prev[:, 1] - p_prev[:, 2]) / (2.0 * dx)
    dpdx_cc[:, -1] = (3.0 * p_prev[:, -1] - 4.0 * p_prev[:, -2] + p_prev[:, -3]) / (2.0 * dx)
    dpdy_cc[1:-1, :] = (p_prev[2:, :] - p_prev[:-2, :]) / (2.0 * dy)
    dpdy_cc[0, :] = (-3.0 * p_prev[0, :] + 4.0 * p_prev[1, :] - p_prev[2, :]) / (2.0 * dy)
    dpdy_cc[-1, :] = (3.0 * p_prev[-1, :] - 4.0 * p_prev[-2, :] + p_prev[-3, :]) / (2.0 * dy)
    inv_rho = 1.0 / rho
    u_face = 0.5 * (a_star[:, :-1] + a_star[:, 1:])
    face_dpdx = (p_prev[:, 1:] - p_prev[:, :-1]) / dx
    avg_dpdx = 0.5 * (dpdx_cc[:, :-1] + dpdx_cc[:, 1:])
    d_f_x = dt * 0.5 * (inv_rho[:, :-1] + inv_rho[:, 1:])
    u_face_rc = u_face - d_f_x * (face_dpdx - avg_dpdx)
    v_face = 0.5 * (b_star[:-1, :] + b_star[1:, :])
    face_dpdy = (p_prev[1:, :] - p_prev[:-1, :]) / dy
    avg_dpdy = 0.5 * (dpdy_cc[:-1, :] + dpdy_cc[1:, :])
    d_f_y = dt * 0.5 * (inv_rho[:-1, :] + inv_rho[1:, :])
    v_face_rc = v_face - d_f_y * (face_dpdy - avg_dpdy)
    divU[1:-1, 1:-1] = ((u_face_rc[1:-1, 1:] - u_face_rc[1:-1, :-1]) / dx +
                        (v_face_rc[1:, 1:-1] - v_face_rc[:-1, 1:-1]) / dy)
    return divU


def _apply_variable_poisson(p_flat, Nx, Ny, dx, dy, inv_rho):
    """functions.py:1122-1168 (NumPy, same operations): div((1/rho) grad p), face-averaged
    1/rho, mirror ghosts."""
    p = p_flat.reshape((Ny, Nx))
    result = np.zeros_like(p)
    cx = 1.0 / dx ** 2
    cy = 1.0 / dy ** 2
    px = np.empty((Ny, Nx + 2)); px[:, 1:-1] = p; px[:, 0] = p[:, 1]; px[:, -1] = p[:, -2]
    py = np.empty((Ny + 2, Nx)); py[1:-1, :] = p; py[0, :] = p[1, :]; py[-1, :] = p[-2, :]
    rx = np.empty((Ny, Nx + 2)); rx[:, 1:-1] = inv_rho
    rx[:, 0] = inv_rho[:, 1]; rx[:, -1] = inv_rho[:, -2]
    be = 0.5 * (rx[:, 1:-1] + rx[:, 2:]); bw = 0.5 * (rx[:, 0:-2] + rx[:, 1:-1])
    result += cx * (be * (px[:, 2:] - p) - bw * (p - px[:, :-2]))
    ry = np.empty((Ny + 2, Nx)); ry[1:-1, :] = inv_rho
    ry[0, :] = inv_rho[1, :]; ry[-1, :] = inv_rho[-2, :]
    bn = 0.5 * (ry[1:-1, :] + ry[2:, :]); bs = 0.5 * (ry[0:-2, :] + ry[1:-1, :])
    result += cy * (bn * (py[2:, :] - p) - bs * (p - py[:-2, :]))
    return result.ravel()


def cg(matvec, b, psolve, rtol, maxiter):
    """scipy.sparse.linalg.cg (scipy 1.15, x0 = 0, atol = 0) restated: the reference calls it
    with tol=1e-6, maxiter=200 and the DCT solve as M (functions.py:1322-1325).  Returns
    (x, iterations run)."""
    r = b.copy()
    x = np.zeros_like(b)
    bnrm2 = np.linalg.norm(b)
    if bnrm2 == 0:
        return b.copy(), 0
    atol = rtol * bnrm2
    rho_prev, p = None, None
    for it in range(maxiter):
        if np.linalg.norm(r) < atol:
            return x, it
        z = psolve(r)
        rho_cur = np.dot(r, z)
        if it > 0:
            beta = rho_cur / rho_prev
            p *= beta
            p += z
        else:
            p = np.empty_like(r)
            p[:] = z[:]
        q = matvec(p)
        alpha = rho_cur / np.dot(p, q)
        x += alpha * p
        r -= alpha * q
        rho_prev = rho_cur
    return x, maxiter


def pressure_projection_variable(a_star, b_star, dx, dy, dt, rho, bc_kind, lid, p_prev, eig,
                                 rtol=1e-6, maxiter=200):
    """functions.py:1296-1328 + :1347-1364 (variable density): returns (a, b, p, iters)."""
    Ny, Nx = a_star.shape
    divU = (_compute_divergence_rc_variable(a_star, b_star, p_prev, dt, rho, dx, dy)
            if p_prev is not None else _compute_divergence(a_star, b_star, dx, dy))
    rhs = (divU / dt).ravel()
    rhs -= np.mean(rhs)
    inv_rho = 1.0 / rho
    x, iters = cg(lambda v: _apply_variable_poisson(v, Nx, Ny, dx, dy, inv_rho), rhs,
                  lambda r: _solve_poisson_dct(r.reshape((Ny, Nx)), eig).ravel(), rtol, maxiter)
    pc = x.reshape((Ny, Nx))
    pc -= np.mean(pc)
    gx, gy = _compute_pressure_gradient(pc, dx, dy)
    a, b = apply_bc(bc_kind, lid, a_star - (dt / rho) * gx, b_star - (dt / rho) * gy)
    p = p_prev + pc if p_prev is not None else pc
    p -= np.mean(p)
    return a, b, p, iters


def _compute_divergence_rc(a, b, p, dt, rho, dx, dy):
    if _is_variable_rho(rho):
        return _compute_divergence_rc_variable(a, b, p, dt, rho, dx, dy)
    d_f = dt / float(np.mean(rho))
    a, b, p = map(_c, (a, b, p)); out = _e(a.shape)
    _lib.rmto_divergence_rc(_p(a), _p(b), _p(p), d_f, a.shape[0], a.shape[1], dx, dy, _p(out))
    return out


def _compute_divergence(a, b, dx, dy):
    a, b = map(_c, (a, b)); out = _e(a.shape)
    _lib.rmto_divergence_central(_p(a), _p(b), a.shape[0], a.shape[1], dx, dy, _p(out))
    return out


def _compute_pressure_gradient(p, dx, dy):
    p = _c(p); gx = _e(p.shape); gy = _e(p.shape)
    _lib.rmto_pressure_gradient(_p(p), p.shape[0], p.shape[1], dx, dy, _p(gx), _p(gy))
    return gx, gy


def pressure_projection(a_star, b_star, dx, dy, dt, rho, bc_kind, lid, p_prev, eig):
    """functions.py:1255-1364, Neumann branch, constant density, DCT direct solve."""
    if isinstance(rho, np.ndarray) and np.ptp(rho) > 1e-10:
        raise NotImplementedError("variable-density projection (CG) is not on the hot path")
    divU = (_compute_divergence_rc(a_star, b_star, p_prev, dt, rho, dx, dy)
            if p_prev is not None else _compute_divergence(a_star, b_star, dx, dy))
    pc = _solve_poisson_dct(rho * divU / dt, eig)
    gx, gy = _compute_pressure_gradient(pc, dx, dy)
    a, b = apply_bc(bc_kind, lid, a_star - (dt / rho) * gx, b_star - (dt / rho) * gy)
    p = p_prev + pc if p_prev is not None else pc
    p -= np.mean(p)
    return a, b, p


# ── periodic branch (functions.py:1171-1252, 1277-1290): NumPy in the reference ─────
def _precompute_poisson_eigenvalues_periodic(Nx, Ny, dx, dy):
    mx, my = Nx - 1, Ny - 1
    lx = -(np.sin(2.0 * np.pi * np.arange(mx) / mx) / dx) ** 2
    ly = -(np.sin(2.0 * np.pi * np.arange(my) / my) / dy) ** 2
    eig = lx[np.newaxis, :] + ly[:, np.newaxis]
    null = np.abs(eig) < 1e-12
    eig = eig.copy()
    eig[null] = 1.0
    return eig, null


def _tile_overlap(red, Ny, Nx):
    out = np.empty((Ny, Nx))
    out[:-1, :-1] = red
    out[-1, :-1] = red[0, :]
    out[:-1, -1] = red[:, 0]
    out[-1, -1] = red[0, 0]
    return out


def _solve_poisson_fft(rhs_full, eigenvalues_periodic):
    eig, null = eigenvalues_periodic
    Ny, Nx = rhs_full.shape
    r = rhs_full[:-1, :-1].copy()
    r -= np.mean(r)
    h = np.fft.fft2(r) / eig
    h[null] = 0.0
    p = _tile_overlap(np.real(np.fft.ifft2(h)), Ny, Nx)
    p -= np.mean(p)
    return p


def _wrap_d(f, axis, h):
    return (np.roll(f, -1, axis=axis) - np.roll(f, 1, axis=axis)) / (2.0 * h)


def _compute_divergence_periodic(a, b, dx, dy):
    Ny, Nx = a.shape
    return _tile_overlap(_wrap_d(a[:-1, :-1], 1, dx) + _wrap_d(b[:-1, :-1], 0, dy), Ny, Nx)


def _compute_pressure_gradient_periodic(p, dx, dy):
    Ny, Nx = p.shape
    r = p[:-1, :-1]
    return _tile_overlap(_wrap_d(r, 1, dx), Ny, Nx), _tile_overlap(_wrap_d(r, 0, dy), Ny, Nx)


def pressure_projection_periodic(a_star, b_star, dx, dy, dt, rho, bc_kind, lid, p_prev, eig):
    """functions.py:1277-1290 (bc_kind 3 = the overlap-grid periodic copy)."""
    divU = _compute_divergence_periodic(a_star, b_star, dx, dy)
    rho_bar = float(np.mean(rho)) if isinstance(rho, np.ndarray) else float(rho)
    pc = _solve_poisson_fft(rho_bar * divU / dt, eig)
    gx, gy = _compute_pressure_gradient_periodic(pc, dx, dy)
    a, b = apply_bc(bc_kind, lid, a_star - (dt / rho) * gx, b_star - (dt / rho) * gy)
    p = (p_prev + pc) if p_prev is not None else pc
    p -= np.mean(p)
    return a, b, p


def compute_timestep(a, b, dx, dy, CFL, dt_min_cap, mu_s, rho_s, gamma, rho_f, mu_f=0.0,
                     eta_s=0.0, kappa=0.0):
    """functions.py:165-192."""
    cs = np.sqrt((kappa + mu_s * 4.0 / 3.0) / (rho_s + 1e-12))
    dts = [CFL * dx / (cs + 1e-14), CFL * dx / (np.max(np.sqrt(a ** 2 + b ** 2)) + 1e-6)]
    if gamma > 1e-12:
        dts.append(np.sqrt((0.5 * (rho_s + rho_f) * dx ** 3) / (2 * np.pi * gamma)) * 0.5)
    else:
        dts.append(1.0)
    mu_max, rho_min = max(mu_f, eta_s), min(rho_s, rho_f)
    dts.append(CFL * rho_min * dx ** 2 / (4.0 * mu_max) if (mu_max > 1e-12 and rho_min > 1e-12)
               else 1.0)
    return min(*dts, dt_min_cap)


# ── diagnostics (benchmarks/common.py:110-115, output.py:6-193) ──────────────────
def disc_centroid(phi, X, Y):
    m = phi <= 0.0
    return (X[m].mean(), Y[m].mean()) if np.any(m) else (np.nan, np.nan)


def divergence_2d_interior(u, v, dx, dy, pad=3):
    """output.py:195-211 (the same slices and operation order)."""
    d = np.zeros_like(u)
    d[pad:-pad, pad:-pad] = ((u[pad:-pad, pad + 1:-pad + 1] - u[pad:-pad, pad - 1:-pad - 1]) / (2 * dx)
                             + (v[pad + 1:-pad + 1, pad:-pad] - v[pad - 1:-pad - 1, pad:-pad]) / (2 * dy))
    return d, d[pad:-pad, pad:-pad]


def compute_kinetic_energy(a, b, rho_f, rho_s, phi, w_t, dx, dy):
    H = smoothed_heaviside(phi, w_t)
    rho = (1 - H) * rho_s + H * rho_f
    return np.sum(0.5 * rho * (a ** 2 + b ** 2)) * dx * dy


def compute_strain_energy(X1, X2, phi, mu_s, dx, dy, kappa=0.0):
    pw = 4
    P1 = np.pad(X1, pw, mode='edge'); P2 = np.pad(X2, pw, mode='edge')
    cut = (slice(pw, -pw), slice(pw, -pw))
    G11 = grad_central_x_2nd(P1, dx)[cut]; G12 = grad_central_y_2nd(P1, dy)[cut]
    G21 = grad_central_x_2nd(P2, dx)[cut]; G22 = grad_central_y_2nd(P2, dy)[cut]
    se = np.zeros_like(phi)
    solid = phi <= 0.0
    if np.any(solid):
        detG = G11 * G22 - G12 * G21
        good = (np.abs(detG) > 1e-10) & solid
        if np.any(good):
            d = detG[good]
            F11 = G22[good] / d; F12 = -G12[good] / d; F21 = -G21[good] / d; F22 = G11[good] / d
            I1 = (F11 ** 2 + F21 ** 2) + (F12 ** 2 + F22 ** 2)
            se[good] = 0.5 * mu_s * (I1 - 2.0) + 0.5 * kappa * (1.0 / d - 1.0) ** 2
    return np.sum(se) * dx * dy


def compute_viscous_dissipation(a, b, mu_f, phi, w_t, dx, dy, eta_s=0.0):
    dudx = grad_central_x_2nd(a, dx); dvdy = grad_central_y_2nd(b, dy)
    Dxy = 0.5 * (grad_central_y_2nd(a, dy) + grad_central_x_2nd(b, dx))
    H = smoothed_heaviside(phi, w_t)
    mu = H * mu_f + (1 - H) * eta_s
    return np.sum(2.0 * mu * (dudx ** 2 + dvdy ** 2 + 2.0 * Dxy ** 2)) * dx * dy


# ── drivers: the per-config loop bodies (the reference's benchmarks/*.py) ─────────
def create_grid(Nx, Ny, Lx, Ly):
    """functions.py:25-31 (np.linspace node grid)."""
    x = np.linspace(0, Lx, Nx); y = np.linspace(0, Ly, Ny)
    X, Y = np.meshgrid(x, y)
    return X, Y, x[1] - x[0], y[1] - y[0]


class SoftDisc:
    """benchmarks/soft_disc_in_lid_driven.py:165-235 (configs 2 and 4) and
    benchmarks/disc_in_taylor_green.py:161-245 (config 3) loop bodies."""

    def __init__(self, N, case="lid", scheme="semilagrangian"):
        self.N = N; self.case = case; self.scheme = scheme
        X, Y, dx, dy = create_grid(N, N, 1.0, 1.0)
        self.X, self.Y, self.dx, self.dy = X, Y, dx, dy
        if case == "lid":
            self.disc = (0.6, 0.5, 0.2)
            self.mu_s, self.kappa, self.rho_s, self.eta_s = 0.1, 0.0, 1.0, 0.01
            self.mu_f, self.rho_f = 0.01, 1.0
            self.bc_kind, self.lid, self.cap = 1, 1.0, 1e-3
        else:  # Taylor-Green box
            self.disc = (0.5, 0.5, 0.2)
            self.mu_s, self.kappa, self.rho_s, self.eta_s = 1.0, 0.0, 1.0, 0.0
            self.mu_f, self.rho_f = 1.0e-3, 1.0
            self.bc_kind, self.lid, self.cap = 2, 0.0, 1e-4
        self.w_t = 2.0 * dx
        self.layers = max(3, int(np.ceil(self.w_t / dx)) + 1)
        phi = self.phi_of(X, Y)
        m = (phi <= 0).astype(float)
        self.X1, self.X2 = extrapolate_reference_map(X * m, Y * m, phi, dx, dy, self.layers)
        if case == "lid":
            self.a = np.zeros((N, N)); self.b = np.zeros((N, N))
        else:
            k = 2.0 * np.pi
            a = 0.05 * k * np.sin(k * X) * np.cos(k * Y)
            b = -0.05 * k * np.cos(k * X) * np.sin(k * Y)
            self.a, self.b = apply_bc(2, 0.0, a, b)
        self.p = np.zeros((N, N))
        self.eig = _precompute_poisson_eigenvalues(N, N, dx, dy)
        self.t = 0.0
        self.integ_diss = 0.0

    def phi_of(self, X1, X2):
        x0, y0, R = self.disc
        return rebuild_phi_disc(X1, X2, x0, y0, R)

    def step(self, t_end=np.inf, energies=False):
        dx, dy = self.dx, self.dy
        dt = compute_timestep(self.a, self.b, dx, dy, 0.2, self.cap, self.mu_s, self.rho_s, 0.0,
                              self.rho_f, mu_f=self.mu_f, eta_s=self.eta_s, kappa=self.kappa)
        if self.t + dt > t_end:
            dt = t_end - self.t
        phi = self.phi_of(self.X1, self.X2)
        m = (phi <= 0).astype(float)
        X1 = advect_reference_map(self.X1, self.a, self.b, self.X, self.Y, dt, dx, dy, phi,
                                  self.scheme) * m
        X2 = advect_reference_map(self.X2, self.a, self.b, self.X, self.Y, dt, dx, dy, phi,
                                  self.scheme) * m
        self.X1, self.X2 = extrapolate_reference_map(X1, X2, phi, dx, dy, self.layers)
        phi = self.phi_of(self.X1, self.X2)
        a_s, b_s, _, _, _, J = momentum_step_rk4(
            self.a, self.b, self.p, self.X1, self.X2, self.bc_kind, self.lid, self.mu_s,
            self.kappa, self.eta_s, dx, dy, dt, self.rho_s, self.rho_f, phi, self.mu_f, self.w_t)
        H = smoothed_heaviside(phi, self.w_t)
        rho = (1 - H) * self.rho_s + H * self.rho_f
        self.a, self.b, self.p = pressure_projection(a_s, b_s, dx, dy, dt, rho, self.bc_kind,
                                                     self.lid, self.p, self.eig)
        self.t += dt
        self.phi = phi
        cx, cy = disc_centroid(phi, self.X, self.Y)
        rec = dict(t=self.t, dt=dt, cx=cx, cy=cy, minJ=J.min(), maxJ=J.max())
        if energies:
            ke = compute_kinetic_energy(self.a, self.b, self.rho_f, self.rho_s, phi, self.w_t, dx, dy)
            se = compute_strain_energy(self.X1, self.X2, phi, self.mu_s, dx, dy, kappa=self.kappa)
            ed = compute_viscous_dissipation(self.a, self.b, self.mu_f, phi, self.w_t, dx, dy,
                                             self.eta_s)
            self.integ_diss += ed * dt
            ys = self.Y[phi <= 0]
            rec.update(ke=ke, se=se, diss=ed, integ=self.integ_diss,
                       E=ke + se + self.integ_diss,
                       ry=0.5 * (ys.max() - ys.min()) if ys.size else np.nan)
        return rec


class LidCavity:
    """benchmarks/lid_driven_cavity.py:26-97 (config 1): pure fluid, phi = 1."""

    def __init__(self, N=129, Re=1000.0):
        self.N = N
        self.X, self.Y, self.dx, self.dy = create_grid(N, N, 1.0, 1.0)
        self.mu_f = 1.0 / Re
        self.phi = np.ones((N, N))
        self.X1, self.X2 = self.X.copy(), self.Y.copy()
        self.a, self.b = apply_bc(1, 1.0, np.zeros((N, N)), np.zeros((N, N)))
        self.p = np.zeros((N, N))
        self.eig = _precompute_poisson_eigenvalues(N, N, self.dx, self.dy)

    def step(self):
        dx, dy = self.dx, self.dy
        dt = compute_timestep(self.a, self.b, dx, dy, 0.2, 1e-2, 0.0, 0.0, 0.0, 1.0, mu_f=self.mu_f)
        a_s, b_s, *_ = momentum_step_rk4(self.a, self.b, self.p, self.X1, self.X2, 1, 1.0, 0.0,
                                         0.0, 0.0, dx, dy, dt, 0.0, 1.0, self.phi, self.mu_f,
                                         2.0 * dx)
        a_prev = self.a
        self.a, self.b, self.p = pressure_projection(a_s, b_s, dx, dy, dt, 1.0, 1, 1.0, self.p,
                                                     self.eig)
        return dt, a_prev

    def ghia_rms(self, y_ref, u_ref):
        i_mid = self.N // 2
        return float(np.sqrt(np.mean((np.interp(y_ref, self.Y[:, i_mid], self.a[:, i_mid])
                                      - u_ref) ** 2)))


__all__ = [k for k in dict(globals()) if not k.startswith("_") or k.startswith("_compute")
           or k.startswith("_solve") or k.startswith("_precompute") or k == "_weno5_rhs"]
_ = math
