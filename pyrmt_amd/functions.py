"""Drop-in operator surface of pyRMT (pyRMT/__init__.py:1-57) on MI355X.

Same names, argument meaning, return values and error behaviour as the reference's
module-level functions; every array operation runs in librmt's HIP kernels on the
current CUDA(=HIP) device.  Arrays may be numpy (copied to / from the device per call,
like a drop-in) or torch CUDA float64 tensors (no copies; results come back as tensors).

Device memory and streams come from torch (plumbing only); the kernels are librmt's.
"""
import ctypes

import numpy as np

from . import _lib as L
from .bc import resolve_bc, resolve_shape, Disc

_ctxs = {}


def _torch():
    import torch
    if not torch.cuda.is_available():
        raise RuntimeError("pyrmt_amd needs a visible MI355X (torch.cuda.is_available() is False)")
    return torch


class _Ctx:
    def __init__(self, ny, nx, device):
        self.ny, self.nx, self.device = ny, nx, device
        h = ctypes.c_void_p()
        L.check(L.lib().rmt_ctx_create(ny, nx, device, None, ctypes.byref(h)), "rmt_ctx_create")
        self.h = h

    def bind(self):
        torch = _torch()
        L.check(L.lib().rmt_ctx_set_stream(self.h, torch.cuda.current_stream().cuda_stream))
        return self.h

    def __del__(self):
        try:
            L.lib().rmt_ctx_destroy(self.h)
        except Exception:
            pass

    def set_option(self, name, value):
        """A per-context implementation switch (include/rmt.h rmt_ctx_set_option)."""
        L.check(L.lib().rmt_ctx_set_option(self.h, name.encode(), int(value)),
                "rmt_ctx_set_option")

    def get_option(self, name):
        v = ctypes.c_int()
        L.check(L.lib().rmt_ctx_get_option(self.h, name.encode(), ctypes.byref(v)),
                "rmt_ctx_get_option")
        return v.value


def ctx_for(ny, nx):
    torch = _torch()
    dev = torch.cuda.current_device()
    key = (int(ny), int(nx), dev)
    if key not in _ctxs:
        _ctxs[key] = _Ctx(int(ny), int(nx), dev)
    return _ctxs[key]


class _IO:
    """Moves inputs to the device and results back to the caller's array type."""

    def __init__(self, *arrays):
        torch = _torch()
        self.torch = torch
        self.host = any(not isinstance(a, torch.Tensor) for a in arrays if a is not None)

    def dev(self, a):
        torch = self.torch
        if a is None:
            return None
        if isinstance(a, torch.Tensor):
            t = a
            if t.dtype != torch.float64 or not t.is_cuda or not t.is_contiguous():
                t = t.to(device="cuda", dtype=torch.float64).contiguous()
            return t
        return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).cuda()

    def empty(self, shape):
        return self.torch.empty(tuple(shape), dtype=self.torch.float64, device="cuda")

    def out(self, t):
        return t.cpu().numpy() if self.host else t


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


# ── grid / setup (host-side, as the reference) ───────────────────────────────────
def create_grid(Nx, Ny, Lx, Ly):
    """functions.py:25-31 (np.linspace node grid; setup, host)."""
    x = np.linspace(0, Lx, Nx)
    y = np.linspace(0, Ly, Ny)
    X, Y = np.meshgrid(x, y)
    return X, Y, x[1] - x[0], y[1] - y[0]


def apply_phi_BCs(phi):
    """functions.py:33-46 (init only, in place on the host array)."""
    phi[0:3, :] = phi[-6:-3, :]
    phi[-3:, :] = phi[3:6, :]
    phi[:, 0:3] = phi[:, -6:-3]
    phi[:, -3:] = phi[:, 3:6]
    return phi


def _precompute_poisson_eigenvalues(Nx, Ny, dx, dy):
    """functions.py:1091-1104 (setup, host).  The device solver recomputes the same
    separable symbol; `eigenvalues` is accepted by the solvers for API parity."""
    lx = -2.0 * (1.0 - np.cos(np.pi * np.arange(Nx) / (Nx - 1))) / dx ** 2
    ly = -2.0 * (1.0 - np.cos(np.pi * np.arange(Ny) / (Ny - 1))) / dy ** 2
    eig = lx[np.newaxis, :] + ly[:, np.newaxis]
    eig[0, 0] = 1.0
    return eig


def _grid_of_eigenvalues(eig):
    """Recover (dx, dy) of a _precompute_poisson_eigenvalues table and check it."""
    eig = np.asarray(eig)
    Ny, Nx = eig.shape
    dx = np.sqrt(-2.0 * (1.0 - np.cos(np.pi / (Nx - 1))) / eig[0, 1])
    dy = np.sqrt(-2.0 * (1.0 - np.cos(np.pi / (Ny - 1))) / eig[1, 0])
    ref = _precompute_poisson_eigenvalues(Nx, Ny, dx, dy)
    if not np.allclose(ref, eig, rtol=1e-12, atol=0):
        raise NotImplementedError("eigenvalues are not the DCT-I Neumann symbol of a uniform grid")
    return float(dx), float(dy)


# ── FD helpers / interpolation (utils.py, interpolators.py) ──────────────────────
def grad_central_x_2nd(f, dx):
    io = _IO(f); f = io.dev(f); out = io.empty(f.shape)
    c = ctx_for(*f.shape)
    L.check(L.lib().rmt_grad_x_2nd(c.bind(), _p(f), dx, _p(out)), "grad_central_x_2nd")
    return io.out(out)


def grad_central_y_2nd(f, dy):
    io = _IO(f); f = io.dev(f); out = io.empty(f.shape)
    c = ctx_for(*f.shape)
    L.check(L.lib().rmt_grad_y_2nd(c.bind(), _p(f), dy, _p(out)), "grad_central_y_2nd")
    return io.out(out)


def diff_upwind_3rd(f, u, h, axis):
    io = _IO(f, u); f = io.dev(f); u = io.dev(u); out = io.empty(f.shape)
    c = ctx_for(*f.shape)
    L.check(L.lib().rmt_diff_upwind_3rd(c.bind(), _p(f), _p(u), h, int(axis), _p(out)),
            "diff_upwind_3rd")
    return io.out(out)


def bilinear_interpolate(u, xq, yq, dx, dy, Nx, Ny):
    io = _IO(u, xq, yq); u = io.dev(u); xq = io.dev(xq); yq = io.dev(yq)
    if u.shape != (Ny, Nx):
        raise ValueError("bilinear_interpolate: u must have shape (Ny, Nx)")
    out = io.empty(xq.shape)
    c = ctx_for(Ny, Nx)
    L.check(L.lib().rmt_bilinear_interpolate(c.bind(), _p(u), _p(xq), _p(yq), xq.numel(), dx, dy,
                                             _p(out)), "bilinear_interpolate")
    return io.out(out)


# ── reference-map transport (functions.py:48-542) ─────────────────────────────────
def extrapolate_reference_map(X1, X2, phi, dx, dy, max_layers):
    io = _IO(X1, X2, phi); X1 = io.dev(X1); X2 = io.dev(X2); phi = io.dev(phi)
    o1 = io.empty(X1.shape); o2 = io.empty(X1.shape)
    c = ctx_for(*X1.shape)
    L.check(L.lib().rmt_extrapolate_reference_map(c.bind(), _p(X1), _p(X2), _p(phi), dx, dy,
                                                  int(max_layers), _p(o1), _p(o2)),
            "extrapolate_reference_map")
    return io.out(o1), io.out(o2)


def extrapolation_mode(mode):
    """librmt diagnostic: 0 chain path (default, sweep on capacity fallback), 1 sweep only,
    2 chain pre-passes then the sweep forced, 3 mode 0 then an abort is reported (error-path
    tests)."""
    L.check(L.lib().rmt_extrap_set_mode(int(mode)), "rmt_extrap_set_mode")


def extrapolation_parallel(on=True):
    """librmt option (no reference counterpart): the parallel extrapolation (extrap_par.hip)
    instead of the exact raster-order chain -- the same targets, acceptance and weights, each
    fit evaluated in offsets from its target (not bit-exact: within the reference's own
    rounding noise).  Process-wide, for the extrapolations that start
    afterwards (a simulation created afterwards also schedules its step for it)."""
    L.check(L.lib().rmt_extrap_set_parallel(int(bool(on))), "rmt_extrap_set_parallel")


def extrapolation_last_path(ny, nx):
    """librmt diagnostic: 0 if the last extrapolation on this grid ran the chain path,
    1 if it ran the row-ticket sweep."""
    p = ctypes.c_int(-1)
    L.check(L.lib().rmt_extrap_last_path(ctx_for(ny, nx).bind(), ctypes.byref(p)),
            "rmt_extrap_last_path")
    return p.value


def advect_semilagrangian_rk4(q, a, b, X, Y, dt, dx, dy):
    io = _IO(q, a, b, X, Y); q, a, b, X, Y = map(io.dev, (q, a, b, X, Y))
    out = io.empty(q.shape)
    c = ctx_for(*q.shape)
    L.check(L.lib().rmt_advect_sl_rk4(c.bind(), _p(q), _p(a), _p(b), _p(X), _p(Y), dt, dx, dy,
                                      _p(out)), "advect_semilagrangian_rk4")
    return io.out(out)


def _weno5_rhs(q, a, b, dx, dy, phi, w_cut):
    io = _IO(q, a, b, phi); q, a, b, phi = map(io.dev, (q, a, b, phi))
    out = io.empty(q.shape)
    c = ctx_for(*q.shape)
    L.check(L.lib().rmt_weno5_rhs(c.bind(), _p(q), _p(a), _p(b), dx, dy, _p(phi), w_cut, _p(out)),
            "_weno5_rhs")
    return io.out(out)


def advect_weno5_rk3(q, a, b, dx, dy, dt, phi, w_cut=0.0):
    io = _IO(q, a, b, phi); q, a, b, phi = map(io.dev, (q, a, b, phi))
    out = io.empty(q.shape)
    c = ctx_for(*q.shape)
    L.check(L.lib().rmt_advect_weno5_rk3(c.bind(), _p(q), _p(a), _p(b), dx, dy, dt, _p(phi), w_cut,
                                         _p(out)), "advect_weno5_rk3")
    return io.out(out)


def bicubic_interpolate(u, xq, yq, dx, dy, Nx, Ny):
    """interpolators.py:64-142 (monotone Catmull-Rom bicubic)."""
    io = _IO(u, xq, yq); u = io.dev(u); xq = io.dev(xq); yq = io.dev(yq)
    if u.shape != (Ny, Nx):
        raise ValueError("bicubic_interpolate: u must have shape (Ny, Nx)")
    out = io.empty(xq.shape)
    c = ctx_for(Ny, Nx)
    L.check(L.lib().rmt_bicubic_interpolate(c.bind(), _p(u), _p(xq), _p(yq), xq.numel(), dx, dy,
                                            _p(out)), "bicubic_interpolate")
    return io.out(out)


def advect_semilagrangian_cubic_rk4(q, a, b, X, Y, dt, dx, dy):
    """functions.py:228-251."""
    io = _IO(q, a, b, X, Y); q, a, b, X, Y = map(io.dev, (q, a, b, X, Y))
    out = io.empty(q.shape)
    c = ctx_for(*q.shape)
    L.check(L.lib().rmt_advect_sl_cubic_rk4(c.bind(), _p(q), _p(a), _p(b), _p(X), _p(Y), dt, dx,
                                            dy, _p(out)), "advect_semilagrangian_cubic_rk4")
    return io.out(out)


def _central_rhs(q, a, b, dx, dy, phi, w_cut, conservative):
    io = _IO(q, a, b, phi); q, a, b, phi = map(io.dev, (q, a, b, phi))
    out = io.empty(q.shape)
    c = ctx_for(*q.shape)
    L.check(L.lib().rmt_central_rhs(c.bind(), _p(q), _p(a), _p(b), dx, dy, _p(phi), w_cut,
                                    int(conservative), _p(out)), "_central_rhs")
    return io.out(out)


def _central2_rhs(q, a, b, dx, dy, phi, w_cut):
    """functions.py:420-444."""
    return _central_rhs(q, a, b, dx, dy, phi, w_cut, False)


def _conservative_rhs(q, a, b, dx, dy, phi, w_cut):
    """functions.py:466-489 (Jain, Kamrin & Mani 2019, eq. 26)."""
    return _central_rhs(q, a, b, dx, dy, phi, w_cut, True)


def _advect_central(q, a, b, dx, dy, dt, phi, w_cut, conservative, name):
    io = _IO(q, a, b, phi); q, a, b, phi = map(io.dev, (q, a, b, phi))
    out = io.empty(q.shape)
    c = ctx_for(*q.shape)
    L.check(L.lib().rmt_advect_central_rk3(c.bind(), _p(q), _p(a), _p(b), dx, dy, dt, _p(phi),
                                           w_cut, int(conservative), _p(out)), name)
    return io.out(out)


def advect_central2_rk3(q, a, b, dx, dy, dt, phi, w_cut=0.0):
    """functions.py:447-463."""
    return _advect_central(q, a, b, dx, dy, dt, phi, w_cut, False, "advect_central2_rk3")


def advect_conservative_rk3(q, a, b, dx, dy, dt, phi, w_cut=0.0):
    """functions.py:492-498."""
    return _advect_central(q, a, b, dx, dy, dt, phi, w_cut, True, "advect_conservative_rk3")


def advect_reference_map(q, a, b, X, Y, dt, dx, dy, phi, scheme='semilagrangian', w_cut=0.0):
    """functions.py:501-542: raises FloatingPointError on non-finite velocity, ValueError
    on an unknown scheme."""
    io = _IO(q, a, b, X, Y, phi)
    ad, bd = io.dev(a), io.dev(b)
    c = ctx_for(*ad.shape)
    fin = ctypes.c_int(0)
    L.check(L.lib().rmt_all_finite2(c.bind(), _p(ad), _p(bd), ctypes.byref(fin)))
    if not fin.value:
        raise FloatingPointError("advect_reference_map: non-finite velocity (the simulation diverged)")
    if scheme == 'semilagrangian':
        return advect_semilagrangian_rk4(q, a, b, X, Y, dt, dx, dy)
    if scheme == 'semilagrangian_cubic':
        return advect_semilagrangian_cubic_rk4(q, a, b, X, Y, dt, dx, dy)
    if scheme == 'central2':
        return advect_central2_rk3(q, a, b, dx, dy, dt, phi, w_cut)
    if scheme == 'weno5':
        return advect_weno5_rk3(q, a, b, dx, dy, dt, phi, w_cut)
    if scheme == 'conservative':
        return advect_conservative_rk3(q, a, b, dx, dy, dt, phi, w_cut)
    raise ValueError("Unknown advection scheme %r (expected 'semilagrangian', "
                     "'central2', 'weno5' or 'conservative')" % (scheme,))


def rebuild_phi_from_reference_map(X1, X2, phi_init_func):
    """functions.py:1366-1367 for a disc level set (the drivers' lambda or bc.Disc)."""
    d = resolve_shape(phi_init_func)
    io = _IO(X1, X2); X1 = io.dev(X1); X2 = io.dev(X2); out = io.empty(X1.shape)
    c = ctx_for(*X1.shape)
    L.check(L.lib().rmt_rebuild_phi_disc(c.bind(), _p(X1), _p(X2), d.x0, d.y0, d.R, _p(out)),
            "rebuild_phi_from_reference_map")
    return io.out(out)


def reinitialize_level_set(phi, dx, dy, method='none', num_iters=20, dt_reinit_factor=0.2,
                           apply_phi_BCs_func=None):
    """functions.py:1436-1456: 'none' is the identity used on the hot path."""
    if method == 'none':
        return phi
    if method in ('pde', 'fmm'):
        raise NotImplementedError(f"reinit method {method!r} is outside this build's path")
    raise ValueError("Unknown reinit method %r (expected 'none', 'pde' or 'fmm')" % (method,))


# ── stress / momentum (functions.py:545-944) ──────────────────────────────────────
def solid_cauchy_stress(X1, X2, dx, dy, mu_s, kappa, phi, w_cut=0.0, detg_clamp=0.0,
                        isochoric=False):
    io = _IO(X1, X2, phi); X1, X2, phi = map(io.dev, (X1, X2, phi))
    outs = [io.empty(X1.shape) for _ in range(4)]
    c = ctx_for(*X1.shape)
    L.check(L.lib().rmt_solid_cauchy_stress(c.bind(), _p(X1), _p(X2), dx, dy, mu_s, kappa, _p(phi),
                                            w_cut, detg_clamp, int(bool(isochoric)),
                                            *map(_p, outs)), "solid_cauchy_stress")
    return tuple(io.out(o) for o in outs)


def smoothed_heaviside(x, w_t):
    io = _IO(x); xd = io.dev(x); out = io.empty(xd.shape)
    c = ctx_for(*(xd.shape if xd.dim() == 2 else (1, xd.numel())))
    L.check(L.lib().rmt_smoothed_heaviside(c.bind(), _p(xd), xd.numel(), w_t, _p(out)),
            "smoothed_heaviside")
    return io.out(out)


def apply_velocity_BCs(bc, u, v):
    """functions.py:946-947: applies the BC to copies."""
    kind, lid = resolve_bc(bc)
    io = _IO(u, v); ud = io.dev(u).clone(); vd = io.dev(v).clone()
    c = ctx_for(*ud.shape)
    L.check(L.lib().rmt_apply_velocity_bc(c.bind(), kind, lid, _p(ud), _p(vd)), "apply_velocity_BCs")
    return io.out(ud), io.out(vd)


def momentum_step_rk4(u, v, p, X1, X2, velocity_bc, mu_s, kappa, eta_s, dx, dy, dt, rho_s, rho_f,
                      phi, mu_f, w_t, gamma=0.0, stress_band=False, detg_clamp=3.0):
    """functions.py:673-762.  Returns (u_new, v_new, sxx, sxy, syy, J)."""
    if gamma > 1e-12:
        raise NotImplementedError("surface tension (gamma > 0) is outside this build's path")
    kind, lid = resolve_bc(velocity_bc)
    io = _IO(u, v, p, X1, X2, phi)
    u, v, p, X1, X2, phi = map(io.dev, (u, v, p, X1, X2, phi))
    outs = [io.empty(u.shape) for _ in range(6)]
    prm = L.rmt_momentum_params(kind, lid, mu_s, kappa, eta_s, rho_s, rho_f, mu_f, w_t, dx, dy, dt,
                                int(bool(stress_band)), detg_clamp)
    c = ctx_for(*u.shape)
    L.check(L.lib().rmt_momentum_step_rk4(c.bind(), ctypes.byref(prm), _p(u), _p(v), _p(p), _p(X1),
                                          _p(X2), _p(phi), *map(_p, outs)), "momentum_step_rk4")
    return tuple(io.out(o) for o in outs)


def momentum_mode(mode):
    """librmt diagnostic: 0 one kernel per RK4 stage (default), 2 unfused per-cell passes
    (bit-identical); any other mode raises."""
    L.check(L.lib().rmt_momentum_set_mode(int(mode)), "rmt_momentum_set_mode")


def velocity_rhs_blended_optimized(u, v, p, sigma_sxx_s_elastic, sigma_sxy_s_elastic,
                                   sigma_syy_s_elastic, dx, dy, phi, mu_f, H, dH_dx, dH_dy,
                                   rho_local, st_force_x, st_force_y):
    """functions.py:897-944: blended-stress divergence + 3rd-order upwind advection - grad p,
    over (rho_local + 1e-12).  H, rho_local and the surface-tension force may be arrays or
    scalars (broadcast as NumPy would); phi, dH_dx, dH_dy are unused, as in the reference."""
    shape = np.shape(u) if not hasattr(u, "shape") else tuple(u.shape)
    torch = _torch()

    def full(a):
        if isinstance(a, torch.Tensor):
            return a.expand(shape) if a.dim() < 2 else a
        return np.array(np.broadcast_to(np.asarray(a, dtype=np.float64), shape))   # writable copy

    zero_f = all(np.ndim(f) == 0 and float(f) == 0.0 and not isinstance(f, torch.Tensor)
                 for f in (st_force_x, st_force_y))
    arrays = (u, v, p, sigma_sxx_s_elastic, sigma_sxy_s_elastic, sigma_syy_s_elastic,
              full(H), full(rho_local))
    io = _IO(*arrays)
    d = [io.dev(a) for a in arrays]
    fx = fy = None
    if not zero_f:   # a non-zero scalar force, or arrays
        fx = io.dev(full(st_force_x)); fy = io.dev(full(st_force_y))
    ru = io.empty(shape); rv = io.empty(shape)
    c = ctx_for(*shape)
    L.check(L.lib().rmt_velocity_rhs_blended(c.bind(), *map(_p, d[:6]), dx, dy, mu_f, _p(d[6]),
                                             _p(d[7]), _p(fx), _p(fy), _p(ru), _p(rv)),
            "velocity_rhs_blended_optimized")
    return io.out(ru), io.out(rv)


# ── diagnostics (output.py:6-193) ─────────────────────────────────────────────────
def compute_kinetic_energy(a, b, rho_f, rho_s, phi, w_t, dx, dy):
    """output.py:6-39: sum(0.5 rho (a^2 + b^2)) dx dy with rho = (1-H) rho_s + H rho_f."""
    io = _IO(a, b, phi); a, b, phi = map(io.dev, (a, b, phi))
    out = ctypes.c_double()
    c = ctx_for(*a.shape)
    L.check(L.lib().rmt_compute_kinetic_energy(c.bind(), _p(a), _p(b), rho_f, rho_s, _p(phi), w_t,
                                               dx, dy, ctypes.byref(out)), "compute_kinetic_energy")
    return out.value


def compute_strain_energy(X1, X2, phi, mu_s, dx, dy, kappa=0.0):
    """output.py:41-134: (mu_s/2)(I1 - 2) + (kappa/2)(J - 1)^2 over the solid cells."""
    io = _IO(X1, X2, phi); X1, X2, phi = map(io.dev, (X1, X2, phi))
    out = ctypes.c_double()
    c = ctx_for(*X1.shape)
    L.check(L.lib().rmt_compute_strain_energy(c.bind(), _p(X1), _p(X2), _p(phi), mu_s, dx, dy,
                                              kappa, ctypes.byref(out)), "compute_strain_energy")
    return out.value


def compute_viscous_dissipation(a, b, mu_f, phi, w_t, dx, dy, eta_s=0.0):
    """output.py:136-193: sum(2 mu (D_xx^2 + D_yy^2 + 2 D_xy^2)) dx dy."""
    io = _IO(a, b, phi); a, b, phi = map(io.dev, (a, b, phi))
    out = ctypes.c_double()
    c = ctx_for(*a.shape)
    L.check(L.lib().rmt_compute_viscous_dissipation(c.bind(), _p(a), _p(b), mu_f, _p(phi), w_t,
                                                    dx, dy, eta_s, ctypes.byref(out)),
            "compute_viscous_dissipation")
    return out.value


def divergence_2d_interior(u, v, dx, dy, pad=3):
    """output.py:195-211: (divU, its interior [pad:-pad, pad:-pad]); central differences on
    the device, 0 within pad cells of every edge."""
    io = _IO(u, v); u, v = io.dev(u), io.dev(v)
    out = io.empty(u.shape)
    c = ctx_for(*u.shape)
    L.check(L.lib().rmt_divergence_2d_interior(c.bind(), _p(u), _p(v), dx, dy, int(pad), _p(out)),
            "divergence_2d_interior")
    d = io.out(out)
    return d, d[pad:-pad, pad:-pad]


# ── projection (functions.py:1005-1364) ──────────────────────────────────────────
def _rho_scalar(rho):
    """The constant-density branch (functions.py:1298): rho scalar, or an array whose
    ptp <= 1e-10 and that is exactly constant (as (1-H) rho_s + H rho_f is for
    rho_s == rho_f == 1).  Variable density -> NotImplementedError."""
    if np.isscalar(rho) or (hasattr(rho, "ndim") and rho.ndim == 0):
        return float(rho)
    r = rho.detach().cpu().numpy() if hasattr(rho, "detach") else np.asarray(rho)
    if np.ptp(r) > 1e-10:
        raise NotImplementedError("variable-density projection (CG) is outside this build's path")
    r0 = float(r.flat[0])
    if not np.all(r == r0):
        raise NotImplementedError("rho must be exactly constant on the device path")
    return r0


def _is_variable_rho(rho):
    """functions.py:1026 / :1297: a 2D array whose ptp exceeds 1e-10."""
    if np.isscalar(rho) or not hasattr(rho, "ndim") or rho.ndim != 2:
        return False
    r = rho.detach().cpu().numpy() if hasattr(rho, "detach") else np.asarray(rho)
    return bool(np.ptp(r) > 1e-10)


def _compute_divergence_rc(a_star, b_star, p_prev, dt, rho, dx, dy):
    if _is_variable_rho(rho):
        io = _IO(a_star, b_star, p_prev, rho)
        a, b, p, r = map(io.dev, (a_star, b_star, p_prev, rho))
        out = io.empty(a.shape)
        c = ctx_for(*a.shape)
        L.check(L.lib().rmt_divergence_rc_variable(c.bind(), _p(a), _p(b), _p(p), dt, _p(r), dx,
                                                   dy, _p(out)), "_compute_divergence_rc")
        return io.out(out)
    r = _rho_scalar(rho)
    io = _IO(a_star, b_star, p_prev); a, b, p = map(io.dev, (a_star, b_star, p_prev))
    out = io.empty(a.shape)
    c = ctx_for(*a.shape)
    L.check(L.lib().rmt_divergence_rc(c.bind(), _p(a), _p(b), _p(p), dt / r, dx, dy, _p(out)),
            "_compute_divergence_rc")
    return io.out(out)


def _apply_variable_poisson(p_flat, Nx, Ny, dx, dy, inv_rho):
    """functions.py:1122-1168 (matrix-free div((1/rho) grad p)); flat in, flat out."""
    io = _IO(p_flat, inv_rho)
    p = io.dev(p_flat).reshape(Ny, Nx).contiguous()
    ir = io.dev(inv_rho).reshape(Ny, Nx).contiguous()
    out = io.empty((Ny, Nx))
    c = ctx_for(Ny, Nx)
    L.check(L.lib().rmt_apply_variable_poisson(c.bind(), _p(p), dx, dy, _p(ir), _p(out)),
            "_apply_variable_poisson")
    return io.out(out).reshape(-1)


def _compute_divergence(a_star, b_star, dx, dy):
    io = _IO(a_star, b_star); a, b = io.dev(a_star), io.dev(b_star)
    out = io.empty(a.shape)
    c = ctx_for(*a.shape)
    L.check(L.lib().rmt_divergence_central(c.bind(), _p(a), _p(b), dx, dy, _p(out)),
            "_compute_divergence")
    return io.out(out)


def _compute_pressure_gradient(p, dx, dy):
    io = _IO(p); pd = io.dev(p); gx = io.empty(pd.shape); gy = io.empty(pd.shape)
    c = ctx_for(*pd.shape)
    L.check(L.lib().rmt_pressure_gradient(c.bind(), _p(pd), dx, dy, _p(gx), _p(gy)),
            "_compute_pressure_gradient")
    return io.out(gx), io.out(gy)


def _solve_poisson_dct(rhs_2d, eigenvalues):
    dx, dy = _grid_of_eigenvalues(eigenvalues)
    io = _IO(rhs_2d); r = io.dev(rhs_2d); out = io.empty(r.shape)
    c = ctx_for(*r.shape)
    L.check(L.lib().rmt_solve_poisson_dct(c.bind(), _p(r), dx, dy, _p(out)), "_solve_poisson_dct")
    return io.out(out)


# ── periodic branch (functions.py:1171-1252, 1277-1290) ────────────────────────────
def _periodic_axis(n, h):
    m = n - 1
    return -(np.sin(2.0 * np.pi * np.arange(m) / m) / h) ** 2


def _precompute_poisson_eigenvalues_periodic(Nx, Ny, dx, dy):
    """functions.py:1177-1202 (setup, host): (eig, null) on the reduced grid."""
    eig = _periodic_axis(Nx, dx)[np.newaxis, :] + _periodic_axis(Ny, dy)[:, np.newaxis]
    null = np.abs(eig) < 1e-12
    eig = eig.copy()
    eig[null] = 1.0
    return eig, null


def _periodic_axes_of(eigenvalues_periodic, dx=None, dy=None):
    """Per-axis symbols behind an (eig, null) pair: recomputed from the grid spacing (given,
    or recovered from eig[0, 1] / eig[1, 0] and nudged by ulps) and checked bit for bit."""
    eig, null = (np.asarray(a) for a in eigenvalues_periodic)
    my, mx = eig.shape

    def cands(n, e):
        h = float(np.sin(2.0 * np.pi / n) / np.sqrt(-e))
        return [h] + [np.nextafter(h, np.inf), np.nextafter(h, -np.inf),
                      np.nextafter(np.nextafter(h, np.inf), np.inf),
                      np.nextafter(np.nextafter(h, -np.inf), -np.inf)]

    hxs = [dx] if dx is not None else cands(mx, eig[0, 1])
    hys = [dy] if dy is not None else cands(my, eig[1, 0])
    for hx in hxs:
        for hy in hys:
            e2, n2 = _precompute_poisson_eigenvalues_periodic(mx + 1, my + 1, hx, hy)
            if np.array_equal(e2, eig) and np.array_equal(n2, null):
                return (np.ascontiguousarray(_periodic_axis(mx + 1, hx)),
                        np.ascontiguousarray(_periodic_axis(my + 1, hy)))
    raise NotImplementedError("eigenvalues are not the periodic symbol of a uniform grid")


def _tile_overlap(field_reduced, Ny, Nx):
    """functions.py:1205-1213 (host helper)."""
    out = np.empty((Ny, Nx))
    out[:-1, :-1] = field_reduced
    out[-1, :-1] = field_reduced[0, :]
    out[:-1, -1] = field_reduced[:, 0]
    out[-1, -1] = field_reduced[0, 0]
    return out


def _solve_poisson_fft(rhs_full, eigenvalues_periodic):
    """functions.py:1216-1233: reduced-grid 2D FFT solve, null modes zeroed."""
    lx, ly = _periodic_axes_of(eigenvalues_periodic)
    io = _IO(rhs_full); r = io.dev(rhs_full); out = io.empty(r.shape)
    c = ctx_for(*r.shape)
    L.check(L.lib().rmt_solve_poisson_fft(c.bind(), _p(r), lx.ctypes.data_as(ctypes.c_void_p),
                                          ly.ctypes.data_as(ctypes.c_void_p), _p(out)),
            "_solve_poisson_fft")
    return io.out(out)


def _compute_divergence_periodic(a_star, b_star, dx, dy):
    """functions.py:1236-1243."""
    io = _IO(a_star, b_star); a = io.dev(a_star); b = io.dev(b_star); out = io.empty(a.shape)
    c = ctx_for(*a.shape)
    L.check(L.lib().rmt_divergence_periodic(c.bind(), _p(a), _p(b), dx, dy, _p(out)),
            "_compute_divergence_periodic")
    return io.out(out)


def _compute_pressure_gradient_periodic(p, dx, dy):
    """functions.py:1246-1252."""
    io = _IO(p); pd = io.dev(p); gx = io.empty(pd.shape); gy = io.empty(pd.shape)
    c = ctx_for(*pd.shape)
    L.check(L.lib().rmt_pressure_gradient_periodic(c.bind(), _p(pd), dx, dy, _p(gx), _p(gy)),
            "_compute_pressure_gradient_periodic")
    return io.out(gx), io.out(gy)


def _projection_periodic(a_star, b_star, dx, dy, dt, rho, velocity_bc, A, ml, p_prev,
                         eigenvalues):
    """functions.py:1277-1290."""
    Ny, Nx = np.shape(a_star)
    if eigenvalues is None:
        eigenvalues = _precompute_poisson_eigenvalues_periodic(Nx, Ny, dx, dy)
    lx, ly = _periodic_axes_of(eigenvalues, dx, dy)
    kind, lid = resolve_bc(velocity_bc)
    torch = _torch()
    io = _IO(a_star, b_star, p_prev)
    a_s, b_s, pp = map(io.dev, (a_star, b_star, p_prev))
    if isinstance(rho, np.ndarray) or isinstance(rho, torch.Tensor):
        rho_bar = float(np.mean(np.asarray(rho.cpu() if isinstance(rho, torch.Tensor) else rho)))
        rc = io.dev(rho)
    else:
        rho_bar, rc = float(rho), None
    a = io.empty(a_s.shape); b = io.empty(a_s.shape); p = io.empty(a_s.shape)
    c = ctx_for(*a_s.shape)
    L.check(L.lib().rmt_pressure_projection_periodic(
        c.bind(), _p(a_s), _p(b_s), dx, dy, dt, rho_bar, _p(rc), kind, lid,
        lx.ctypes.data_as(ctypes.c_void_p), ly.ctypes.data_as(ctypes.c_void_p), _p(pp), _p(a),
        _p(b), _p(p)), "pressure_projection_amg(periodic)")
    return io.out(a), io.out(b), io.out(p), A, ml


def pressure_projection_amg(a_star, b_star, dx, dy, dt, rho, velocity_bc, A=None, ml=None,
                            p_prev=None, eigenvalues=None, bc_type='neumann'):
    """functions.py:1255-1364: the Neumann branch (DCT direct solve, constant density) and
    the periodic branch (reduced-grid FFT).  Returns (a, b, p, A, ml) like the reference."""
    if bc_type == 'periodic':
        return _projection_periodic(a_star, b_star, dx, dy, dt, rho, velocity_bc, A, ml,
                                    p_prev, eigenvalues)
    if bc_type != 'neumann':
        raise NotImplementedError("bc_type %r is outside this build's path" % (bc_type,))
    if eigenvalues is None:
        raise NotImplementedError("the AMG fallback (eigenvalues=None) is outside this build's path")
    _grid_of_eigenvalues(eigenvalues)
    kind, lid = resolve_bc(velocity_bc)
    if _is_variable_rho(rho):
        return _projection_variable(a_star, b_star, dx, dy, dt, rho, kind, lid, A, ml, p_prev)
    r = _rho_scalar(rho)
    io = _IO(a_star, b_star, p_prev)
    a_s, b_s, pp = map(io.dev, (a_star, b_star, p_prev))
    a = io.empty(a_s.shape); b = io.empty(a_s.shape); p = io.empty(a_s.shape)
    c = ctx_for(*a_s.shape)
    L.check(L.lib().rmt_pressure_projection(c.bind(), _p(a_s), _p(b_s), dx, dy, dt, r, kind, lid,
                                            _p(pp), _p(a), _p(b), _p(p)), "pressure_projection_amg")
    return io.out(a), io.out(b), io.out(p), A, ml


# the reference's scipy.sparse.linalg.cg call (functions.py:1323): tol=1e-6, maxiter=200
CG_RTOL, CG_MAXITER = 1e-6, 200
last_cg_iterations = None


def _projection_variable(a_star, b_star, dx, dy, dt, rho, kind, lid, A, ml, p_prev):
    """functions.py:1296-1328 + :1350-1364 (variable density, DCT-preconditioned CG)."""
    global last_cg_iterations
    io = _IO(a_star, b_star, p_prev, rho)
    a_s, b_s, pp, r = map(io.dev, (a_star, b_star, p_prev, rho))
    a = io.empty(a_s.shape); b = io.empty(a_s.shape); p = io.empty(a_s.shape)
    c = ctx_for(*a_s.shape)
    it = ctypes.c_int()
    L.check(L.lib().rmt_pressure_projection_variable(
        c.bind(), _p(a_s), _p(b_s), dx, dy, dt, _p(r), kind, lid, _p(pp), CG_RTOL, CG_MAXITER,
        _p(a), _p(b), _p(p), ctypes.byref(it)), "pressure_projection_amg")
    last_cg_iterations = it.value
    return io.out(a), io.out(b), io.out(p), A, ml


def compute_timestep(a, b, dx, dy, CFL, dt_min_cap, mu_s, rho_s, gamma, rho_f, mu_f=0.0,
                     eta_s=0.0, kappa=0.0):
    """functions.py:165-192 (max |u| reduced on the device)."""
    io = _IO(a, b); ad, bd = io.dev(a), io.dev(b)
    c = ctx_for(*ad.shape)
    out = ctypes.c_double()
    L.check(L.lib().rmt_compute_timestep(c.bind(), _p(ad), _p(bd), dx, dy, CFL, dt_min_cap, mu_s,
                                         rho_s, gamma, rho_f, mu_f, eta_s, kappa,
                                         ctypes.byref(out)), "compute_timestep")
    return out.value


# Deprecated aliases (functions.py:1462-1466)
velocity_RK4 = momentum_step_rk4
heaviside_smooth_alt = smoothed_heaviside
compute_solid_stress = solid_cauchy_stress
extrapolate_transverse_layers_2field = extrapolate_reference_map
advect_semi_lagrangian_rk4 = advect_semilagrangian_rk4
__all__ = [k for k in dir() if not k.startswith("__")]
_ = Disc
