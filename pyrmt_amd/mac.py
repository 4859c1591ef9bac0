"""Staggered (MAC) operators of pyRMT/mac.py and the config-5 loop body on MI355X.

Same names, arguments and return values as the reference module (mac.py:22-139,
196-232, 729-749); the arrays go through librmt's HIP kernels (include/rmt.h, rmt_mac_*).
Layout as the reference: p / phi (Ny, Nx) cell centres, u (Ny, Nx+1) x-faces,
v (Ny+1, Nx) y-faces (square grids: Nx == Ny).  ``MacMultiDisc`` is the device-resident
loop body of benchmarks/mac_multi_disc_lid.py:36-98 (K soft discs with pair contact).
"""
import ctypes
import math

import numpy as np

from . import _lib as L
from .functions import _IO, _p, ctx_for, extrapolate_reference_map
from .simulation import _wrap_device


def mac_grid(Nx, Ny, Lx=1.0, Ly=1.0):
    """mac.py:22-23."""
    return Lx / Nx, Ly / Ny


def poisson_eigs_neumann(Nx, Ny, dx, dy):
    """mac.py:104-115 (setup, host): DCT-II symbol, (0,0) pinned to 1."""
    lx = -2.0 * (1.0 - np.cos(np.pi * np.arange(Nx) / Nx)) / dx ** 2
    ly = -2.0 * (1.0 - np.cos(np.pi * np.arange(Ny) / Ny)) / dy ** 2
    eig = (lx[np.newaxis, :] + ly[:, np.newaxis]).copy()
    eig[0, 0] = 1.0
    return eig


def _axis_eigs(eig):
    """Per-axis eigenvalues of a separable eig table (row 0 and column 0; the reference's
    lam[0] is -0.0, so eig[0, k] == lam_x[k] exactly).  Raises if eig is not separable."""
    eig = np.asarray(eig, dtype=np.float64)
    lx = eig[0, :].copy(); ly = eig[:, 0].copy()
    lx[0] = ly[0] = -0.0
    chk = lx[np.newaxis, :] + ly[:, np.newaxis]
    chk[0, 0] = eig[0, 0]
    if not np.array_equal(chk, eig):
        raise NotImplementedError("eig is not a separable per-axis symbol (DCT-II solve)")
    return np.ascontiguousarray(lx), np.ascontiguousarray(ly)


def _ctx(N):
    return ctx_for(N, N).bind()


def divergence(u, v, dx, dy):
    """mac.py:81-84."""
    io = _IO(u, v); u = io.dev(u); v = io.dev(v)
    N = u.shape[0]
    out = io.empty((N, N))
    L.check(L.lib().rmt_mac_divergence(_ctx(N), _p(u), _p(v), dx, dy, _p(out)), "divergence")
    return io.out(out)


def _gradients(p, dx, dy):
    io = _IO(p); p = io.dev(p)
    N = p.shape[0]
    gu = io.empty((N, N + 1)); gv = io.empty((N + 1, N))
    L.check(L.lib().rmt_mac_gradient_p(_ctx(N), _p(p), dx, dy, _p(gu), _p(gv)), "gradient_p")
    return io, gu, gv


def gradient_p_u(p, dx):
    """mac.py:87-93."""
    io, gu, _ = _gradients(p, dx, dx)
    return io.out(gu)


def gradient_p_v(p, dy):
    """mac.py:96-101."""
    io, _, gv = _gradients(p, dy, dy)
    return io.out(gv)


def solve_poisson_neumann(rhs, eig):
    """mac.py:118-123 (orthonormal DCT-II both ways, constant mode zeroed)."""
    lx, ly = _axis_eigs(eig)
    io = _IO(rhs); r = io.dev(rhs)
    N = r.shape[0]
    out = io.empty((N, N))
    L.check(L.lib().rmt_mac_solve_poisson_neumann(
        _ctx(N), _p(r), 1.0 / N, 1.0 / N, lx.ctypes.data_as(ctypes.c_void_p),
        ly.ctypes.data_as(ctypes.c_void_p), _p(out)), "solve_poisson_neumann")
    return io.out(out)


def project(u_star, v_star, dx, dy, dt, rho, eig):
    """mac.py:126-139: returns (u, v, phi)."""
    lx, ly = _axis_eigs(eig)
    io = _IO(u_star, v_star); us = io.dev(u_star); vs = io.dev(v_star)
    N = us.shape[0]
    u = io.empty(us.shape); v = io.empty(vs.shape); phi = io.empty((N, N))
    L.check(L.lib().rmt_mac_project(_ctx(N), _p(us), _p(vs), dx, dy, dt, float(rho),
                                    lx.ctypes.data_as(ctypes.c_void_p),
                                    ly.ctypes.data_as(ctypes.c_void_p), _p(u), _p(v), _p(phi)),
            "project")
    return io.out(u), io.out(v), io.out(phi)


def momentum_predictor(u, v, nu, dx, dy, dt, U_lid, fu=None, fv=None, rho=1.0):
    """mac.py:196-232."""
    if (fu is None) != (fv is None):
        raise NotImplementedError("momentum_predictor: give both face forces or neither")
    io = _IO(u, v); ud = io.dev(u); vd = io.dev(v)
    fud, fvd = io.dev(fu), io.dev(fv)
    us = io.empty(ud.shape); vs = io.empty(vd.shape)
    L.check(L.lib().rmt_mac_momentum_predictor(_ctx(ud.shape[0]), _p(ud), _p(vd), nu, dx, dy,
                                               dt, U_lid, _p(fud), _p(fvd), float(rho), _p(us),
                                               _p(vs)), "momentum_predictor")
    return io.out(us), io.out(vs)


# ------------------------------------------------------------------ IMEX tier --------
# mac.py:243-442 through imex.hip: the homogeneous ghost-cell Laplacians,
# CG / DST-preconditioned CG Helmholtz solves and the IMEX lid-cavity predictor.
def _lap_hom(kind, f, dx, dy):
    io = _IO(f); fd = io.dev(f)
    N = fd.shape[0] if kind == 0 else fd.shape[1]
    out = io.empty((N, N - 1) if kind == 0 else (N - 1, N))
    L.check(L.lib().rmt_mac_lap_lid_hom(_ctx(N), kind, _p(fd), float(dx), float(dy), _p(out)),
            "_lap_lid_hom")
    return io.out(out)


def _lap_u_lid_hom(u, dx, dy):
    """mac.py:243-250: Laplacian of u (Ny, Nx+1) on the interior faces (Ny, Nx-1)."""
    return _lap_hom(0, u, dx, dy)


def _lap_v_lid_hom(v, dx, dy):
    """mac.py:253-260: Laplacian of v (Ny+1, Nx) on the interior faces (Ny-1, Nx)."""
    return _lap_hom(1, v, dx, dy)


def _dst_helmholtz_eigs(shp, dx, dy):
    """mac.py:278-284 (setup, host): DST-II eigenvalues of the Dirichlet Laplacian."""
    Ny, Nx = shp
    lx = -2.0 * (1.0 - np.cos(np.pi * (np.arange(Nx) + 1) / Nx)) / dx ** 2
    ly = -2.0 * (1.0 - np.cos(np.pi * (np.arange(Ny) + 1) / Ny)) / dy ** 2
    return ly[:, None] + lx[None, :]


def _helmholtz_operator(apply_lap_hom, embed, shp):
    """The reference hands the operator over as callables (mac.py:351, 366 and its tests:
    ``lambda w: _lap_u_lid_hom(w, dx, dy)``, ``np.pad`` embeddings).  Identify the face kind
    and (dx, dy) from the lambda's closure and verify both on a probe (the embedding pads
    the kind's wall axis with zeros, the operator equals this module's kernel bit for bit);
    anything else raises NotImplementedError -- there is no host fallback."""
    code = getattr(apply_lap_hom, "__code__", None)
    names = code.co_names if code is not None else ()
    kind = 0 if "_lap_u_lid_hom" in names else 1 if "_lap_v_lid_hom" in names else None
    cells = {}
    if code is not None and apply_lap_hom.__closure__:
        cells = {k: c.cell_contents for k, c in zip(code.co_freevars, apply_lap_hom.__closure__)}
    dx, dy = cells.get("dx"), cells.get("dy")
    Ny, Nx = shp
    if kind is None or dx is None or dy is None or (kind == 0 and Nx != Ny - 1) or \
            (kind == 1 and Ny != Nx - 1):
        raise NotImplementedError("helmholtz: apply_lap_hom must be the reference's "
                                  "lambda w: _lap_u_lid_hom / _lap_v_lid_hom(w, dx, dy)")
    probe = np.random.default_rng(0).standard_normal(shp)
    e = np.asarray(embed(probe), dtype=np.float64)
    pad = np.pad(probe, ((0, 0), (1, 1)) if kind == 0 else ((1, 1), (0, 0)))
    if not np.array_equal(e, pad):
        raise NotImplementedError("helmholtz: embed must zero-pad the walls as mac.py:350/365")
    host = np.asarray(apply_lap_hom(e), dtype=np.float64)
    if not np.array_equal(host, _lap_hom(kind, e, dx, dy)):
        raise NotImplementedError("helmholtz: apply_lap_hom is not the homogeneous lid Laplacian")
    return kind, float(dx), float(dy)


def _solve_helmholtz(rhs_int, kind, coef, dx, dy, rtol, maxiter, precond):
    io = _IO(rhs_int); b = io.dev(rhs_int)
    N = b.shape[0] if kind == 0 else b.shape[1]
    x = io.empty(b.shape)
    it = ctypes.c_int(0)
    L.check(L.lib().rmt_mac_helmholtz(_ctx(N), kind, _p(b), float(coef), dx, dy, float(rtol),
                                      int(maxiter), int(precond), _p(x), ctypes.byref(it)),
            "helmholtz")
    return io.out(x), it.value


def _cg_helmholtz(rhs_int, apply_lap_hom, embed, coef, rtol=1e-10, maxiter=500):
    """mac.py:263-275: (I - coef Lap_hom) x = rhs_int by CG (x0 = rhs_int)."""
    kind, dx, dy = _helmholtz_operator(apply_lap_hom, embed, tuple(rhs_int.shape))
    return _solve_helmholtz(rhs_int, kind, coef, dx, dy, rtol, maxiter, 0)[0]


def _pcg_helmholtz(rhs_int, apply_lap_hom, embed, coef, dx, dy, rtol=1e-8, maxiter=500,
                   count=None):
    """mac.py:287-316: DST-II-preconditioned CG; appends the iteration count to `count`."""
    kind, ldx, ldy = _helmholtz_operator(apply_lap_hom, embed, tuple(rhs_int.shape))
    if (ldx, ldy) != (float(dx), float(dy)):
        raise NotImplementedError("_pcg_helmholtz: the preconditioner's (dx, dy) differ from "
                                  "the operator's")
    x, it = _solve_helmholtz(rhs_int, kind, coef, ldx, ldy, rtol, maxiter, 1)
    if count is not None:
        count.append(it)
    return x


def momentum_predictor_lid_imex(u, v, nu, dx, dy, dt, U_lid, fu=None, fv=None, rho=1.0,
                                rtol=1e-8, cs2=0.0):
    """mac.py:319-369: explicit central advection + face forces, implicit (backward-Euler)
    viscosity (+ the trapezoidal elastic term, cs2 > 0) by DST-preconditioned CG."""
    io = _IO(u, v); ud = io.dev(u); vd = io.dev(v)
    fud, fvd = io.dev(fu), io.dev(fv)
    us = io.empty(ud.shape); vs = io.empty(vd.shape)
    it = (ctypes.c_int * 2)()
    L.check(L.lib().rmt_mac_momentum_predictor_lid_imex(
        _ctx(ud.shape[0]), _p(ud), _p(vd), float(nu), float(dx), float(dy), float(dt),
        float(U_lid), _p(fud), _p(fvd), float(rho), float(rtol), float(cs2), _p(us), _p(vs),
        ctypes.cast(it, ctypes.c_void_p)), "momentum_predictor_lid_imex")
    return io.out(us), io.out(vs)


def momentum_predictor_lid_semilag(u, v, nu, dx, dy, dt, U_lid, fu=None, fv=None, rho=1.0,
                                   cs2=0.0, rtol=1e-8, cfl_switch=0.9):
    """mac.py:381-442: adaptive predictor -- momentum_predictor_lid_imex at an advective
    CFL <= cfl_switch (mac.py:387-390), else the semi-Lagrangian midpoint backtrace through
    cubic-spline interpolation (map_coordinates order 3, 'nearest') and the same PCG
    viscosity solve."""
    io = _IO(u, v); ud = io.dev(u); vd = io.dev(v)
    cfl = dt * max(float(ud.abs().max()) / dx, float(vd.abs().max()) / dy)
    if cfl <= cfl_switch:
        return momentum_predictor_lid_imex(u, v, nu, dx, dy, dt, U_lid, fu=fu, fv=fv, rho=rho,
                                           rtol=rtol, cs2=cs2)
    fud, fvd = io.dev(fu), io.dev(fv)
    us = io.empty(ud.shape); vs = io.empty(vd.shape)
    it = (ctypes.c_int * 2)()
    L.check(L.lib().rmt_mac_momentum_predictor_lid_semilag(
        _ctx(ud.shape[0]), _p(ud), _p(vd), float(nu), float(dx), float(dy), float(dt),
        float(U_lid), _p(fud), _p(fvd), float(rho), float(cs2), float(rtol), _p(us), _p(vs),
        ctypes.cast(it, ctypes.c_void_p)), "momentum_predictor_lid_semilag")
    return io.out(us), io.out(vs)


def contact_stress(phi_a, phi_b, eta, Gsum, eps, dx, dy):
    """mac.py:729-749: (txx, txy, tyy)."""
    io = _IO(phi_a, phi_b); a = io.dev(phi_a); b = io.dev(phi_b)
    out = [io.empty(a.shape) for _ in range(3)]
    L.check(L.lib().rmt_mac_contact_stress(_ctx(a.shape[0]), _p(a), _p(b), eta, Gsum, eps, dx,
                                           dy, *map(_p, out)), "contact_stress")
    return tuple(io.out(t) for t in out)


# ------------------------------------------------------------------ config 5 loop --
def place_discs(n, seed, Rrange=(0.07, 0.12), box=(0.18, 0.82)):
    """mac_multi_disc_lid.py:22-33 (setup, host): non-overlapping random discs (R, cx, cy)."""
    rng = np.random.default_rng(seed)
    discs = []
    for _ in range(2000):
        if len(discs) == n:
            break
        R = rng.uniform(*Rrange)
        cx = rng.uniform(box[0] + R, box[1] - R); cy = rng.uniform(box[0] + R, box[1] - R)
        if all((cx - d[1]) ** 2 + (cy - d[2]) ** 2 > (R + d[0] + 0.03) ** 2 for d in discs):
            discs.append((R, cx, cy))
    return discs


def mac_params(N, specs, U_lid=1.0, mu_s=0.3, mu_f=0.01, rho=1.0, eta=2.0):
    """rmt_mac_params and the fixed dt of mac_multi_disc_lid.py:36-60."""
    dx, _ = mac_grid(N, N)
    specs = list(specs)
    if not 1 <= len(specs) <= 8:
        raise ValueError("1..8 discs")
    cs = np.sqrt(mu_s / rho)
    dt = min(0.3 * dx / U_lid, 0.2 * dx * dx / (mu_f / rho), 0.3 * dx / (cs + 1e-9))
    P = L.rmt_mac_params()
    P.N = N; P.dx = dx; P.n_discs = len(specs)
    for k, (R, cx, cy) in enumerate(specs):
        P.R[k], P.cx[k], P.cy[k] = R, cx, cy
    P.U_lid, P.mu_s, P.mu_f, P.rho, P.eta = U_lid, mu_s, mu_f, rho, eta
    P.layers = 3
    P.dt = float(dt)
    return P, float(dt)


def initial_maps(N, specs):
    """(X1, X2, phi) per disc (mac_multi_disc_lid.py:51-56): xi = x_c * mask, extrapolated."""
    dx, dy = mac_grid(N, N)
    xc = (np.arange(N) + 0.5) * dx
    Xc, Yc = np.meshgrid(xc, xc)
    out = []
    for R, cx, cy in specs:
        phi = np.sqrt((Xc - cx) ** 2 + (Yc - cy) ** 2) - R
        m = (phi <= 0).astype(float)
        X1, X2 = extrapolate_reference_map(Xc * m, Yc * m, phi, dx, dy, 3)
        out.append((X1, X2, np.sqrt((X1 - cx) ** 2 + (X2 - cy) ** 2) - R))
    return out


class MacMultiDisc:
    """benchmarks/mac_multi_disc_lid.py:36-98 on the GPU (rmt_mac_sim_*): state (u, v, p and
    every disc's X1, X2, phi) stays in HBM; one host sync per step reads the diagnostics."""

    FIELDS = {"u": 0, "v": 1, "p": 2, "X1": 3, "X2": 4, "phi": 5}

    def __init__(self, N=128, n_discs=3, seed=3, U_lid=1.0, mu_s=0.3, mu_f=0.01, rho=1.0,
                 eta=2.0, specs=None, options=None):
        import torch
        if not torch.cuda.is_available():
            raise RuntimeError("pyrmt_amd needs a visible MI355X")
        self.torch, self.N = torch, N
        dx, dy = mac_grid(N, N)
        self.dx = dx
        self.specs = list(specs) if specs is not None else place_discs(n_discs, seed)
        if not 1 <= len(self.specs) <= 8:
            raise ValueError("1..8 discs")
        P, self.dt = mac_params(N, self.specs, U_lid, mu_s, mu_f, rho, eta)
        if options:
            # a context of its own with these implementation switches (rmt_ctx_set_option)
            from .functions import _Ctx
            self.ctx = _Ctx(N, N, torch.cuda.current_device())
            for k, v in options.items():
                self.ctx.set_option(k, v)
        else:
            self.ctx = ctx_for(N, N)
        h = ctypes.c_void_p()
        L.check(L.lib().rmt_mac_sim_create(self.ctx.bind(), ctypes.byref(P), ctypes.byref(h)),
                "rmt_mac_sim_create")
        self.h, self.params = h, P
        self._views = {}
        # the initial maps go up through one pinned staging plane: a DMA copy per map instead of
        # the runtime's pageable staging (≈0.6 MB chunks: ~7,800 copies at N=8192)
        stage = torch.empty((N, N), dtype=torch.float64, pin_memory=True)
        cur = torch.cuda.current_stream()
        for k, maps in enumerate(initial_maps(N, self.specs)):
            for name, a in zip(("X1", "X2", "phi"), maps):
                stage.numpy()[...] = a
                self.field(name, k).copy_(stage, non_blocking=True)
                cur.synchronize()   # (before the staging plane is refilled)

    def __del__(self):
        try:
            L.lib().rmt_mac_sim_destroy(self.h)
        except Exception:
            pass

    def field(self, name, disc=0):
        key = (name, disc if name in ("X1", "X2", "phi") else 0)
        if key not in self._views:
            ptr = ctypes.c_void_p()
            L.check(L.lib().rmt_mac_sim_field(self.h, self.FIELDS[name], key[1], ctypes.byref(ptr)))
            N = self.N
            shape = {"u": (N, N + 1), "v": (N + 1, N)}.get(name, (N, N))
            self._views[key] = _wrap_device(self.torch, ptr.value, shape)
        return self._views[key]

    def get(self, name, disc=0):
        self.torch.cuda.synchronize()
        return self.field(name, disc).cpu().numpy()

    def step(self, nsteps=1, t_end=math.inf):
        self.ctx.bind()
        L.check(L.lib().rmt_mac_sim_step(self.h, int(nsteps), float(t_end)), "rmt_mac_sim_step")

    def diagnostics(self):
        n = ctypes.c_int()
        L.check(L.lib().rmt_mac_sim_diagnostics(self.h, None, 0, ctypes.byref(n)))
        buf = (L.rmt_mac_diag * max(n.value, 1))()
        L.check(L.lib().rmt_mac_sim_diagnostics(self.h, buf, n.value, ctypes.byref(n)))
        K = len(self.specs)
        out = {k: np.array([getattr(buf[i], k) for i in range(n.value)])
               for k in ("t", "dt", "minJ", "maxJ", "umax")}
        out["diverged"] = np.array([buf[i].diverged for i in range(n.value)], dtype=np.int32)
        out["cx"] = np.array([[buf[i].cx[k] for k in range(K)] for i in range(n.value)])
        out["cy"] = np.array([[buf[i].cy[k] for k in range(K)] for i in range(n.value)])
        return out
