"""mac_oracle -- CPU restatement of pyRMT's MAC path, config 5 (TEST INFRASTRUCTURE ONLY).

Only tests/ and bench.py's cpu_baseline leg may import this module, as the checker.
pyRMT/mac.py is pure NumPy in the reference; it is restated here with the same NumPy
operations in the same order (so bit-exact with the reference), the DCT-II through
scipy.fft like mac.py:118-123.  The per-disc reference-map advection / extrapolation /
stress reuse the C restatement in oracle.py.  Pinned by tests/golden/mac_ops.npz and
mac_trace.npz (tests/test_oracle_golden.py).  The IMEX tier (mac.py:243-369): the ghost-cell
Laplacians with the same NumPy expressions, scipy 1.15's cg restated (oracle.cg's loop with
x0 = rhs) and the DST preconditioner through scipy.fft.dstn / idstn as mac.py:304-306;
pinned by tests/golden/imex.npz.
"""
import numpy as np

from .oracle import (advect_reference_map, extrapolate_reference_map, grad_central_x_2nd,
                     grad_central_y_2nd, rebuild_phi_disc, smoothed_heaviside,
                     solid_cauchy_stress)


def mac_grid(Nx, Ny, Lx=1.0, Ly=1.0):
    """mac.py:22-23: cell sizes of an Nx x Ny cell grid."""
    return Lx / Nx, Ly / Ny


def divergence(u, v, dx, dy):
    """mac.py:81-84: cell-centred divergence of the face velocities."""
    return (u[:, 1:] - u[:, :-1]) / dx + (v[1:, :] - v[:-1, :]) / dy


def gradient_p_u(p, dx):
    """mac.py:87-93: dp/dx on the interior u faces, wall faces 0."""
    g = np.zeros((p.shape[0], p.shape[1] + 1))
    g[:, 1:-1] = (p[:, 1:] - p[:, :-1]) / dx
    return g


def gradient_p_v(p, dy):
    """mac.py:96-101: dp/dy on the interior v faces, wall faces 0."""
    g = np.zeros((p.shape[0] + 1, p.shape[1]))
    g[1:-1, :] = (p[1:, :] - p[:-1, :]) / dy
    return g


def poisson_eigs_neumann(Nx, Ny, dx, dy):
    """mac.py:104-115: DCT-II symbol of the cell-centred Neumann Laplacian, (0,0) -> 1."""
    lx = -2.0 * (1.0 - np.cos(np.pi * np.arange(Nx) / Nx)) / dx ** 2
    ly = -2.0 * (1.0 - np.cos(np.pi * np.arange(Ny) / Ny)) / dy ** 2
    eig = (lx[np.newaxis, :] + ly[:, np.newaxis]).copy()
    eig[0, 0] = 1.0
    return eig


def solve_poisson_neumann(rhs, eig):
    """mac.py:118-123: orthonormal DCT-II both ways, constant mode zeroed."""
    from scipy.fft import dctn, idctn
    h = dctn(rhs, type=2, norm='ortho') / eig
    h[0, 0] = 0.0
    return idctn(h, type=2, norm='ortho')


def project(u_star, v_star, dx, dy, dt, rho, eig):
    """mac.py:126-139: exact projection of the face velocities."""
    rhs = (rho / dt) * divergence(u_star, v_star, dx, dy)
    rhs = rhs - rhs.mean()
    phi = solve_poisson_neumann(rhs, eig)
    return (u_star - (dt / rho) * gradient_p_u(phi, dx),
            v_star - (dt / rho) * gradient_p_v(phi, dy), phi)


def momentum_predictor(u, v, nu, dx, dy, dt, U_lid, fu=None, fv=None, rho=1.0):
    """mac.py:196-232 (+ ghosts :147-166, face averages :168-177): explicit central
    advection + diffusion, lid / no-slip by reflected ghosts, face forces / rho."""
    Ny, Nx = u.shape[0], u.shape[1] - 1
    ug = np.empty((Ny + 2, Nx + 1)); ug[1:-1] = u
    ug[0] = -u[0]; ug[-1] = 2.0 * U_lid - u[-1]
    vg = np.empty((Ny + 1, Nx + 2)); vg[:, 1:-1] = v
    vg[:, 0] = -v[:, 0]; vg[:, -1] = -v[:, -1]
    uc = u[:, 1:-1]
    vu = 0.25 * (v[:-1, :-1] + v[:-1, 1:] + v[1:, :-1] + v[1:, 1:])
    ru = (-(uc * ((u[:, 2:] - u[:, :-2]) / (2 * dx))
            + vu * ((ug[2:, 1:-1] - ug[:-2, 1:-1]) / (2 * dy)))
          + nu * ((u[:, 2:] - 2 * uc + u[:, :-2]) / dx ** 2
                  + (ug[2:, 1:-1] - 2 * ug[1:-1, 1:-1] + ug[:-2, 1:-1]) / dy ** 2))
    if fu is not None:
        ru = ru + fu[:, 1:-1] / rho
    us = u.copy(); us[:, 1:-1] = uc + dt * ru
    us[:, 0] = 0.0; us[:, -1] = 0.0
    vc = v[1:-1, :]
    uv = 0.25 * (u[:-1, :-1] + u[:-1, 1:] + u[1:, :-1] + u[1:, 1:])
    rv = (-(uv * ((vg[1:-1, 2:] - vg[1:-1, :-2]) / (2 * dx))
            + vc * ((v[2:, :] - v[:-2, :]) / (2 * dy)))
          + nu * ((vg[1:-1, 2:] - 2 * vg[1:-1, 1:-1] + vg[1:-1, :-2]) / dx ** 2
                  + (v[2:, :] - 2 * vc + v[:-2, :]) / dy ** 2))
    if fv is not None:
        rv = rv + fv[1:-1, :] / rho
    vs = v.copy(); vs[1:-1, :] = vc + dt * rv
    vs[0, :] = 0.0; vs[-1, :] = 0.0
    return us, vs


def contact_stress(phi_a, phi_b, eta, Gsum, eps, dx, dy):
    """mac.py:729-749: trace-free pair contact stress (Rycroft et al. 2018)."""
    f = [np.where(q < eps, 0.5 * (1.0 - q / eps), 0.0) for q in (phi_a, phi_b)]
    fc = np.minimum(f[0], f[1])
    d = phi_a - phi_b
    gx = np.zeros_like(d); gy = np.zeros_like(d)
    gx[:, 1:-1] = (d[:, 2:] - d[:, :-2]) / (2 * dx)
    gy[1:-1, :] = (d[2:, :] - d[:-2, :]) / (2 * dy)
    mag = np.sqrt(gx * gx + gy * gy) + 1e-12
    nx_, ny_ = gx / mag, gy / mag
    s = -eta * fc * Gsum
    return s * (nx_ * nx_ - 0.5), s * (nx_ * ny_), s * (ny_ * ny_ - 0.5)


def place_discs(n, seed, Rrange=(0.07, 0.12), box=(0.18, 0.82)):
    """mac_multi_disc_lid.py:22-33: rejection-sampled non-overlapping discs (R, cx, cy)."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(2000):
        if len(out) == n:
            break
        R = rng.uniform(*Rrange)
        cx = rng.uniform(box[0] + R, box[1] - R); cy = rng.uniform(box[0] + R, box[1] - R)
        if all((cx - d[1]) ** 2 + (cy - d[2]) ** 2 > (R + d[0] + 0.03) ** 2 for d in out):
            out.append((R, cx, cy))
    return out


class MacMultiDisc:
    """benchmarks/mac_multi_disc_lid.py:36-111 (config 5) loop body: K discs, each with
    its own reference map advected on the cell-centre velocity, blended solid stress +
    pair contact stress -> face force, explicit MAC predictor, exact DCT-II projection."""

    def __init__(self, N, n_discs=3, seed=3, U_lid=1.0, mu_s=0.3, mu_f=0.01, rho=1.0, eta=2.0):
        dx, dy = mac_grid(N, N)
        self.N, self.dx, self.dy = N, dx, dy
        xc = (np.arange(N) + 0.5) * dx
        self.Xc, self.Yc = np.meshgrid(xc, xc)
        self.Xg, self.Yg = np.meshgrid(np.arange(N) * dx, np.arange(N) * dy)
        self.w_t, self.nu, self.eps = 2.0 * dx, mu_f / rho, 3.0 * dx
        self.U, self.mu_s, self.rho, self.eta = U_lid, mu_s, rho, eta
        self.specs = place_discs(n_discs, seed)
        self.refs = []
        for (R, cx, cy) in self.specs:
            phi = rebuild_phi_disc(self.Xc, self.Yc, cx, cy, R)
            m = (phi <= 0).astype(float)
            self.refs.append(list(extrapolate_reference_map(self.Xc * m, self.Yc * m, phi,
                                                            dx, dy, 3)))
        self.u = np.zeros((N, N + 1)); self.v = np.zeros((N + 1, N)); self.p = None
        self.eig = poisson_eigs_neumann(N, N, dx, dy)
        cs = np.sqrt(mu_s / rho)
        self.dt = min(0.3 * dx / U_lid, 0.2 * dx * dx / self.nu, 0.3 * dx / (cs + 1e-9))
        self.t = 0.0

    def step(self, t_end=np.inf):
        N, dx, dy = self.N, self.dx, self.dy
        dt = self.dt
        if self.t + dt > t_end:
            dt = t_end - self.t
        u_c = 0.5 * (self.u[:, :-1] + self.u[:, 1:]); v_c = 0.5 * (self.v[:-1, :] + self.v[1:, :])
        phis = []
        for k, (R, cx, cy) in enumerate(self.specs):
            X1, X2 = self.refs[k]
            phi = rebuild_phi_disc(X1, X2, cx, cy, R); m = (phi <= 0).astype(float)
            X1 = advect_reference_map(X1, u_c, v_c, self.Xg, self.Yg, dt, dx, dy, phi) * m
            X2 = advect_reference_map(X2, u_c, v_c, self.Xg, self.Yg, dt, dx, dy, phi) * m
            X1, X2 = extrapolate_reference_map(X1, X2, phi, dx, dy, 3)
            self.refs[k] = [X1, X2]
            phis.append(rebuild_phi_disc(X1, X2, cx, cy, R))
        S = [np.zeros((N, N)) for _ in range(3)]
        Jmin = Jmax = 1.0
        for k in range(len(self.refs)):
            sxx, sxy, syy, J = solid_cauchy_stress(self.refs[k][0], self.refs[k][1], dx, dy,
                                                   self.mu_s, 0.0, phis[k])
            H = smoothed_heaviside(phis[k], self.w_t)
            S[0] += (1 - H) * sxx; S[1] += (1 - H) * sxy; S[2] += (1 - H) * syy
            Jmin = min(Jmin, J.min()); Jmax = max(Jmax, J.max())
        if self.eta > 0:
            for i in range(len(phis)):
                for j in range(i + 1, len(phis)):
                    t3 = contact_stress(phis[i], phis[j], self.eta, 2 * self.mu_s, self.eps,
                                        dx, dy)
                    for q in range(3):
                        S[q] += t3[q]
        divx = grad_central_x_2nd(S[0], dx) + grad_central_y_2nd(S[1], dy)
        divy = grad_central_x_2nd(S[1], dx) + grad_central_y_2nd(S[2], dy)
        fu = np.zeros((N, N + 1)); fu[:, 1:-1] = 0.5 * (divx[:, 1:] + divx[:, :-1])
        fv = np.zeros((N + 1, N)); fv[1:-1, :] = 0.5 * (divy[1:, :] + divy[:-1, :])
        us, vs = momentum_predictor(self.u, self.v, self.nu, dx, dy, dt, self.U,
                                    fu=fu, fv=fv, rho=self.rho)
        self.u, self.v, self.p = project(us, vs, dx, dy, dt, self.rho, self.eig)
        self.t += dt
        self.phis = phis
        cents = [(self.Xc[q <= 0].mean(), self.Yc[q <= 0].mean()) for q in phis]
        return dict(t=self.t, dt=dt, minJ=Jmin, maxJ=Jmax,
                    cx=np.array([c[0] for c in cents]), cy=np.array([c[1] for c in cents]))


# ------------------------------------------------------------------ IMEX tier --------
def lap_u_lid_hom(u, dx, dy):
    """mac.py:243-250: Laplacian of u (Ny, Nx+1) on the interior faces, walls u = 0 and
    reflected (homogeneous) ghost rows."""
    up = np.empty((u.shape[0] + 2, u.shape[1])); up[1:-1] = u; up[0] = -u[0]; up[-1] = -u[-1]
    uc = u[:, 1:-1]
    return ((u[:, 2:] - 2 * uc + u[:, :-2]) / dx ** 2
            + (up[2:, 1:-1] - 2 * up[1:-1, 1:-1] + up[:-2, 1:-1]) / dy ** 2)


def lap_v_lid_hom(v, dx, dy):
    """mac.py:253-260: Laplacian of v (Ny+1, Nx) on the interior faces, reflected ghost
    columns."""
    vp = np.empty((v.shape[0], v.shape[1] + 2)); vp[:, 1:-1] = v
    vp[:, 0] = -v[:, 0]; vp[:, -1] = -v[:, -1]
    vc = v[1:-1, :]
    return ((vp[1:-1, 2:] - 2 * vp[1:-1, 1:-1] + vp[1:-1, :-2]) / dx ** 2
            + (v[2:, :] - 2 * vc + v[:-2, :]) / dy ** 2)


def dst_helmholtz_eigs(shp, dx, dy):
    """mac.py:278-284: homogeneous-Dirichlet Laplacian eigenvalues of the DST-II."""
    Ny, Nx = shp
    lx = -2.0 * (1.0 - np.cos(np.pi * (np.arange(Nx) + 1) / Nx)) / dx ** 2
    ly = -2.0 * (1.0 - np.cos(np.pi * (np.arange(Ny) + 1) / Ny)) / dy ** 2
    return ly[:, None] + lx[None, :]


def cg_x0(matvec, b, psolve, rtol, maxiter):
    """scipy.sparse.linalg.cg (scipy 1.15) with x0 = b and atol = 0 (mac.py:274, 312):
    r = b - A x0, then the loop of oracle.cg.  Returns (x, iterations run)."""
    x = b.copy()
    bnrm2 = np.linalg.norm(b)
    if bnrm2 == 0:
        return b.copy(), 0
    atol = rtol * bnrm2
    r = b - matvec(x) if x.any() else b.copy()
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


def helmholtz(rhs, kind, coef, dx, dy, rtol, maxiter=500, precond=True):
    """mac.py:263-316: (I - coef Lap_hom) x = rhs on the u (kind 0) or v (kind 1) interior
    faces; CG, or PCG with the DST-II preconditioner (I - coef Lap_Dirichlet)^-1.
    Returns (x, iterations)."""
    from scipy.fft import dstn, idstn
    shp = rhs.shape
    if kind == 0:
        emb = lambda x: np.pad(x, ((0, 0), (1, 1)))
        lap = lambda w: lap_u_lid_hom(w, dx, dy)
    else:
        emb = lambda x: np.pad(x, ((1, 1), (0, 0)))
        lap = lambda w: lap_v_lid_hom(w, dx, dy)
    denom = 1.0 - coef * dst_helmholtz_eigs(shp, dx, dy)

    def matvec(xf):
        x = xf.reshape(shp)
        return (x - coef * lap(emb(x))).ravel()

    def prec(rf):
        return idstn(dstn(rf.reshape(shp), type=2, norm='ortho') / denom, type=2,
                     norm='ortho').ravel()

    x, it = cg_x0(matvec, rhs.ravel().copy(), prec if precond else (lambda r: r), rtol, maxiter)
    return x.reshape(shp), it


def momentum_predictor_lid_imex(u, v, nu, dx, dy, dt, U_lid, fu=None, fv=None, rho=1.0,
                                rtol=1e-8, cs2=0.0):
    """mac.py:319-369: explicit central advection + face forces, implicit viscosity (+ the
    trapezoidal elastic term for cs2 > 0) by DST-preconditioned CG.  Returns (u*, v*)."""
    Ny, Nx = u.shape[0], u.shape[1] - 1
    up = np.empty((Ny + 2, Nx + 1)); up[1:-1] = u; up[0] = -u[0]; up[-1] = 2.0 * U_lid - u[-1]
    vp = np.empty((Ny + 1, Nx + 2)); vp[:, 1:-1] = v; vp[:, 0] = -v[:, 0]; vp[:, -1] = -v[:, -1]
    c_el = 0.25 * dt * dt * cs2
    coef = dt * nu + c_el
    uc = u[:, 1:-1]
    dudx = (u[:, 2:] - u[:, :-2]) / (2 * dx)
    dudy = (up[2:, 1:-1] - up[:-2, 1:-1]) / (2 * dy)
    v_u = 0.25 * (v[:-1, :-1] + v[:-1, 1:] + v[1:, :-1] + v[1:, 1:])
    rhs_u = uc + dt * (-(uc * dudx + v_u * dudy))
    if fu is not None:
        rhs_u = rhs_u + dt * fu[:, 1:-1] / rho
    if c_el > 0.0:
        rhs_u = rhs_u + c_el * lap_u_lid_hom(u, dx, dy)
    rhs_u[-1, :] += coef * (2.0 * U_lid / dy ** 2)
    sol_u, _ = helmholtz(rhs_u, 0, coef, dx, dy, rtol)
    ustar = u.copy(); ustar[:, 1:-1] = sol_u; ustar[:, 0] = 0.0; ustar[:, -1] = 0.0
    vc = v[1:-1, :]
    dvdy = (v[2:, :] - v[:-2, :]) / (2 * dy)
    dvdx = (vp[1:-1, 2:] - vp[1:-1, :-2]) / (2 * dx)
    u_v = 0.25 * (u[:-1, :-1] + u[:-1, 1:] + u[1:, :-1] + u[1:, 1:])
    rhs_v = vc + dt * (-(u_v * dvdx + vc * dvdy))
    if fv is not None:
        rhs_v = rhs_v + dt * fv[1:-1, :] / rho
    if c_el > 0.0:
        rhs_v = rhs_v + c_el * lap_v_lid_hom(v, dx, dy)
    sol_v, _ = helmholtz(rhs_v, 1, coef, dx, dy, rtol)
    vstar = v.copy(); vstar[1:-1, :] = sol_v; vstar[0, :] = 0.0; vstar[-1, :] = 0.0
    return ustar, vstar


def momentum_predictor_lid_semilag(u, v, nu, dx, dy, dt, U_lid, fu=None, fv=None, rho=1.0,
                                   cs2=0.0, rtol=1e-8, cfl_switch=0.9):
    """mac.py:381-442: IMEX below cfl_switch, else the midpoint semi-Lagrangian backtrace
    through scipy.ndimage.map_coordinates(order=3, mode='nearest') (the reference's own
    call, mac.py:374-378) and the PCG viscosity solve."""
    from scipy.ndimage import map_coordinates
    interp = lambda f, iq, jq: map_coordinates(f, [jq, iq], order=3, mode="nearest")
    cfl = dt * max(np.max(np.abs(u)) / dx, np.max(np.abs(v)) / dy)
    if cfl <= cfl_switch:
        return momentum_predictor_lid_imex(u, v, nu, dx, dy, dt, U_lid, fu=fu, fv=fv, rho=rho,
                                           rtol=rtol, cs2=cs2)
    Ny, Nx = u.shape[0], u.shape[1] - 1
    up = np.empty((Ny + 2, Nx + 1)); up[1:-1] = u; up[0] = -u[0]; up[-1] = 2.0 * U_lid - u[-1]
    vp = np.empty((Ny + 1, Nx + 2)); vp[:, 1:-1] = v; vp[:, 0] = -v[:, 0]; vp[:, -1] = -v[:, -1]
    Ii, Jj = np.meshgrid(np.arange(1, Nx), np.arange(Ny))
    xf = Ii * dx; yf = (Jj + 0.5) * dy
    velx = u[:, 1:-1]; vely = 0.25 * (v[:-1, :-1] + v[:-1, 1:] + v[1:, :-1] + v[1:, 1:])
    xm = xf - 0.5 * dt * velx; ym = yf - 0.5 * dt * vely
    vxm = interp(u, xm / dx, ym / dy)
    vym = interp(vp, xm / dx + 0.5, ym / dy - 0.0)
    xd = xf - dt * vxm; yd = yf - dt * vym
    u_adv = np.zeros_like(u)
    u_adv[:, 1:-1] = interp(up, xd / dx, yd / dy + 0.5)
    Iv, Jv = np.meshgrid(np.arange(Nx), np.arange(1, Ny))
    xfv = (Iv + 0.5) * dx; yfv = Jv * dy
    velxv = 0.25 * (u[:-1, :-1] + u[:-1, 1:] + u[1:, :-1] + u[1:, 1:]); velyv = v[1:-1, :]
    xmv = xfv - 0.5 * dt * velxv; ymv = yfv - 0.5 * dt * velyv
    vxmv = interp(up, xmv / dx, ymv / dy + 0.5)
    vymv = interp(v, xmv / dx - 0.5, ymv / dy)
    xdv = xfv - dt * vxmv; ydv = yfv - dt * vymv
    v_adv = np.zeros_like(v)
    v_adv[1:-1, :] = interp(vp, xdv / dx + 0.5, ydv / dy)
    c_el = 0.25 * dt * dt * cs2
    coef = dt * nu + c_el
    rhs_u = u_adv[:, 1:-1].copy()
    if fu is not None:
        rhs_u = rhs_u + dt * fu[:, 1:-1] / rho
    if c_el > 0.0:
        rhs_u = rhs_u + c_el * lap_u_lid_hom(u, dx, dy)
    rhs_u[-1, :] += coef * (2.0 * U_lid / dy ** 2)
    sol_u, _ = helmholtz(rhs_u, 0, coef, dx, dy, rtol)
    ustar = u.copy(); ustar[:, 1:-1] = sol_u; ustar[:, 0] = 0.0; ustar[:, -1] = 0.0
    rhs_v = v_adv[1:-1, :].copy()
    if fv is not None:
        rhs_v = rhs_v + dt * fv[1:-1, :] / rho
    if c_el > 0.0:
        rhs_v = rhs_v + c_el * lap_v_lid_hom(v, dx, dy)
    sol_v, _ = helmholtz(rhs_v, 1, coef, dx, dy, rtol)
    vstar = v.copy(); vstar[1:-1, :] = sol_v; vstar[0, :] = 0.0; vstar[-1, :] = 0.0
    return ustar, vstar
