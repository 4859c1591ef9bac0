"""Golden-vector generator: runs the pyRMT reference (read-only, at /root/reference)
in pure-Python mode and writes small input/output fixtures to tests/golden/*.npz.

This script is TEST INFRASTRUCTURE. It is run only in the development container
(the reference never travels to the GPU box); the committed .npz files are data.

How the reference is made importable:
  * numba is absent -> a stand-in module whose ``njit`` is the identity decorator and
    ``prange`` is ``range`` (Numba semantics: no fastmath anywhere in the reference,
    so per-element IEEE results are the same);
  * pyamg / h5py are absent -> empty stand-ins (never reached on the fixture paths);
  * Numba lowers scalar ``np.exp`` to libm ``exp``; numpy's SIMD exp differs from libm
    in a few % of inputs, so ``pyRMT.functions.np.exp`` is patched to ``math.exp``
    (the only patch).
  * PYTHONDONTWRITEBYTECODE keeps __pycache__ out of the reference tree.

Usage:  python tests/golden/gen_golden.py [--ghia]
"""
import math
import os
import sys
import tempfile
import time
import types

sys.dont_write_bytecode = True
REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))

_STUB_NUMBA = '''
def njit(*a, **k):
    return a[0] if (len(a) == 1 and callable(a[0]) and not k) else (lambda f: f)
prange = range
'''


def _import_reference():
    stub_dir = tempfile.mkdtemp(prefix="rmt_stubs_")
    for name, body in (("numba", _STUB_NUMBA),
                       ("pyamg", "def ruge_stuben_solver(*a, **k):\n    raise RuntimeError('stub')\n"),
                       ("h5py", "")):
        os.makedirs(os.path.join(stub_dir, name))
        with open(os.path.join(stub_dir, name, "__init__.py"), "w") as f:
            f.write(body)
    sys.path[:0] = [stub_dir, REF]
    import numpy as np
    import pyRMT.functions as F
    # Numba-faithful scalar exp (libm), see module docstring.
    F.np = types.SimpleNamespace(**{k: getattr(np, k) for k in dir(np) if not k.startswith("__")})
    F.np.exp = math.exp
    import pyRMT.interpolators as I
    import pyRMT.utils as U
    import pyRMT.output as O
    import pyRMT.mac as M
    import benchmarks.common as C
    return F, I, U, O, M, C


F, I, U, O, M, C = _import_reference()
import numpy as np  # noqa: E402


def save(name, **arrs):
    path = os.path.join(OUT, name + ".npz")
    np.savez_compressed(path, **{k: np.asarray(v) for k, v in arrs.items()})
    print(f"  wrote {name}.npz ({os.path.getsize(path)/1024:.0f} KiB)")


# ── 1. FD helpers / interpolators on random data (all branches) ─────────────────
def gen_primitives():
    rng = np.random.default_rng(1234)
    N = 33
    X, Y, dx, dy = F.create_grid(N, N, 1.0, 1.0)
    f = rng.standard_normal((N, N))
    u = rng.standard_normal((N, N))
    u[rng.random((N, N)) < 0.1] = 0.0          # exercise the vel<=0 / ==0 branches
    gx = U.grad_central_x_2nd(f, dx)
    gy = U.grad_central_y_2nd(f, dy)
    up1 = U.diff_upwind_3rd(f, u, dx, 1)
    up0 = U.diff_upwind_3rd(f, u, dy, 0)
    # bilinear: random queries incl. out-of-range, non-finite and huge
    xq = rng.uniform(-0.2, 1.2, (N, N)); yq = rng.uniform(-0.2, 1.2, (N, N))
    xq[0, 0] = np.nan; yq[1, 1] = np.inf; xq[2, 2] = -np.inf
    xq[3, 3] = 1e200; yq[4, 4] = -1e200
    xq[5, 5] = 1.0; yq[5, 5] = 1.0                 # exact top-right corner
    bil = I.bilinear_interpolate(f, xq, yq, dx, dy, N, N)
    H = F.smoothed_heaviside(rng.uniform(-3 * dx, 3 * dx, (N, N)), 2 * dx)
    Hin = rng.uniform(-3 * dx, 3 * dx, (N, N))
    H = F.smoothed_heaviside(Hin, 2 * dx)
    # 3x3 Cramer solve
    A = rng.standard_normal((64, 3, 3)); bb = rng.standard_normal((64, 3))
    A[0] = 0.0                                     # singular -> zeros
    sol = np.stack([U.fast_solve_3x3(A[k], bb[k]) for k in range(64)])
    save("primitives", N=N, dx=dx, dy=dy, f=f, u=u, gx=gx, gy=gy, up1=up1, up0=up0,
         xq=xq, yq=yq, bil=bil, Hin=Hin, H=H, A=A, b=bb, sol=sol)


# ── 2. Soft disc in lid cavity (configs 2/4 physics): driver loop + op fixtures ──
def soft_disc_loop(N, nsteps, capture_steps=(), t_end=8.0):
    """Restates benchmarks/soft_disc_in_lid_driven.py:165-235 (the driver loop) by
    calling the reference operators in the same order; verified against run()."""
    X, Y, dx, dy = F.create_grid(N, N, 1.0, 1.0)
    bc = lambda u, v: C.no_slip_lid_bc(u, v, 1.0)
    x0, y0, R = 0.6, 0.5, 0.2
    phi_init = lambda Xq, Yq: C.initialize_disc(Xq, Yq, x0, y0, R)
    phi = F.apply_phi_BCs(phi_init(X, Y))
    solid_mask = (phi <= 0).astype(float)
    mu_s, kappa, rho_s, eta_s = 0.1, 0.0, 1.0, 0.01
    mu_f, rho_f = 0.01, 1.0
    w_t = 2.0 * dx
    num_layers = max(3, C.check_narrow_band(w_t, dx, 3))
    X1 = X * solid_mask; X2 = Y * solid_mask
    init_in = dict(X1m=X1.copy(), X2m=X2.copy(), phi0=phi.copy())
    X1, X2 = F.extrapolate_reference_map(X1, X2, phi, dx, dy, num_layers)
    init_out = dict(X1e=X1.copy(), X2e=X2.copy())
    a = np.zeros((N, N)); b = np.zeros((N, N)); p = np.zeros((N, N))
    CFL, cap = 0.2, 1e-3
    eig = F._precompute_poisson_eigenvalues(N, N, dx, dy)
    traj = []; caps = {}
    t = 0.0
    for step in range(1, nsteps + 1):
        if not t < t_end:
            break
        dt = F.compute_timestep(a, b, dx, dy, CFL, cap, mu_s, rho_s, 0.0, rho_f,
                                mu_f=mu_f, eta_s=eta_s, kappa=kappa)
        if t + dt > t_end:
            dt = t_end - t
        rec = step in capture_steps
        c = {}
        if rec:
            c.update(a=a.copy(), b=b.copy(), p=p.copy(), X1=X1.copy(), X2=X2.copy(), dt=dt, t=t)
        phi = F.rebuild_phi_from_reference_map(X1, X2, phi_init)
        phi = F.reinitialize_level_set(phi, dx, dy, method='none')
        solid_mask = (phi <= 0).astype(float)
        X1a = F.advect_reference_map(X1, a, b, X, Y, dt, dx, dy, phi, 'semilagrangian', 0.0)
        X2a = F.advect_reference_map(X2, a, b, X, Y, dt, dx, dy, phi, 'semilagrangian', 0.0)
        X1 = X1a * solid_mask; X2 = X2a * solid_mask
        if rec:
            c.update(phi_pre=phi.copy(), X1_adv=X1a, X2_adv=X2a, X1_m=X1.copy(), X2_m=X2.copy())
        X1, X2 = F.extrapolate_reference_map(X1, X2, phi, dx, dy, num_layers)
        phi = F.rebuild_phi_from_reference_map(X1, X2, phi_init)
        if rec:
            c.update(X1_ext=X1.copy(), X2_ext=X2.copy(), phi_post=phi.copy())
        a_star, b_star, sxx, sxy, syy, J = F.momentum_step_rk4(
            a, b, p, X1, X2, bc, mu_s, kappa, eta_s, dx, dy, dt,
            rho_s, rho_f, phi, mu_f, w_t, 0.0, stress_band=False, detg_clamp=3.0)
        H = F.smoothed_heaviside(phi, w_t)
        rho_local = (1 - H) * rho_s + H * rho_f
        if rec:
            c.update(a_star=a_star, b_star=b_star, sxx=sxx, sxy=sxy, syy=syy, J=J, H=H,
                     rho_local=rho_local)
        p_in = p
        a, b, p, _, _ = F.pressure_projection_amg(
            a_star, b_star, dx, dy, dt, rho_local, velocity_bc=bc,
            A=None, ml=None, p_prev=p_in, eigenvalues=eig, bc_type='neumann')
        if rec:
            c.update(divU=F._compute_divergence_rc(a_star, b_star, p_in, dt, rho_local, dx, dy),
                     a_new=a.copy(), b_new=b.copy(), p_new=p.copy())
            caps[step] = c
        cx, cy = C.disc_centroid(phi, X, Y)
        t += dt
        traj.append((t, cx, cy, J.min(), J.max()))
    return np.array(traj), dict(a=a, b=b, p=p, X1=X1, X2=X2, phi=phi), caps, init_in, init_out


def gen_soft_disc():
    N, nsteps = 65, 30
    t0 = time.time()
    traj, fin, caps, ii, io = soft_disc_loop(N, nsteps, capture_steps=(1, 12, 30))
    print(f"  soft disc N={N}: {nsteps} steps in {time.time()-t0:.1f}s; "
          f"final centroid {traj[-1,1]:.10f},{traj[-1,2]:.10f}")
    save("soft_disc_trace", N=N, traj=traj, **fin)
    save("soft_disc_init", N=N, **ii, **io)
    for s, c in caps.items():
        save(f"soft_disc_step{s:02d}", N=N, step=s, **c)


def gen_soft_disc_driver_check():
    """Check the loop restatement against the reference driver run() itself."""
    import benchmarks.soft_disc_in_lid_driven as SD
    out = tempfile.mkdtemp(prefix="rmt_out_")
    import io, contextlib
    with contextlib.redirect_stdout(io.StringIO()):
        traj_ref = SD.run(N=33, t_end=0.006, out_root=out)
    traj, *_ = soft_disc_loop(33, 1000, t_end=0.006)
    assert np.array_equal(traj_ref, traj), "driver restatement mismatch"
    save("soft_disc_driver33", traj=traj_ref)
    print(f"  soft disc driver restatement == run() over {len(traj)} steps")


# ── 3. Operator edge cases: stress modes, extrapolation exactness, projection ───
def gen_operator_cases():
    rng = np.random.default_rng(99)
    N = 49
    X, Y, dx, dy = F.create_grid(N, N, 1.0, 1.0)
    phi = np.sqrt((X - 0.5) ** 2 + (Y - 0.5) ** 2) - 0.25
    # deformed map: smooth nonlinear perturbation of identity
    X1 = X + 0.05 * np.sin(2 * np.pi * Y) * np.cos(np.pi * X)
    X2 = Y - 0.04 * np.sin(np.pi * X) * np.sin(2 * np.pi * Y)
    out = {}
    out["legacy"] = F.solid_cauchy_stress(X1, X2, dx, dy, 0.7, 0.3, phi)
    out["band"] = F.solid_cauchy_stress(X1, X2, dx, dy, 0.7, 0.3, phi, w_cut=2 * dx, detg_clamp=3.0)
    out["iso"] = F.solid_cauchy_stress(X1, X2, dx, dy, 0.7, 0.3, phi, w_cut=2 * dx, detg_clamp=0.0,
                                       isochoric=True)
    X1c = 10.0 * X
    out["clamp"] = F.solid_cauchy_stress(X1c, Y.copy(), dx, dy, 1.0, 0.0, phi, w_cut=2 * dx,
                                         detg_clamp=3.0)
    stress = {f"{k}_{n}": v for k, tup in out.items() for n, v in zip(("sxx", "sxy", "syy", "J"), tup)}
    # extrapolation: linear map (exactness) and deformed map, 3 layers
    solid = (phi < 0).astype(float)
    L1 = (1.3 * X + 0.2 * Y) * solid; L2 = (-0.4 * X + 0.9 * Y) * solid
    L1e, L2e = F.extrapolate_reference_map(L1, L2, phi, dx, dy, 3)
    D1e, D2e = F.extrapolate_reference_map(X1 * solid, X2 * solid, phi, dx, dy, 3)
    # velocity rhs + RK4 momentum on random smooth velocity with free-slip BC
    a = 0.3 * np.sin(2 * np.pi * X) * np.cos(np.pi * Y) + 0.01 * rng.standard_normal((N, N))
    b = -0.2 * np.cos(np.pi * X) * np.sin(2 * np.pi * Y) + 0.01 * rng.standard_normal((N, N))
    p = 0.1 * np.cos(np.pi * X) * np.cos(np.pi * Y)
    mom_fs = F.momentum_step_rk4(a, b, p, X1, X2, C.free_slip_box_bc, 0.7, 0.3, 0.02, dx, dy, 2e-3,
                                 1.0, 1.0, phi, 0.01, 2 * dx, 0.0)
    lid = lambda u, v: C.no_slip_lid_bc(u, v, 1.0)
    mom_band = F.momentum_step_rk4(a, b, p, X1, X2, lid, 0.7, 0.3, 0.0, dx, dy, 2e-3,
                                   1.0, 1.0, phi, 0.01, 2 * dx, 0.0, stress_band=True, detg_clamp=3.0)
    H = F.smoothed_heaviside(phi, 2 * dx)
    rho = (1 - H) * 1.0 + H * 1.0
    eig = F._precompute_poisson_eigenvalues(N, N, dx, dy)
    dct = F._solve_poisson_dct(a, eig)
    proj = F.pressure_projection_amg(a, b, dx, dy, 2e-3, rho, lid, p_prev=p, eigenvalues=eig)
    proj_nop = F.pressure_projection_amg(a, b, dx, dy, 2e-3, 1.0, lid, p_prev=None, eigenvalues=eig)
    rc = F._compute_divergence_rc(a, b, p, 2e-3, rho, dx, dy)
    gp = F._compute_pressure_gradient(p, dx, dy)
    # periodic branch (tests only in the reference)
    eigp = F._precompute_poisson_eigenvalues_periodic(N, N, dx, dy)
    ap = a.copy(); bp = b.copy()
    ap[:, -1] = ap[:, 0]; bp[:, -1] = bp[:, 0]; ap[-1, :] = ap[0, :]; bp[-1, :] = bp[0, :]
    per_bc = lambda u, v: (u.copy(), v.copy())
    proj_per = F.pressure_projection_amg(ap, bp, dx, dy, 2e-3, 1.0, per_bc, p_prev=p,
                                         eigenvalues=eigp, bc_type='periodic')
    # timestep variants
    dts = np.array([
        F.compute_timestep(a, b, dx, dy, 0.2, 1e-3, 0.1, 1.0, 0.0, 1.0, mu_f=0.01, eta_s=0.01),
        F.compute_timestep(a, b, dx, dy, 0.2, 1e-2, 0.0, 0.0, 0.0, 1.0, mu_f=1e-3),
        F.compute_timestep(a, b, dx, dy, 0.2, 1e-4, 1.0, 1.0, 0.0, 1.0, mu_f=1e-3, kappa=2.0),
        F.compute_timestep(a, b, dx, dy, 0.3, 1.0, 1.0, 2.0, 0.05, 1.0, mu_f=1e-3, eta_s=0.1),
    ])
    # energies
    ke = O.compute_kinetic_energy(a, b, 1.0, 1.0, phi, 2 * dx, dx, dy)
    se = O.compute_strain_energy(X1, X2, phi, 0.7, dx, dy, kappa=0.3)
    ed = O.compute_viscous_dissipation(a, b, 0.01, phi, 2 * dx, dx, dy, eta_s=0.02)
    save("operators", N=N, dx=dx, dy=dy, phi=phi, X1=X1, X2=X2, a=a, b=b, p=p, **stress,
         L1e=L1e, L2e=L2e, D1e=D1e, D2e=D2e,
         mfs_u=mom_fs[0], mfs_v=mom_fs[1], mfs_J=mom_fs[5],
         mband_u=mom_band[0], mband_v=mom_band[1], mband_J=mom_band[5],
         dct=dct, proj_a=proj[0], proj_b=proj[1], proj_p=proj[2],
         projn_a=proj_nop[0], projn_b=proj_nop[1], projn_p=proj_nop[2],
         rc=rc, gpx=gp[0], gpy=gp[1], ap=ap, bp=bp,
         per_a=proj_per[0], per_b=proj_per[1], per_p=proj_per[2],
         dts=dts, ke=ke, se=se, ed=ed)


# ── 3b. velocity_rhs_blended_optimized standalone (pyRMT/__init__.py:16 export) ────
def gen_vrhs():
    """functions.py:897-944 on the operator-case inputs: blended stress with a non-trivial
    density (rho_s = 2), surface-tension force as the scalar 0.0 (the momentum path) and as
    arrays."""
    rng = np.random.default_rng(7)
    N = 49
    X, Y, dx, dy = F.create_grid(N, N, 1.0, 1.0)
    phi = np.sqrt((X - 0.5) ** 2 + (Y - 0.5) ** 2) - 0.25
    X1 = X + 0.05 * np.sin(2 * np.pi * Y) * np.cos(np.pi * X)
    X2 = Y - 0.04 * np.sin(np.pi * X) * np.sin(2 * np.pi * Y)
    sxx, sxy, syy, _ = F.solid_cauchy_stress(X1, X2, dx, dy, 0.7, 0.3, phi)
    u = 0.3 * np.sin(2 * np.pi * X) * np.cos(np.pi * Y) + 0.01 * rng.standard_normal((N, N))
    v = -0.2 * np.cos(np.pi * X) * np.sin(2 * np.pi * Y) + 0.01 * rng.standard_normal((N, N))
    p = 0.1 * np.cos(np.pi * X) * np.cos(np.pi * Y)
    H = F.smoothed_heaviside(phi, 2 * dx)
    rho = (1 - H) * 2.0 + H * 1.0
    dHx = np.gradient(H, dx, axis=1); dHy = np.gradient(H, dy, axis=0)
    fx = 0.05 * rng.standard_normal((N, N)); fy = 0.05 * rng.standard_normal((N, N))
    r0 = F.velocity_rhs_blended_optimized(u, v, p, sxx, sxy, syy, dx, dy, phi, 0.01, H, dHx, dHy,
                                          rho, 0.0, 0.0)
    r1 = F.velocity_rhs_blended_optimized(u, v, p, sxx, sxy, syy, dx, dy, phi, 0.01, H, dHx, dHy,
                                          rho, fx, fy)
    save("vrhs", N=N, dx=dx, dy=dy, phi=phi, u=u, v=v, p=p, sxx=sxx, sxy=sxy, syy=syy, H=H,
         rho=rho, fx=fx, fy=fy, ru0=r0[0], rv0=r0[1], ru1=r1[0], rv1=r1[1])


# ── 4. WENO5 (config 3) ─────────────────────────────────────────────────────────
def gen_weno():
    rng = np.random.default_rng(7)
    N = 24
    X, Y, dx, dy = F.create_grid(N, N, 1.0, 1.0)
    q = np.sin(3 * X) + 0.1 * rng.standard_normal((N, N))
    a = rng.standard_normal((N, N)); b = rng.standard_normal((N, N))
    a[rng.random((N, N)) < 0.1] = 0.0
    phi = -np.ones((N, N))                      # every cell active: hits edge fallbacks
    phi[rng.random((N, N)) < 0.2] = 1.0
    rhs = F._weno5_rhs(q, a, b, dx, dy, phi, 0.0)
    qn = F.advect_weno5_rk3(q, a, b, dx, dy, 1e-3, phi, 0.0)
    save("weno", N=N, dx=dx, dy=dy, q=q, a=a, b=b, phi=phi, rhs=rhs, qn=qn)


def disc_tg_loop(N, nsteps, scheme='weno5'):
    """Restates benchmarks/disc_in_taylor_green.py:161-245 by calling the reference
    operators in the driver's order."""
    X, Y, dx, dy = F.create_grid(N, N, 1.0, 1.0)
    x0, y0, R = 0.5, 0.5, 0.2
    phi_init = lambda Xq, Yq: C.initialize_disc(Xq, Yq, x0, y0, R)
    phi = F.apply_phi_BCs(phi_init(X, Y))
    solid_mask = (phi <= 0).astype(float)
    mu_s, kappa, rho_s, eta_s = 1.0, 0.0, 1.0, 0.0
    mu_f, rho_f = 1.0e-3, 1.0
    w_t = 2.0 * dx
    num_layers = max(3, C.check_narrow_band(w_t, dx, 3))
    X1 = X * solid_mask; X2 = Y * solid_mask
    X1, X2 = F.extrapolate_reference_map(X1, X2, phi, dx, dy, num_layers)
    a, b = C.taylor_green_velocity(X, Y, U0=0.05)
    a, b = C.free_slip_box_bc(a, b)
    p = np.zeros((N, N))
    CFL, cap = 0.2, 1e-4
    eig = F._precompute_poisson_eigenvalues(N, N, dx, dy)
    hist = []; t = 0.0; integ = 0.0
    for step in range(1, nsteps + 1):
        dt = F.compute_timestep(a, b, dx, dy, CFL, cap, mu_s, rho_s, 0.0, rho_f,
                                mu_f=mu_f, eta_s=eta_s, kappa=kappa)
        phi = F.rebuild_phi_from_reference_map(X1, X2, phi_init)
        solid_mask = (phi <= 0).astype(float)
        X1 = F.advect_reference_map(X1, a, b, X, Y, dt, dx, dy, phi, scheme, 0.0) * solid_mask
        X2 = F.advect_reference_map(X2, a, b, X, Y, dt, dx, dy, phi, scheme, 0.0) * solid_mask
        X1, X2 = F.extrapolate_reference_map(X1, X2, phi, dx, dy, num_layers)
        phi = F.rebuild_phi_from_reference_map(X1, X2, phi_init)
        a_star, b_star, sxx, sxy, syy, J = F.momentum_step_rk4(
            a, b, p, X1, X2, C.free_slip_box_bc, mu_s, kappa, eta_s, dx, dy, dt,
            rho_s, rho_f, phi, mu_f, w_t, gamma=0.0, stress_band=False)
        H = F.smoothed_heaviside(phi, w_t)
        rho_local = (1 - H) * rho_s + H * rho_f
        a, b, p, _, _ = F.pressure_projection_amg(
            a_star, b_star, dx, dy, dt, rho_local, velocity_bc=C.free_slip_box_bc,
            p_prev=p, eigenvalues=eig, bc_type='neumann')
        ke = O.compute_kinetic_energy(a, b, rho_f, rho_s, phi, w_t, dx, dy)
        se = O.compute_strain_energy(X1, X2, phi, mu_s, dx, dy, kappa=kappa)
        diss = O.compute_viscous_dissipation(a, b, mu_f, phi, w_t, dx, dy, eta_s)
        integ += diss * dt
        ys = Y[(phi <= 0)]
        ry = 0.5 * (ys.max() - ys.min()) if ys.size else np.nan
        t += dt
        hist.append((t, ke, se, diss, integ, ke + se + integ, ry, J.min()))
    return np.array(hist), dict(a=a, b=b, p=p, X1=X1, X2=X2, phi=phi)


def gen_disc_tg():
    N, nsteps = 64, 10
    t0 = time.time()
    hist, fin = disc_tg_loop(N, nsteps)
    print(f"  disc TG N={N}: {nsteps} steps in {time.time()-t0:.1f}s; "
          f"E drift {(hist[-1,5]-hist[0,5])/hist[0,5]:.3e}")
    save("disc_tg_trace", N=N, hist=hist, **fin)


# ── 5. Pure-fluid lid-driven cavity (config 1) ──────────────────────────────────
def lid_cavity_loop(Re, N, max_steps, steady_tol=2e-5, upwind=None):
    """Restates benchmarks/lid_driven_cavity.py:26-97."""
    if upwind is not None:
        F.diff_upwind_3rd = upwind
    X, Y, dx, dy = F.create_grid(N, N, 1.0, 1.0)
    mu_f = 1.0 * 1.0 * 1.0 / Re
    rho_f = 1.0
    mu_s = kappa = rho_s = eta_s = 0.0
    w_t = 2.0 * dx
    phi = np.ones((N, N))
    X1, X2 = X.copy(), Y.copy()
    a = np.zeros((N, N)); b = np.zeros((N, N)); p = np.zeros((N, N))
    a, b = C.no_slip_lid_bc(a, b, 1.0)
    eig = F._precompute_poisson_eigenvalues(N, N, dx, dy)
    bc = lambda u, v: C.no_slip_lid_bc(u, v, 1.0)
    res_hist = []
    steps_done = 0
    for step in range(1, max_steps + 1):
        dt = F.compute_timestep(a, b, dx, dy, 0.2, 1e-2, mu_s, rho_s, 0.0, rho_f, mu_f=mu_f)
        a_prev = a
        a_star, b_star, *_ = F.momentum_step_rk4(
            a, b, p, X1, X2, bc, mu_s, kappa, eta_s, dx, dy, dt,
            rho_s, rho_f, phi, mu_f, w_t, 0.0)
        a, b, p, _, _ = F.pressure_projection_amg(
            a_star, b_star, dx, dy, dt, rho_f, velocity_bc=bc,
            p_prev=p, eigenvalues=eig, bc_type='neumann')
        steps_done = step
        if step % 200 == 0 or step == 1:
            res = np.max(np.abs(a - a_prev)) / dt
            res_hist.append((step, res))
            if step > 1 and res < steady_tol:
                break
    y, u_line, x, v_line = C.extract_centerlines(a, b, X, Y)
    gd = np.loadtxt(os.path.join(REF, "data", f"plot_u_y_Ghia{int(Re)}.csv"), delimiter=",", skiprows=1)
    err = float(np.sqrt(np.mean((np.interp(gd[:, 0], y, u_line) - gd[:, 1]) ** 2)))
    return err, steps_done, dict(a=a, b=b, p=p), np.array(res_hist)


def gen_lid_cavity_short():
    N, nsteps = 129, 40
    t0 = time.time()
    _, _, fin, _ = lid_cavity_loop(1000.0, N, nsteps)
    print(f"  lid cavity Re=1000 N={N}: {nsteps} steps in {time.time()-t0:.1f}s")
    save("lid_cavity_short", N=N, Re=1000.0, nsteps=nsteps, **fin)
    for Re in (100, 1000):
        gd = np.loadtxt(os.path.join(REF, "data", f"plot_u_y_Ghia{Re}.csv"), delimiter=",", skiprows=1)
        save(f"ghia{Re}_data", y=gd[:, 0], u=gd[:, 1])


def _upwind_vectorised(f, u, h, axis):
    """Bit-identical vectorised restatement of utils.diff_upwind_3rd (asserted below),
    used only to make the 36k-step Ghia run affordable in pure Python."""
    if axis == 0:
        return _upwind_vectorised(f.T, u.T, h, 1).T
    df = np.zeros_like(f)
    Nx = f.shape[1]
    v = u[:, 2:Nx - 2]
    pos = (2 * f[:, 3:Nx - 1] + 3 * f[:, 2:Nx - 2] - 6 * f[:, 1:Nx - 3] + f[:, 0:Nx - 4]) / (6 * h)
    neg = (-f[:, 4:Nx] + 6 * f[:, 3:Nx - 1] - 3 * f[:, 2:Nx - 2] - 2 * f[:, 1:Nx - 3]) / (6 * h)
    df[:, 2:Nx - 2] = np.where(v > 0, pos, neg)
    for i in (0, 1, Nx - 2, Nx - 1):
        vel = u[:, i]
        bwd = (f[:, i] - f[:, i - 1]) / h if i > 0 else None
        fwd = (f[:, i + 1] - f[:, i]) / h if i < Nx - 1 else None
        if i == 0:
            df[:, i] = fwd
        elif i == Nx - 1:
            df[:, i] = bwd
        else:
            df[:, i] = np.where(vel > 0, bwd, fwd)
    return df


def gen_ghia():
    rng = np.random.default_rng(5)
    import pyRMT.utils as Uref
    ref_upwind = Uref.diff_upwind_3rd
    for shape in ((17, 23), (33, 33)):
        f = rng.standard_normal(shape); u = rng.standard_normal(shape)
        u[rng.random(shape) < 0.2] = 0.0
        for ax in (0, 1):
            assert np.array_equal(ref_upwind(f, u, 0.1, ax), _upwind_vectorised(f, u, 0.1, ax))
    res = {}
    for Re in (100.0, 1000.0):
        t0 = time.time()
        err, steps, fin, rh = lid_cavity_loop(Re, 129, 60000, upwind=_upwind_vectorised)
        print(f"  Ghia Re={Re:.0f}: RMS={err!r} steady at step {steps} ({time.time()-t0:.0f}s)")
        res[f"Re{int(Re)}_rms"] = err
        res[f"Re{int(Re)}_steps"] = steps
        res[f"Re{int(Re)}_res"] = rh
        res[f"Re{int(Re)}_a"] = fin["a"]
        res[f"Re{int(Re)}_b"] = fin["b"]
    F.diff_upwind_3rd = ref_upwind
    save("ghia_pinned", **res)


# ── 6. MAC path (config 5) ──────────────────────────────────────────────────────
def gen_mac():
    rng = np.random.default_rng(11)
    N = 32
    dx, dy = M.mac_grid(N, N)
    u = 0.1 * rng.standard_normal((N, N + 1)); v = 0.1 * rng.standard_normal((N + 1, N))
    u[:, 0] = u[:, -1] = 0.0; v[0, :] = v[-1, :] = 0.0
    fu = rng.standard_normal((N, N + 1)); fv = rng.standard_normal((N + 1, N))
    us, vs = M.momentum_predictor(u, v, 0.01, dx, dy, 1e-3, 1.0, fu=fu, fv=fv, rho=1.0)
    eig = M.poisson_eigs_neumann(N, N, dx, dy)
    pu, pv, pp = M.project(us, vs, dx, dy, 1e-3, 1.0, eig)
    xc = (np.arange(N) + 0.5) * dx
    Xc, Yc = np.meshgrid(xc, xc)
    pa = np.sqrt((Xc - 0.4) ** 2 + (Yc - 0.5) ** 2) - 0.15
    pb = np.sqrt((Xc - 0.65) ** 2 + (Yc - 0.5) ** 2) - 0.12
    txx, txy, tyy = M.contact_stress(pa, pb, 2.0, 0.6, 3 * dx, dx, dy)
    save("mac_ops", N=N, dx=dx, dy=dy, u=u, v=v, fu=fu, fv=fv, us=us, vs=vs,
         pu=pu, pv=pv, pp=pp, pa=pa, pb=pb, txx=txx, txy=txy, tyy=tyy)


def gen_schemes(N=41):
    """The other advection schemes behind advect_reference_map (functions.py:228-251,
    420-498; interpolators.py:64-156) on a deformed disc map."""
    rng = np.random.default_rng(77)
    X, Y, dx, dy = F.create_grid(N, N, 1.0, 1.0)
    f = rng.standard_normal((N, N))
    xq = rng.uniform(-0.2, 1.2, (N, N)); yq = rng.uniform(-0.2, 1.2, (N, N))
    xq[0, 0] = np.nan; yq[1, 1] = np.inf; xq[3, 3] = 1e200; xq[5, 5] = 1.0; yq[5, 5] = 1.0
    bic = I.bicubic_interpolate(f, xq, yq, dx, dy, N, N)
    a = 0.3 * np.sin(2 * np.pi * Y) * np.cos(np.pi * X) + 0.1
    b = -0.2 * np.cos(2 * np.pi * X) * np.sin(np.pi * Y)
    X1 = X + 0.02 * np.sin(2 * np.pi * Y); X2 = Y + 0.03 * np.sin(2 * np.pi * X)
    phi = np.sqrt((X1 - 0.5) ** 2 + (X2 - 0.5) ** 2) - 0.3
    dt = 0.2 * dx / 0.4
    out = dict(N=N, dx=dx, dy=dy, f=f, xq=xq, yq=yq, bic=bic, a=a, b=b, X1=X1, X2=X2, phi=phi,
               dt=dt)
    out["sl_cubic"] = F.advect_reference_map(X1, a, b, X, Y, dt, dx, dy, phi, 'semilagrangian_cubic')
    for name in ("central2", "conservative"):
        for wc in (0.0, 2 * dx):
            out[f"{name}_{int(wc > 0)}"] = F.advect_reference_map(X1, a, b, X, Y, dt, dx, dy, phi,
                                                                 name, wc)
    out["c2_rhs"] = F._central2_rhs(X1, a, b, dx, dy, phi, 0.0)
    out["cons_rhs"] = F._conservative_rhs(X1, a, b, dx, dy, phi, 2 * dx)
    save("schemes", **out)


def gen_periodic(N=65):
    """functions.py:1177-1290 periodic branch on tests/test_poisson.py:24-78's fields."""
    X, Y, dx, dy = F.create_grid(N, N, 1.0, 1.0)
    k = 2 * np.pi
    p_true = np.cos(k * X) * np.sin(k * Y) + 0.5 * np.sin(2 * k * X)
    gx, gy = F._compute_pressure_gradient_periodic(p_true, dx, dy)
    lap = F._compute_divergence_periodic(gx, gy, dx, dy)
    eig, null = F._precompute_poisson_eigenvalues_periodic(N, N, dx, dy)
    p = F._solve_poisson_fft(lap, (eig, null))

    def periodic_bc(u, v):
        u = u.copy(); v = v.copy()
        u[:, -1] = u[:, 0]; v[:, -1] = v[:, 0]
        u[-1, :] = u[0, :]; v[-1, :] = v[0, :]
        return u, v
    a = np.sin(k * X) * np.cos(k * Y) + 0.3 * np.cos(k * X)
    b = -np.cos(k * X) * np.sin(k * Y) + 0.2 * np.sin(k * Y)
    a, b = periodic_bc(a, b)
    rng = np.random.default_rng(5)
    p_prev = rng.standard_normal((N, N))
    an, bn, pn, _, _ = F.pressure_projection_amg(a, b, dx, dy, 1e-2, 1.0, periodic_bc,
                                                 p_prev=p_prev, eigenvalues=(eig, null),
                                                 bc_type='periodic')
    save("periodic", N=N, dx=dx, dy=dy, p_true=p_true, gx=gx, gy=gy, lap=lap, eig=eig,
         null=null, p=p, a=a, b=b, p_prev=p_prev, an=an, bn=bn, pn=pn)


def gen_varrho(N=33):
    """functions.py:1016-1070, 1122-1168, 1296-1328: variable-density Rhie-Chow divergence,
    the matrix-free operator, and the DCT-preconditioned CG projection.  The reference calls
    scipy.sparse.linalg.cg(..., tol=1e-6, ...); scipy >= 1.14 (1.15 here) renamed tol to
    rtol, so the call is routed through a keyword shim (tol -> rtol, nothing else) and the
    iterations are counted with scipy's own callback.  scipy 1.15's LinearOperator also
    probes an untyped matvec with an int8 vector, which the reference's operator cannot
    take (it accumulates into zeros_like(p)); the shim passes dtype=float64, as older scipy
    inferred."""
    import scipy.sparse.linalg as sla
    X, Y, dx, dy = F.create_grid(N, N, 1.0, 1.0)
    rng = np.random.default_rng(21)
    phi = np.sqrt((X - 0.5) ** 2 + (Y - 0.45) ** 2) - 0.25
    H = F.smoothed_heaviside(phi, 2 * dx)
    rho = (1 - H) * 4.0 + H * 1.0
    p = rng.standard_normal((N, N))
    Ap = F._apply_variable_poisson(p.ravel(), N, N, dx, dy, 1.0 / rho)
    k = 2 * np.pi
    a = 0.5 * np.sin(k * X) * np.cos(k * Y) + 0.1 * rng.standard_normal((N, N))
    b = -0.5 * np.cos(k * X) * np.sin(k * Y) + 0.1 * rng.standard_normal((N, N))
    p_prev = 0.1 * rng.standard_normal((N, N))
    dt = 1e-3
    divU = F._compute_divergence_rc(a, b, p_prev, dt, rho, dx, dy)
    eig = F._precompute_poisson_eigenvalues(N, N, dx, dy)
    iters = []

    def cg_compat(A, rhs, x0=None, tol=1e-5, maxiter=None, M=None):
        n = [0]
        x, info = sla.cg(A, rhs, x0=x0, rtol=tol, maxiter=maxiter, M=M,
                         callback=lambda xk: n.__setitem__(0, n[0] + 1))
        iters.append(n[0])
        return x, info
    cg_ref, lo_ref = F.cg, F.LinearOperator
    F.cg = cg_compat
    F.LinearOperator = lambda shape, matvec: sla.LinearOperator(shape, matvec=matvec,
                                                                dtype=np.float64)
    try:
        an, bn, pn, _, _ = F.pressure_projection_amg(a, b, dx, dy, dt, rho, C.free_slip_box_bc,
                                                     p_prev=p_prev, eigenvalues=eig)
    finally:
        F.cg, F.LinearOperator = cg_ref, lo_ref
    save("varrho", N=N, dx=dx, dy=dy, rho=rho, p=p, Ap=Ap, a=a, b=b, p_prev=p_prev, dt=dt,
         divU=divU, eig=eig, an=an, bn=bn, pn=pn, iters=iters[0])


def gen_mac_trace(N=64, nsteps=8, n_discs=3, seed=3):
    """Config 5 loop body (benchmarks/mac_multi_disc_lid.py:36-98) with the reference's
    own functions, no I/O: per-step centroids / J range and the final state."""
    import importlib
    drv = importlib.import_module("benchmarks.mac_multi_disc_lid")
    U_lid, mu_s, mu_f, rho, eta = 1.0, 0.3, 0.01, 1.0, 2.0
    dx, dy = M.mac_grid(N, N)
    xc = (np.arange(N) + 0.5) * dx
    Xc, Yc = np.meshgrid(xc, xc)
    Xg, Yg = np.meshgrid(np.arange(N) * dx, np.arange(N) * dy)
    w_t = 2.0 * dx; nu = mu_f / rho; eps = 3.0 * dx
    specs = drv._place_discs(n_discs, seed)
    inits = [(lambda X, Y, cx=cx, cy=cy, R=R: np.sqrt((X-cx)**2 + (Y-cy)**2) - R)
             for (R, cx, cy) in specs]
    refs = []
    for pin in inits:
        phi = pin(Xc, Yc); m = (phi <= 0).astype(float)
        refs.append(list(F.extrapolate_reference_map(Xc * m, Yc * m, phi, dx, dy, 3)))
    init_refs = [[a.copy() for a in r] for r in refs]
    u = np.zeros((N, N + 1)); v = np.zeros((N + 1, N))
    eig = M.poisson_eigs_neumann(N, N, dx, dy)
    cs = np.sqrt(mu_s / rho)
    dt = min(0.3 * dx / U_lid, 0.2 * dx * dx / nu, 0.3 * dx / (cs + 1e-9))
    rec = {k: [] for k in ("cx", "cy", "minJ", "maxJ")}
    for _ in range(nsteps):
        u_c = 0.5 * (u[:, :-1] + u[:, 1:]); v_c = 0.5 * (v[:-1, :] + v[1:, :])
        phis = []
        for k, pin in enumerate(inits):
            X1, X2 = refs[k]
            phi = F.rebuild_phi_from_reference_map(X1, X2, pin); m = (phi <= 0).astype(float)
            X1 = F.advect_reference_map(X1, u_c, v_c, Xg, Yg, dt, dx, dy, phi, 'semilagrangian', 0.0) * m
            X2 = F.advect_reference_map(X2, u_c, v_c, Xg, Yg, dt, dx, dy, phi, 'semilagrangian', 0.0) * m
            X1, X2 = F.extrapolate_reference_map(X1, X2, phi, dx, dy, 3)
            refs[k] = [X1, X2]
            phis.append(F.rebuild_phi_from_reference_map(X1, X2, pin))
        Sxx = np.zeros((N, N)); Sxy = np.zeros((N, N)); Syy = np.zeros((N, N))
        Jmin = 1.0; Jmax = 1.0
        for k in range(len(refs)):
            sxx, sxy, syy, J = F.solid_cauchy_stress(refs[k][0], refs[k][1], dx, dy, mu_s, 0.0, phis[k])
            H = F.smoothed_heaviside(phis[k], w_t)
            Sxx += (1 - H) * sxx; Sxy += (1 - H) * sxy; Syy += (1 - H) * syy
            Jmin = min(Jmin, J.min()); Jmax = max(Jmax, J.max())
        for i in range(len(phis)):
            for j in range(i + 1, len(phis)):
                txx, txy, tyy = M.contact_stress(phis[i], phis[j], eta, 2 * mu_s, eps, dx, dy)
                Sxx += txx; Sxy += txy; Syy += tyy
        divx = U.grad_central_x_2nd(Sxx, dx) + U.grad_central_y_2nd(Sxy, dy)
        divy = U.grad_central_x_2nd(Sxy, dx) + U.grad_central_y_2nd(Syy, dy)
        fu = np.zeros((N, N + 1)); fu[:, 1:-1] = 0.5 * (divx[:, 1:] + divx[:, :-1])
        fv = np.zeros((N + 1, N)); fv[1:-1, :] = 0.5 * (divy[1:, :] + divy[:-1, :])
        ustar, vstar = M.momentum_predictor(u, v, nu, dx, dy, dt, U_lid, fu=fu, fv=fv, rho=rho)
        u, v, p = M.project(ustar, vstar, dx, dy, dt, rho, eig)
        cents = [(Xc[pp <= 0].mean(), Yc[pp <= 0].mean()) for pp in phis]
        rec["cx"].append([c[0] for c in cents]); rec["cy"].append([c[1] for c in cents])
        rec["minJ"].append(Jmin); rec["maxJ"].append(Jmax)
    save("mac_trace", N=N, nsteps=nsteps, specs=np.array(specs), dt=dt, u=u, v=v, p=p,
         X1_0=init_refs[0][0], X2_0=init_refs[0][1],
         **{f"X{c}_{k}_end": refs[k][c - 1] for k in range(len(refs)) for c in (1, 2)},
         **{f"phi_{k}": phis[k] for k in range(len(phis))},
         Sxx=Sxx, Sxy=Sxy, Syy=Syy, fu=fu, fv=fv, ustar=ustar, vstar=vstar,
         **{k: np.array(val) for k, val in rec.items()})


def gen_imex(N=32):
    """mac.py:243-369 (the MAC IMEX tier): the homogeneous-BC ghost-cell
    Laplacians, the DST-II Helmholtz eigenvalues, CG and DST-preconditioned CG Helmholtz
    solves (with scipy's own callback counting the PCG iterations, as the reference's
    `count`), and momentum_predictor_lid_imex with and without forces / the trapezoidal
    elastic term, on seeded lid-cavity-like fields."""
    rng = np.random.default_rng(77)
    dx, dy = M.mac_grid(N, N)
    u = 0.3 * rng.standard_normal((N, N + 1)); u[:, 0] = 0.0; u[:, -1] = 0.0
    v = 0.3 * rng.standard_normal((N + 1, N)); v[0, :] = 0.0; v[-1, :] = 0.0
    lap_u = M._lap_u_lid_hom(u, dx, dy)
    lap_v = M._lap_v_lid_hom(v, dx, dy)
    eig_u = M._dst_helmholtz_eigs((N, N - 1), dx, dy)
    eig_v = M._dst_helmholtz_eigs((N - 1, N), dx, dy)
    rhs_u = rng.standard_normal((N, N - 1))
    rhs_v = rng.standard_normal((N - 1, N))
    emb_u = lambda x: np.pad(x, ((0, 0), (1, 1)))
    emb_v = lambda x: np.pad(x, ((1, 1), (0, 0)))
    lu = lambda w: M._lap_u_lid_hom(w, dx, dy)
    lv = lambda w: M._lap_v_lid_hom(w, dx, dy)
    coef = 0.5e-3
    cg_u = M._cg_helmholtz(rhs_u, lu, emb_u, coef)
    cnt_u, cnt_v = [], []
    pcg_u = M._pcg_helmholtz(rhs_u, lu, emb_u, coef, dx, dy, rtol=1e-8, count=cnt_u)
    pcg_v = M._pcg_helmholtz(rhs_v, lv, emb_v, coef, dx, dy, rtol=1e-8, count=cnt_v)
    nu, dt, U_lid = 0.01, 2e-3, 1.0
    us0, vs0 = M.momentum_predictor_lid_imex(u, v, nu, dx, dy, dt, U_lid)
    fu = 0.1 * rng.standard_normal((N, N + 1)); fv = 0.1 * rng.standard_normal((N + 1, N))
    us1, vs1 = M.momentum_predictor_lid_imex(u, v, nu, dx, dy, dt, U_lid, fu=fu, fv=fv,
                                             rho=1.3, cs2=4.0)
    # the semi-Lagrangian branch (CFL > 0.9 at this dt), with forces and the elastic term
    dts = 0.05
    sl0 = M.momentum_predictor_lid_semilag(u, v, nu, dx, dy, dts, U_lid)
    sl1 = M.momentum_predictor_lid_semilag(u, v, nu, dx, dy, dts, U_lid, fu=fu, fv=fv, rho=1.3,
                                           cs2=4.0)
    save("imex_sl", N=N, dx=dx, dy=dy, u=u, v=v, nu=nu, dt=dts, U_lid=U_lid, fu=fu, fv=fv,
         us0=sl0[0], vs0=sl0[1], us1=sl1[0], vs1=sl1[1])
    save("imex", N=N, dx=dx, dy=dy, u=u, v=v, lap_u=lap_u, lap_v=lap_v, eig_u=eig_u,
         eig_v=eig_v, rhs_u=rhs_u, rhs_v=rhs_v, coef=coef, cg_u=cg_u, pcg_u=pcg_u, pcg_v=pcg_v,
         cnt_u=cnt_u[0], cnt_v=cnt_v[0], nu=nu, dt=dt, U_lid=U_lid, us0=us0, vs0=vs0, fu=fu,
         fv=fv, us1=us1, vs1=vs1)


# ── 11. output.py:213-321 output_simulation_data (HDF5 writer recorded, not written) ─
def gen_output(N=33):
    """The reference's writer on a synthetic deformed-disc state; h5py is replaced by a
    recorder of its datasets / attrs (h5py is absent here), the CSV and the log line are
    kept as text."""
    import contextlib
    import io
    rng = np.random.default_rng(11)
    X, Y, dx, dy = F.create_grid(N, N, 1.0, 1.0)
    X1 = X + 0.02 * np.sin(2 * np.pi * Y); X2 = Y + 0.015 * np.sin(2 * np.pi * X)
    phi = np.sqrt((X1 - 0.5) ** 2 + (X2 - 0.5) ** 2) - 0.25
    solid = (phi <= 0).astype(float)
    k = 2 * np.pi
    a = 0.05 * np.sin(k * X) * np.cos(k * Y) + 0.01 * rng.standard_normal((N, N))
    b = -0.05 * np.cos(k * X) * np.sin(k * Y) + 0.01 * rng.standard_normal((N, N))
    p = rng.standard_normal((N, N))
    sxx, sxy, syy, J = (rng.standard_normal((N, N)) for _ in range(4))
    rec = {}

    class _File:
        def __init__(self, path, mode):
            self.path = os.path.basename(path); self.ds = {}; self.attrs = {}
        def __enter__(self):
            return self
        def __exit__(self, *a):
            rec[self.path] = (self.ds, self.attrs)
        def create_dataset(self, name, data):
            self.ds[name] = np.array(data)
    O.h5py = types.SimpleNamespace(File=_File)
    kw = dict(mu_s=0.7, mu_f=1e-3, rho_s=1.0, rho_f=1.0, w_t=2 * dx, eta_s=0.02, kappa=0.3,
              time=0.125, integrated_dissipation=3.5e-4)
    cwd = os.getcwd()
    tmp = tempfile.mkdtemp(prefix="rmt_out_")
    os.chdir(tmp)
    try:
        log = io.StringIO()
        with contextlib.redirect_stdout(log):
            ret = O.output_simulation_data(dx, dy, phi, solid, X1, X2, a, b, p, 5, "case", 1, 2.5e-3,
                                           sxx, sxy, syy, J, **kw)
            O.output_simulation_data(dx, dy, phi, solid, X1, X2, a, b, p, 5, "case", 7, 2.5e-3,
                                     sxx, sxy, syy, J, **kw)   # not an output step
            O.output_simulation_data(dx, dy, phi, solid, X1, X2, a, b, p, 5, "case", 10, 2.5e-3,
                                     sxx, sxy, syy, J, **kw)
        csv_text = open(os.path.join("outputs", "case", "energy_history.csv")).read()
    finally:
        os.chdir(cwd)
    ds, at = rec["data_000001.h5"]
    assert set(rec) == {"data_000001.h5", "data_000010.h5"}
    save("output_sim", N=N, dx=dx, dy=dy, phi=phi, solid=solid, X1=X1, X2=X2, a=a, b=b, p=p,
         sxx=sxx, sxy=sxy, syy=syy, J=J, ret=ret, csv=csv_text, log=log.getvalue(),
         **{"kw_" + k: v for k, v in kw.items()},
         **{"ds_" + k: v for k, v in ds.items()}, **{"at_" + k: v for k, v in at.items()})


if __name__ == "__main__":
    if "--only" in sys.argv:     # regenerate the named fixtures only
        for name in sys.argv[sys.argv.index("--only") + 1:]:
            globals()[f"gen_{name}"]()
        sys.exit(0)
    t0 = time.time()
    gen_primitives()
    gen_operator_cases()
    gen_vrhs()
    gen_weno()
    gen_mac()
    gen_soft_disc_driver_check()
    gen_soft_disc()
    gen_disc_tg()
    gen_lid_cavity_short()
    if "--ghia" in sys.argv:
        gen_ghia()
    print(f"done in {time.time()-t0:.0f}s")
