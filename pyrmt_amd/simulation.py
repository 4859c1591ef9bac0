"""Device-resident RMT time stepping: the loop bodies of the reference drivers.

The reference has no step() function; every benchmark hand-rolls the same loop
(docs/REFACTORING.md:55-57).  `Simulation` runs that loop body on the GPU through
rmt_sim_* (include/rmt.h), keeping (u, v, p, X1, X2) in HBM; the driver functions
below set up the three configurations exactly as the reference scripts do:
  soft_disc_in_lid_driven   benchmarks/soft_disc_in_lid_driven.py:165-235 (configs 2, 4)
  disc_in_taylor_green      benchmarks/disc_in_taylor_green.py:161-245   (config 3)
  lid_driven_cavity         benchmarks/lid_driven_cavity.py:26-97        (config 1)
"""
import ctypes
import math
import weakref

import numpy as np

from . import _lib as L
from . import functions as F
from .bc import NOSLIP_LID, FREESLIP_BOX

FIELDS = {"u": 0, "a": 0, "v": 1, "b": 1, "p": 2, "X1": 3, "X2": 4, "phi": 5, "J": 6,
          "sigma_xx": 7, "sigma_xy": 8, "sigma_yy": 9}
SCHEMES = {"semilagrangian": 0, "weno5": 1, "central2": 2, "conservative": 3,
           "semilagrangian_cubic": 4}


class Simulation:
    def __init__(self, N, *, scheme="semilagrangian", bc_kind=NOSLIP_LID, lid=1.0, disc=None,
                 mu_s=0.0, kappa=0.0, rho_s=1.0, eta_s=0.0, mu_f=0.01, rho_f=1.0, w_t=None,
                 layers=3, cfl=0.2, dt_cap=1e-3, stress_band=False, detg_clamp=3.0,
                 energies=False, options=None):
        if scheme not in SCHEMES:
            raise ValueError(f"Unknown advection scheme {scheme!r}")
        torch = F._torch()
        self.torch = torch
        self.N = N
        self.X, self.Y, self.dx, self.dy = F.create_grid(N, N, 1.0, 1.0)
        self.xs = np.ascontiguousarray(self.X[0, :]); self.ys = np.ascontiguousarray(self.Y[:, 0])
        self.disc = disc
        w_t = 2.0 * self.dx if w_t is None else w_t
        if options:
            # a context of its own with these implementation switches (rmt_ctx_set_option)
            self.ctx = F._Ctx(N, N, torch.cuda.current_device())
            for k, v in options.items():
                self.ctx.set_option(k, v)
        else:
            self.ctx = F.ctx_for(N, N)
        P = L.rmt_sim_params()
        P.ny = P.nx = N; P.dx = self.dx; P.dy = self.dy
        P.xs = self.xs.ctypes.data; P.ys = self.ys.ctypes.data
        P.scheme = SCHEMES[scheme]; P.bc_kind = bc_kind; P.lid = lid
        P.shape = 1 if disc is not None else 0
        if disc is not None:
            P.x0, P.y0, P.R = disc
        P.mu_s, P.kappa, P.rho_s, P.eta_s, P.mu_f, P.rho_f = mu_s, kappa, rho_s, eta_s, mu_f, rho_f
        P.w_t = w_t; P.layers = layers; P.cfl = cfl; P.dt_cap = dt_cap
        P.stress_band = int(bool(stress_band)); P.detg_clamp = detg_clamp
        P.energies = int(bool(energies))
        self.params = P
        h = ctypes.c_void_p()
        L.check(L.lib().rmt_sim_create(self.ctx.bind(), ctypes.byref(P), ctypes.byref(h)),
                "rmt_sim_create")
        self.h = h
        self._views = {}
        self._lent = []   # weak references to the views field() handed out
        # carry the last step's prepared state into the next step() call (rmt_sim_set_carry);
        # every write path below (field views, set_field) invalidates it, and so does step()
        # while a view handed out by field() is alive (it may have been written through)
        L.check(L.lib().rmt_sim_set_carry(self.h, 1), "rmt_sim_set_carry")

    def __del__(self):
        try:
            L.lib().rmt_sim_destroy(self.h)
        except Exception:
            pass

    def _view(self, name):
        fid = FIELDS[name]
        if fid not in self._views:
            ptr = ctypes.c_void_p()
            L.check(L.lib().rmt_sim_field(self.h, fid, ctypes.byref(ptr)))
            self._views[fid] = _wrap_device(self.torch, ptr.value, (self.N, self.N))
        return self._views[fid]

    def field(self, name):
        """A torch CUDA view (no copy) of a state field: u/a, v/b, p, X1, X2, phi, J.  The
        caller may write through it -- or through any view derived from it (a slice, .T,
        .view) -- at any time: while any tensor on its storage is alive, every step() starts
        from the fields as they are (the carried state of the previous call is dropped)."""
        self.invalidate()
        fid = FIELDS[name]
        ptr = ctypes.c_void_p()
        L.check(L.lib().rmt_sim_field(self.h, fid, ctypes.byref(ptr)))
        return _wrap_device(self.torch, ptr.value, (self.N, self.N), lent=self._lent)

    def invalidate(self):
        """The state was changed from outside: the next step() recomputes everything it
        derives from it (rmt_sim_invalidate)."""
        L.check(L.lib().rmt_sim_invalidate(self.h), "rmt_sim_invalidate")

    def set_field(self, name, value):
        t = self.field(name)
        t.copy_(self.torch.as_tensor(np.ascontiguousarray(value, dtype=np.float64)).to(t.device))

    def get(self, name):
        self.torch.cuda.synchronize()
        return self._view(name).cpu().numpy()

    def step(self, nsteps=1, t_end=math.inf):
        self.ctx.bind()
        if self._lent:
            self._lent = [r for r in self._lent if r() is not None]
            if self._lent:
                self.invalidate()
        L.check(L.lib().rmt_sim_step(self.h, int(nsteps), float(t_end)), "rmt_sim_step")

    PHASES = ("dt", "advect", "extrapolate", "momentum", "projection", "diagnostics",
              "rk4_stage_kernels", "extrap_sweep_kernel")

    def set_sync_every(self, k):
        """Read the device diagnostics / error flags back every k steps (1..64; default 64).
        An error is raised at the next read-back; the fields are then those of the last
        enqueued step (k = 1: the failing step's)."""
        L.check(L.lib().rmt_sim_set_sync_every(self.h, int(k)), "rmt_sim_set_sync_every")

    def set_profiling(self, on=True):
        L.check(L.lib().rmt_sim_set_profiling(self.h, int(bool(on))))

    def phase_times(self):
        """{phase: (total_ms, intervals)} from HIP events on the sim's stream."""
        ms = (ctypes.c_double * 8)(); calls = (ctypes.c_long * 8)()
        L.check(L.lib().rmt_sim_phase_times(self.h, ms, calls))
        return {k: (ms[i], calls[i]) for i, k in enumerate(self.PHASES)}

    def diagnostics(self):
        n = ctypes.c_int()
        L.check(L.lib().rmt_sim_diagnostics(self.h, None, 0, ctypes.byref(n)))
        buf = (L.rmt_diag * max(n.value, 1))()
        L.check(L.lib().rmt_sim_diagnostics(self.h, buf, n.value, ctypes.byref(n)))
        keys = [k for k, _ in L.rmt_diag._fields_]
        return {k: np.array([getattr(buf[i], k) for i in range(n.value)]) for k in keys}


class _CAI:
    """__cuda_array_interface__ exporter of a librmt buffer.  torch.as_tensor keeps a strong
    reference to it in the tensor's storage (released when the storage is freed), so a weak
    reference to it is alive exactly while any tensor on that storage is: the returned view
    and every view derived from it (slices, .T, .view, ...)."""

    def __init__(self, ptr, shape):
        self.__cuda_array_interface__ = {"shape": shape, "typestr": "<f8", "data": (ptr, False),
                                         "version": 3, "strides": None}


def _wrap_device(torch, ptr, shape, lent=None):
    """Zero-copy torch view of librmt-owned device memory (valid while the sim lives).
    lent: a list that receives a weak reference that lives as long as the view's storage."""
    cai = _CAI(ptr, shape)
    t = torch.as_tensor(cai, device="cuda")
    if lent is not None:
        lent.append(weakref.ref(cai))
    return t


def _init_disc_map(sim, x0, y0, R, layers):
    """Drivers' set-up (soft_disc_in_lid_driven.py:177-193): phi0 with apply_phi_BCs,
    xi = x * mask, then the initial narrow-band extrapolation (on the GPU)."""
    X, Y = sim.X, sim.Y
    phi = F.apply_phi_BCs(np.sqrt((X - x0) ** 2 + (Y - y0) ** 2) - R)
    m = (phi <= 0).astype(float)
    X1, X2 = F.extrapolate_reference_map(X * m, Y * m, phi, sim.dx, sim.dy, layers)
    sim.set_field("X1", X1)
    sim.set_field("X2", X2)


def soft_disc_params(N, stress_band=False, detg_clamp=3.0):
    """Configs 2 and 4 physics (soft_disc_in_lid_driven.py:165-199 parameters): neo-Hookean
    disc (0.6, 0.5, R=0.2) in the lid cavity, semi-Lagrangian map advection."""
    w_t = 2.0 * np.linspace(0, 1, N)[1]
    layers = max(3, int(np.ceil(w_t / (np.linspace(0, 1, N)[1]))) + 1)
    return dict(bc_kind=NOSLIP_LID, lid=1.0, disc=(0.6, 0.5, 0.2), mu_s=0.1, kappa=0.0,
                rho_s=1.0, eta_s=0.01, mu_f=0.01, rho_f=1.0, w_t=w_t, layers=layers, cfl=0.2,
                dt_cap=1e-3, stress_band=stress_band, detg_clamp=detg_clamp)


def initial_disc_map(N, x0, y0, R, layers):
    """The drivers' initial reference map (soft_disc_in_lid_driven.py:177-193): phi0 with
    apply_phi_BCs, xi = x * mask, then the narrow-band extrapolation (on the GPU)."""
    X, Y, dx, dy = F.create_grid(N, N, 1.0, 1.0)
    phi = F.apply_phi_BCs(np.sqrt((X - x0) ** 2 + (Y - y0) ** 2) - R)
    m = (phi <= 0).astype(float)
    return F.extrapolate_reference_map(X * m, Y * m, phi, dx, dy, layers)


def soft_disc_in_lid_driven(N=128, scheme="semilagrangian", stress_band=False, detg_clamp=3.0,
                            options=None):
    """Configs 2 and 4: neo-Hookean disc (0.6, 0.5, R=0.2) in the lid cavity
    (soft_disc_in_lid_driven.py:165-199 parameters).  options: implementation switches of a
    context of the sim's own (Simulation)."""
    kw = soft_disc_params(N, stress_band, detg_clamp)
    sim = Simulation(N, scheme=scheme, options=options, **kw)
    _init_disc_map(sim, 0.6, 0.5, 0.2, kw["layers"])
    return sim


def disc_in_taylor_green(N=128, scheme="semilagrangian", stress_band=False):
    """Config 3: disc (0.5, 0.5, 0.2) in a Taylor-Green vortex, free-slip box, with the
    per-step energies (disc_in_taylor_green.py:161-190 parameters).  The default scheme is the
    reference driver's ('semilagrangian', disc_in_taylor_green.py:39, :150); config 3 passes
    'weno5'."""
    sim0 = F.create_grid(N, N, 1.0, 1.0)
    w_t = 2.0 * sim0[2]
    layers = max(3, int(np.ceil(w_t / sim0[2])) + 1)
    sim = Simulation(N, scheme=scheme, bc_kind=FREESLIP_BOX, lid=0.0, disc=(0.5, 0.5, 0.2),
                     mu_s=1.0, kappa=0.0, rho_s=1.0, eta_s=0.0, mu_f=1.0e-3, rho_f=1.0, w_t=w_t,
                     layers=layers, cfl=0.2, dt_cap=1e-4, stress_band=stress_band, energies=True)
    _init_disc_map(sim, 0.5, 0.5, 0.2, layers)
    k = 2.0 * np.pi
    a = 0.05 * k * np.sin(k * sim.X) * np.cos(k * sim.Y)
    b = -0.05 * k * np.cos(k * sim.X) * np.sin(k * sim.Y)
    from .bc import FreeSlipBox
    a, b = FreeSlipBox()(a, b)
    sim.set_field("u", a)
    sim.set_field("v", b)
    return sim


def lid_driven_cavity(Re=100.0, N=129):
    """Config 1: pure fluid (phi = 1), rho_s = mu_s = 0 (lid_driven_cavity.py:26-52)."""
    X, Y, dx, dy = F.create_grid(N, N, 1.0, 1.0)
    sim = Simulation(N, bc_kind=NOSLIP_LID, lid=1.0, disc=None, mu_s=0.0, kappa=0.0, rho_s=0.0,
                     eta_s=0.0, mu_f=1.0 / Re, rho_f=1.0, w_t=2.0 * dx, layers=0, cfl=0.2,
                     dt_cap=1e-2)
    from .bc import NoSlipLid
    a, b = NoSlipLid(1.0)(np.zeros((N, N)), np.zeros((N, N)))
    sim.set_field("u", a); sim.set_field("v", b)
    sim.set_field("X1", X); sim.set_field("X2", Y)
    return sim


def run_lid_driven_cavity(Re=100.0, N=129, max_steps=60000, steady_tol=2e-5, chunk=200):
    """lid_driven_cavity.py:54-97: steady-state loop.  The reference checks
    max|u - u_prev| / dt < tol at step 1 and every `chunk` steps; the device advances in
    bulk between checks and snapshots u only before a checked step."""
    sim = lid_driven_cavity(Re, N)
    torch = sim.torch
    u = sim._view("u")   # read only
    step = 0
    while step < max_steps:
        nxt = step + 1
        if nxt == 1 or nxt % chunk == 0:
            prev = u.clone()
            sim.step(1)
            step = nxt
            dt = sim.diagnostics()["dt"][-1]
            res = float(torch.max(torch.abs(u - prev))) / dt
            if step > 1 and res < steady_tol:
                break
        else:
            nchk = ((nxt + chunk - 1) // chunk) * chunk
            n_adv = min(nchk - 1, max_steps) - step
            sim.step(n_adv)
            step += n_adv
    return sim, step


def ghia_rms(sim, y_ref, u_ref):
    """lid_driven_cavity.py:90-97: RMS of u(x=0.5) against Ghia et al."""
    a = sim.get("u")
    i_mid = sim.N // 2
    return float(np.sqrt(np.mean((np.interp(y_ref, sim.Y[:, i_mid], a[:, i_mid]) - u_ref) ** 2)))
