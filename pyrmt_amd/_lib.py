"""ctypes binding of librmt.so (include/rmt.h).  The product path has no CPU fallback:
if the HIP library is missing or no GPU is visible, calls fail loudly."""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# RMT_LIB: an alternative build of the same sources (A/B measurements of compile-time
# variants, e.g. `make -C pyrmt_amd/csrc VARIANT=w16 DEFS=-DRMT_CH_W=16`)
LIB_PATH = os.environ.get("RMT_LIB") or os.path.join(_HERE, "librmt.so")

RMT_OK, RMT_EINVAL, RMT_ENONFINITE, RMT_EDEVICE, RMT_ENOTSUP, RMT_ENOMEM = range(6)


class RMTError(RuntimeError):
    pass


class rmt_momentum_params(ctypes.Structure):
    _fields_ = [("bc_kind", ctypes.c_int), ("lid", ctypes.c_double),
                ("mu_s", ctypes.c_double), ("kappa", ctypes.c_double),
                ("eta_s", ctypes.c_double), ("rho_s", ctypes.c_double),
                ("rho_f", ctypes.c_double), ("mu_f", ctypes.c_double), ("w_t", ctypes.c_double),
                ("dx", ctypes.c_double), ("dy", ctypes.c_double), ("dt", ctypes.c_double),
                ("stress_band", ctypes.c_int), ("detg_clamp", ctypes.c_double)]


class rmt_sim_params(ctypes.Structure):
    _fields_ = [("ny", ctypes.c_int), ("nx", ctypes.c_int),
                ("dx", ctypes.c_double), ("dy", ctypes.c_double),
                ("xs", ctypes.c_void_p), ("ys", ctypes.c_void_p),
                ("scheme", ctypes.c_int), ("bc_kind", ctypes.c_int), ("lid", ctypes.c_double),
                ("shape", ctypes.c_int), ("x0", ctypes.c_double), ("y0", ctypes.c_double),
                ("R", ctypes.c_double),
                ("mu_s", ctypes.c_double), ("kappa", ctypes.c_double), ("rho_s", ctypes.c_double),
                ("eta_s", ctypes.c_double), ("mu_f", ctypes.c_double), ("rho_f", ctypes.c_double),
                ("w_t", ctypes.c_double), ("layers", ctypes.c_int),
                ("cfl", ctypes.c_double), ("dt_cap", ctypes.c_double),
                ("stress_band", ctypes.c_int), ("detg_clamp", ctypes.c_double),
                ("energies", ctypes.c_int)]


class rmt_diag(ctypes.Structure):
    _fields_ = [(k, ctypes.c_double) for k in
                ("t", "dt", "cx", "cy", "minJ", "maxJ", "umax", "ke", "se", "diss", "integ", "ry")]


class rmt_mac_params(ctypes.Structure):
    _fields_ = [("N", ctypes.c_int), ("dx", ctypes.c_double), ("n_discs", ctypes.c_int),
                ("R", ctypes.c_double * 8), ("cx", ctypes.c_double * 8),
                ("cy", ctypes.c_double * 8), ("U_lid", ctypes.c_double),
                ("mu_s", ctypes.c_double), ("mu_f", ctypes.c_double), ("rho", ctypes.c_double),
                ("eta", ctypes.c_double), ("layers", ctypes.c_int), ("dt", ctypes.c_double)]


class rmt_mac_diag(ctypes.Structure):
    _fields_ = [("t", ctypes.c_double), ("dt", ctypes.c_double), ("minJ", ctypes.c_double),
                ("maxJ", ctypes.c_double), ("umax", ctypes.c_double), ("n_discs", ctypes.c_int),
                ("cx", ctypes.c_double * 8), ("cy", ctypes.c_double * 8),
                ("diverged", ctypes.c_int)]


_P, _D, _I, _L = ctypes.c_void_p, ctypes.c_double, ctypes.c_int, ctypes.c_long
SIGNATURES = {
    "rmt_last_error": (ctypes.c_char_p, []),
    "rmt_version": (_I, []),
    "rmt_ctx_create": (_I, [_I, _I, _I, _P, ctypes.POINTER(_P)]),
    "rmt_ctx_set_stream": (_I, [_P, _P]),
    "rmt_ctx_destroy": (_I, [_P]),
    "rmt_ctx_sync": (_I, [_P]),
    "rmt_ctx_set_profiling": (_I, [_P, _I]),
    "rmt_ctx_kernel_ms": (_I, [_P, ctypes.POINTER(_D)]),
    "rmt_ctx_set_option": (_I, [_P, ctypes.c_char_p, _I]),
    "rmt_ctx_get_option": (_I, [_P, ctypes.c_char_p, ctypes.POINTER(_I)]),
    "rmt_grad_x_2nd": (_I, [_P, _P, _D, _P]),
    "rmt_grad_y_2nd": (_I, [_P, _P, _D, _P]),
    "rmt_diff_upwind_3rd": (_I, [_P, _P, _P, _D, _I, _P]),
    "rmt_bilinear_interpolate": (_I, [_P, _P, _P, _P, _L, _D, _D, _P]),
    "rmt_advect_sl_rk4": (_I, [_P, _P, _P, _P, _P, _P, _D, _D, _D, _P]),
    "rmt_weno5_rhs": (_I, [_P, _P, _P, _P, _D, _D, _P, _D, _P]),
    "rmt_advect_weno5_rk3": (_I, [_P, _P, _P, _P, _D, _D, _D, _P, _D, _P]),
    "rmt_all_finite2": (_I, [_P, _P, _P, ctypes.POINTER(_I)]),
    "rmt_selftest_divk": (_I, [_P, _P, _L, _D, _P, _P]),
    "rmt_central_rhs": (_I, [_P, _P, _P, _P, _D, _D, _P, _D, _I, _P]),
    "rmt_advect_central_rk3": (_I, [_P, _P, _P, _P, _D, _D, _D, _P, _D, _I, _P]),
    "rmt_bicubic_interpolate": (_I, [_P, _P, _P, _P, _L, _D, _D, _P]),
    "rmt_advect_sl_cubic_rk4": (_I, [_P, _P, _P, _P, _P, _P, _D, _D, _D, _P]),
    "rmt_extrapolate_reference_map": (_I, [_P, _P, _P, _P, _D, _D, _I, _P, _P]),
    "rmt_extrap_set_mode": (_I, [_I]),
    "rmt_extrap_set_parallel": (_I, [_I]),
    "rmt_momentum_set_mode": (_I, [_I]),
    "rmt_extrap_last_path": (_I, [_P, ctypes.POINTER(_I)]),
    "rmt_rebuild_phi_disc": (_I, [_P, _P, _P, _D, _D, _D, _P]),
    "rmt_solid_cauchy_stress": (_I, [_P, _P, _P, _D, _D, _D, _D, _P, _D, _D, _I, _P, _P, _P, _P]),
    "rmt_smoothed_heaviside": (_I, [_P, _P, _L, _D, _P]),
    "rmt_apply_velocity_bc": (_I, [_P, _I, _D, _P, _P]),
    "rmt_momentum_step_rk4": (_I, [_P, ctypes.POINTER(rmt_momentum_params), _P, _P, _P, _P, _P,
                                   _P, _P, _P, _P, _P, _P, _P]),
    "rmt_divergence_rc": (_I, [_P, _P, _P, _P, _D, _D, _D, _P]),
    "rmt_divergence_central": (_I, [_P, _P, _P, _D, _D, _P]),
    "rmt_pressure_gradient": (_I, [_P, _P, _D, _D, _P, _P]),
    "rmt_solve_poisson_dct": (_I, [_P, _P, _D, _D, _P]),
    "rmt_pressure_projection": (_I, [_P, _P, _P, _D, _D, _D, _D, _I, _D, _P, _P, _P, _P]),
    "rmt_pressure_projection_variable": (_I, [_P, _P, _P, _D, _D, _D, _P, _I, _D, _P, _D, _I,
                                              _P, _P, _P, ctypes.POINTER(_I)]),
    "rmt_apply_variable_poisson": (_I, [_P, _P, _D, _D, _P, _P]),
    "rmt_divergence_rc_variable": (_I, [_P, _P, _P, _P, _D, _P, _D, _D, _P]),
    "rmt_compute_timestep": (_I, [_P, _P, _P, _D, _D, _D, _D, _D, _D, _D, _D, _D, _D, _D,
                                  ctypes.POINTER(_D)]),
    "rmt_divergence_2d_interior": (_I, [_P, _P, _P, _D, _D, _I, _P]),
    "rmt_compute_kinetic_energy": (_I, [_P, _P, _P, _D, _D, _P, _D, _D, _D, ctypes.POINTER(_D)]),
    "rmt_compute_strain_energy": (_I, [_P, _P, _P, _P, _D, _D, _D, _D, ctypes.POINTER(_D)]),
    "rmt_compute_viscous_dissipation": (_I, [_P, _P, _P, _D, _P, _D, _D, _D, _D,
                                             ctypes.POINTER(_D)]),
    "rmt_velocity_rhs_blended": (_I, [_P, _P, _P, _P, _P, _P, _P, _D, _D, _D, _P, _P, _P, _P,
                                      _P, _P]),
    "rmt_sim_create": (_I, [_P, ctypes.POINTER(rmt_sim_params), ctypes.POINTER(_P)]),
    "rmt_sim_destroy": (_I, [_P]),
    "rmt_sim_set_sync_every": (_I, [_P, _I]),
    "rmt_sim_field": (_I, [_P, _I, ctypes.POINTER(_P)]),
    "rmt_sim_step": (_I, [_P, _I, _D]),
    "rmt_sim_diagnostics": (_I, [_P, ctypes.POINTER(rmt_diag), _I, ctypes.POINTER(_I)]),
    "rmt_sim_set_profiling": (_I, [_P, _I]),
    "rmt_sim_set_carry": (_I, [_P, _I]),
    "rmt_sim_invalidate": (_I, [_P]),
    "rmt_sim_phase_times": (_I, [_P, ctypes.POINTER(_D), ctypes.POINTER(_L)]),
    # periodic branch
    "rmt_divergence_periodic": (_I, [_P, _P, _P, _D, _D, _P]),
    "rmt_pressure_gradient_periodic": (_I, [_P, _P, _D, _D, _P, _P]),
    "rmt_solve_poisson_fft": (_I, [_P, _P, _P, _P, _P]),
    "rmt_pressure_projection_periodic": (_I, [_P, _P, _P, _D, _D, _D, _D, _P, _I, _D, _P, _P,
                                              _P, _P, _P, _P]),
    # slab-decomposed step (distributed.py)
    "rmt_slab_create": (_I, [_P, ctypes.POINTER(rmt_sim_params), _I, _I, ctypes.POINTER(_I),
                             ctypes.POINTER(_I), ctypes.POINTER(_P)]),
    "rmt_slab_destroy": (_I, [_P]),
    "rmt_slab_info": (_I, [_P, ctypes.POINTER(_I), ctypes.POINTER(_D)]),
    "rmt_slab_buffer": (_I, [_P, _I, ctypes.POINTER(_P)]),
    "rmt_slab_begin": (_I, [_P]),
    "rmt_slab_advect_interior": (_I, [_P, _D]),
    "rmt_slab_advect": (_I, [_P, _D]),
    "rmt_slab_rim_pack": (_I, [_P]),
    "rmt_slab_extrapolate": (_I, [_P, _P, ctypes.POINTER(ctypes.c_longlong), ctypes.c_longlong]),
    "rmt_slab_momentum": (_I, [_P, _D]),
    "rmt_slab_project_rows": (_I, [_P, _D]),
    "rmt_slab_project_cols": (_I, [_P]),
    "rmt_slab_project_unrows": (_I, [_P]),
    "rmt_slab_sub_mean": (_I, [_P, _I, _P]),
    "rmt_slab_project_correct": (_I, [_P, _D]),
    "rmt_slab_finish": (_I, [_P]),
    "rmt_slab_set_device_dt": (_I, [_P, _I]),
    "rmt_slab_next_dt": (_I, [_P, _P, _I, _P]),
    "rmt_slab_rim_cap": (_I, [_P, ctypes.c_longlong]),
    "rmt_slab_next_bits": (_I, [_P]),
    "rmt_slab_geometry": (_I, [_P]),
    "rmt_slab_drop_geometry": (_I, [_P]),
    "rmt_slab_extrapolate_dev": (_I, [_P, _P, _P, ctypes.c_longlong]),
    # MAC slabs (distributed.py MacDistributedSim)
    "rmt_mac_slab_create": (_I, [_P, ctypes.POINTER(rmt_mac_params), _I, _I, ctypes.POINTER(_I),
                                 ctypes.POINTER(_I), ctypes.POINTER(_P)]),
    "rmt_mac_slab_destroy": (_I, [_P]),
    "rmt_mac_slab_info": (_I, [_P, ctypes.POINTER(_I)]),
    "rmt_mac_slab_buffer": (_I, [_P, _I, _I, ctypes.POINTER(_P)]),
    "rmt_mac_slab_advect": (_I, [_P, _D]),
    "rmt_mac_slab_rim_pack": (_I, [_P]),
    "rmt_mac_slab_extrapolate": (_I, [_P, _I, _P, ctypes.POINTER(ctypes.c_longlong),
                                      ctypes.c_longlong]),
    "rmt_mac_slab_extrapolate_identity": (_I, [_P, _I]),
    "rmt_mac_slab_predict": (_I, [_P, _D]),
    "rmt_mac_slab_project_rows": (_I, [_P, _P]),
    "rmt_mac_slab_project_cols": (_I, [_P]),
    "rmt_mac_slab_project_unrows": (_I, [_P]),
    "rmt_mac_slab_correct": (_I, [_P, _D]),
    # MAC path (mac.py)
    "rmt_mac_divergence": (_I, [_P, _P, _P, _D, _D, _P]),
    "rmt_mac_gradient_p": (_I, [_P, _P, _D, _D, _P, _P]),
    "rmt_mac_solve_poisson_neumann": (_I, [_P, _P, _D, _D, _P, _P, _P]),
    "rmt_mac_project": (_I, [_P, _P, _P, _D, _D, _D, _D, _P, _P, _P, _P, _P]),
    "rmt_mac_momentum_predictor": (_I, [_P, _P, _P, _D, _D, _D, _D, _D, _P, _P, _D, _P, _P]),
    "rmt_mac_lap_lid_hom": (_I, [_P, _I, _P, _D, _D, _P]),
    "rmt_mac_helmholtz": (_I, [_P, _I, _P, _D, _D, _D, _D, _I, _I, _P, ctypes.POINTER(_I)]),
    "rmt_mac_momentum_predictor_lid_imex": (_I, [_P, _P, _P, _D, _D, _D, _D, _D, _P, _P, _D, _D,
                                                 _D, _P, _P, _P]),
    "rmt_mac_momentum_predictor_lid_semilag": (_I, [_P, _P, _P, _D, _D, _D, _D, _D, _P, _P, _D,
                                                    _D, _D, _P, _P, _P]),
    "rmt_mac_contact_stress": (_I, [_P, _P, _P, _D, _D, _D, _D, _D, _P, _P, _P]),
    "rmt_mac_sim_create": (_I, [_P, ctypes.POINTER(rmt_mac_params), ctypes.POINTER(_P)]),
    "rmt_mac_sim_destroy": (_I, [_P]),
    "rmt_mac_sim_field": (_I, [_P, _I, _I, ctypes.POINTER(_P)]),
    "rmt_mac_sim_step": (_I, [_P, _I, _D]),
    "rmt_mac_sim_diagnostics": (_I, [_P, ctypes.POINTER(rmt_mac_diag), _I, ctypes.POINTER(_I)]),
}

_lib = None


def lib():
    """Load librmt.so (once).  Raises if the HIP library was not built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"librmt.so not found at {LIB_PATH}: build it first "
                "(python -c 'import __graft_entry__ as g; g.build()')")
        # torch first: librmt's libamdhip64 dependency then binds to the HIP runtime torch
        # loaded (loaded the other way round, torch's device calls found no device)
        import torch  # noqa: F401
        h = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(h, name)
            fn.restype = res
            fn.argtypes = args
        _lib = h
    return _lib


_DEBUG_SYNC = bool(os.environ.get("RMT_DEBUG_SYNC"))


def check(status, what=""):
    if status == RMT_OK:
        if _DEBUG_SYNC:      # debugging aid: surface asynchronous faults at the call
            import torch
            torch.cuda.synchronize()
        return
    msg = (lib().rmt_last_error() or b"").decode(errors="replace")
    if status == RMT_ENONFINITE:
        raise FloatingPointError(msg or what)
    if status == RMT_EINVAL:
        raise ValueError(msg or what)
    if status == RMT_ENOTSUP:
        raise NotImplementedError(msg or what)
    raise RMTError(f"{what}: {msg} (status {status})")
