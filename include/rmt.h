/*
 * rmt.h -- C ABI of librmt, the MI355X-native 2D Reference Map Technique (RMT) time step.
 *
 * This is the drop-in boundary for pyRMT's per-step hot path.  The
 * reference has no native library: its operator surface is the set of module-level
 * Python functions re-exported by pyRMT/__init__.py:1-57, called by the benchmark loop
 * bodies (e.g. benchmarks/soft_disc_in_lid_driven.py:206-235).  Each entry point below
 * replaces one of those functions (cited per entry); pyrmt_amd/functions.py binds them
 * with ctypes under the reference names and signatures.
 *
 * Conventions
 *   - Fields are float64, C-contiguous, shape (ny, nx), element [j*nx + i] (j <-> y).
 *   - Every array argument is a DEVICE pointer (hipMalloc / torch.cuda memory) on the
 *     context's device.  Calls are stream-ordered on the context stream and return once
 *     enqueued, except where a host result is returned (documented per call).
 *   - The caller allocates and frees every I/O buffer.  The context owns scratch space,
 *     FFT plans and the step state of an rmt_sim.
 *   - Errors: every call returns an rmt_status; rmt_last_error() describes the last
 *     failure on the calling thread.  The Python shim maps RMT_ENONFINITE to
 *     FloatingPointError and RMT_EINVAL to ValueError, like the reference
 *     (functions.py:524-526, :539-542).
 *   - Velocity BCs and level-set shapes cross as enums + parameters instead of the
 *     reference's Python callables (functions.py:946-947, :1366-1367).
 *   - Not re-entrant per context.
 */
#ifndef RMT_H
#define RMT_H

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
    RMT_OK = 0,
    RMT_EINVAL = 1,      /* bad argument (unknown scheme / bc / shape, bad size)   */
    RMT_ENONFINITE = 2,  /* non-finite velocity fed to advection                  */
    RMT_EDEVICE = 3,     /* HIP / rocFFT failure                                   */
    RMT_ENOTSUP = 4,     /* valid in the reference but outside this build's path   */
    RMT_ENOMEM = 5
} rmt_status;

/* Velocity boundary conditions (benchmarks/common.py:27-50). */
typedef enum {
    RMT_BC_NONE = 0,          /* identity                                            */
    RMT_BC_NOSLIP_LID = 1,    /* no_slip_lid_bc: walls 0, top row u = lid, corners 0  */
    RMT_BC_FREESLIP_BOX = 2,  /* free_slip_box_bc: normal 0, tangential copied        */
    RMT_BC_PERIODIC = 3       /* overlap grid: last column / row copy column / row 0  */
} rmt_bc_kind;

/* Reference-map advection schemes (functions.py:501-542). */
typedef enum {
    RMT_SCHEME_SEMILAGRANGIAN = 0,  /* advect_semilagrangian_rk4 (bilinear)            */
    RMT_SCHEME_WENO5 = 1,           /* advect_weno5_rk3                               */
    RMT_SCHEME_CENTRAL2 = 2,        /* advect_central2_rk3                            */
    RMT_SCHEME_CONSERVATIVE = 3,    /* advect_conservative_rk3 (Jain 2019 eq. 26)      */
    RMT_SCHEME_SEMILAGRANGIAN_CUBIC = 4 /* advect_semilagrangian_cubic_rk4 (bicubic)  */
} rmt_scheme;

typedef struct rmt_ctx rmt_ctx;

const char *rmt_last_error(void);
int rmt_version(void);

/* Context: one device, one stream, one grid shape.  stream may be NULL (null stream)
 * or a hipStream_t (e.g. torch.cuda.current_stream().cuda_stream). */
int rmt_ctx_create(int ny, int nx, int device, void *stream, rmt_ctx **out);
int rmt_ctx_set_stream(rmt_ctx *ctx, void *stream);
int rmt_ctx_destroy(rmt_ctx *ctx);
int rmt_ctx_sync(rmt_ctx *ctx);
/* HIP-event kernel timers on the ctx stream: after each momentum / extrapolation call,
 * ms2[0] = the four RK4 stage kernels of the last momentum call, ms2[1] = the last
 * extrapolation chain (0 if none was recorded).  Blocks until the events complete. */
int rmt_ctx_set_profiling(rmt_ctx *ctx, int on);
int rmt_ctx_kernel_ms(rmt_ctx *ctx, double *ms2);
/* Per-context implementation switches (bit-identical alternatives of the schedule and the
 * kernels, for A/B measurements and the regression tests): each starts from its environment
 * variable at rmt_ctx_create.  Names: ext_events, ex_arena_bump, ex_profile, fix_all,
 * dct_rocfft, transpose2, sim_hiprio, sim_sync, early_geometry, early_transpose, fused_fluid,
 * no_overlap, side_tail, par_overlap, fused_fixprep, merged_join, test_delay_side,
 * test_delay_main, chain_cols, chain_layer_groups, edge_slots, edge_stream, sl_phi,
 * mac_boxes, skip_marked_rows, tail_stream, diag_first, mac_noop_host, mac_face_sl,
 * mac_m2_bound, diag_seg, sl_zero_flags, dct_desc, and the test-only test_delay_geo / test_nowait_drop (a slab's
 * early geometry delayed; a dropped geometry not waited for).  Set them before creating a sim or slab on the context (sim_hiprio is read
 * at rmt_sim_create); a change ends a carried step state.
 * Unknown name: RMT_EINVAL. */
int rmt_ctx_set_option(rmt_ctx *ctx, const char *name, int value);
int rmt_ctx_get_option(rmt_ctx *ctx, const char *name, int *value);

/* ---- finite-difference helpers (pyRMT/utils.py) ----------------------------------- */
/* utils.py:4-14 grad_central_x_2nd / utils.py:16-25 grad_central_y_2nd */
int rmt_grad_x_2nd(rmt_ctx *ctx, const double *f, double h, double *out);
int rmt_grad_y_2nd(rmt_ctx *ctx, const double *f, double h, double *out);
/* utils.py:61-114 diff_upwind_3rd (axis 1 = x, 0 = y) */
int rmt_diff_upwind_3rd(rmt_ctx *ctx, const double *f, const double *vel, double h, int axis,
                        double *out);

/* ---- interpolation / reference-map transport (interpolators.py, functions.py) ------ */
/* interpolators.py:4-61 bilinear_interpolate: u is (ny, nx) of the ctx grid, nq queries. */
int rmt_bilinear_interpolate(rmt_ctx *ctx, const double *u, const double *xq, const double *yq,
                             long nq, double dx, double dy, double *out);
/* functions.py:194-227 advect_semilagrangian_rk4 */
int rmt_advect_sl_rk4(rmt_ctx *ctx, const double *q, const double *a, const double *b,
                      const double *X, const double *Y, double dt, double dx, double dy,
                      double *out);
/* functions.py:321-393 _weno5_rhs and functions.py:396-415 advect_weno5_rk3 */
int rmt_weno5_rhs(rmt_ctx *ctx, const double *q, const double *a, const double *b, double dx,
                  double dy, const double *phi, double w_cut, double *rhs);
int rmt_advect_weno5_rk3(rmt_ctx *ctx, const double *q, const double *a, const double *b,
                         double dx, double dy, double dt, const double *phi, double w_cut,
                         double *out);
/* functions.py:524-526 guard: sets *finite (host) to 1 if every a, b is finite.  Blocks. */
/* functions.py:420-495 _central2_rhs / _conservative_rhs and the SSP-RK3 drivers
 * advect_central2_rk3 / advect_conservative_rk3 (conservative = 0 / 1) */
int rmt_central_rhs(rmt_ctx *ctx, const double *q, const double *a, const double *b, double dx,
                    double dy, const double *phi, double w_cut, int conservative, double *rhs);
int rmt_advect_central_rk3(rmt_ctx *ctx, const double *q, const double *a, const double *b,
                           double dx, double dy, double dt, const double *phi, double w_cut,
                           int conservative, double *out);
/* interpolators.py:64-156 bicubic_interpolate; functions.py:228-251 the bicubic SL-RK4 */
int rmt_bicubic_interpolate(rmt_ctx *ctx, const double *u, const double *xq, const double *yq,
                            long nq, double dx, double dy, double *out);
int rmt_advect_sl_cubic_rk4(rmt_ctx *ctx, const double *q, const double *a, const double *b,
                            const double *X, const double *Y, double dt, double dx, double dy,
                            double *out);
int rmt_all_finite2(rmt_ctx *ctx, const double *a, const double *b, int *finite);
/* Test hook (no reference counterpart): q = divk(x, d), the correctly rounded division by a
 * precomputed divisor that the stencil kernels use for x / (2h), x / (6h), xq / dx, ...
 * (pyrmt_amd/csrc/divk.hpp), and q_ieee = x / d, both on the device (device pointers). */
int rmt_selftest_divk(rmt_ctx *ctx, const double *x, long n, double d, double *q,
                      double *q_ieee);

/* functions.py:48-163 extrapolate_reference_map: exact raster-order (Gauss-Seidel)
 * semantics of the reference; outputs may alias the inputs.  Blocks until the result is
 * complete and returns RMT_EDEVICE if the extrapolation aborted (bug guard / spin timeout),
 * so a caller never sees a partly extrapolated map with RMT_OK. */
int rmt_extrapolate_reference_map(rmt_ctx *ctx, const double *X1, const double *X2,
                                  const double *phi, double dx, double dy, int max_layers,
                                  double *X1_out, double *X2_out);
/* librmt diagnostics for the extrapolation (no reference counterpart).  mode 0 (default):
 * geometry-first chain path, row-ticket sweep when its capacity limits are exceeded;
 * 1: sweep only; 2: chain path's pre-passes, then the sweep forced; 3: mode 0, then the
 * abort status is raised (exercises the callers' error paths).  rmt_extrap_last_path
 * (blocks) reports what the last call on ctx ran: 0 chain, 1 sweep. */
int rmt_extrap_set_mode(int mode);
/* Parallel extrapolation (no reference counterpart; default off, or RMT_EXTRAP_PARALLEL=1):
 * every fit of functions.py:95-161 -- the same targets, acceptance, weights and raster-order
 * known sets -- evaluated as the weighted least-squares plane in offsets from the target and
 * the layer solved as one sparse triangular system by segments (extrap_par.hip), instead of
 * the exact raster-order chain.  Not bit-exact: each fit differs from the reference by the
 * reference's own rounding of Cramer's rule on absolute coordinates (~1e-7 at N = 4096,
 * the size of 1-ulp weight noise).  Process-wide; applies to the
 * extrapolations started after the call. */
int rmt_extrap_set_parallel(int on);
int rmt_extrap_last_path(rmt_ctx *ctx, int *path);

/* functions.py:1366-1367 with benchmarks/common.py:55-57: phi = |xi - (x0,y0)| - R */
int rmt_rebuild_phi_disc(rmt_ctx *ctx, const double *X1, const double *X2, double x0, double y0,
                         double R, double *phi);

/* ---- stress / momentum (functions.py:545-944) -------------------------------------- */
/* functions.py:545-658 solid_cauchy_stress */
int rmt_solid_cauchy_stress(rmt_ctx *ctx, const double *X1, const double *X2, double dx,
                            double dy, double mu_s, double kappa, const double *phi,
                            double w_cut, double detg_clamp, int isochoric, double *sxx,
                            double *sxy, double *syy, double *J);
/* functions.py:660-671 smoothed_heaviside; n elements */
int rmt_smoothed_heaviside(rmt_ctx *ctx, const double *x, long n, double w_t, double *H);
/* benchmarks/common.py:27-50, in place */
int rmt_apply_velocity_bc(rmt_ctx *ctx, int bc_kind, double lid, double *u, double *v);

typedef struct {
    int bc_kind;        /* rmt_bc_kind */
    double lid;         /* lid speed for RMT_BC_NOSLIP_LID */
    double mu_s, kappa, eta_s, rho_s, rho_f, mu_f, w_t;
    double dx, dy, dt;
    int stress_band;    /* functions.py:673-674 stress_band */
    double detg_clamp;
} rmt_momentum_params;

/* functions.py:673-762 momentum_step_rk4 (gamma = 0: surface tension is outside the
 * path).  Outputs u*, v* and the elastic sxx, sxy, syy, J it precomputes. */
int rmt_momentum_step_rk4(rmt_ctx *ctx, const rmt_momentum_params *prm, const double *u,
                          const double *v, const double *p, const double *X1, const double *X2,
                          const double *phi, double *u_new, double *v_new, double *sxx,
                          double *sxy, double *syy, double *J);

/* librmt diagnostic (no reference counterpart): 0 (default) one LDS-tiled kernel per RK4
 * stage, 2 unfused per-cell passes.  Bit-identical results in both; other modes: RMT_EINVAL. */
int rmt_momentum_set_mode(int mode);

/* ---- projection (functions.py:1005-1364) ------------------------------------------- */
/* functions.py:1016-1071 _compute_divergence_rc, constant density: d_f = dt / mean(rho) */
int rmt_divergence_rc(rmt_ctx *ctx, const double *a, const double *b, const double *p,
                      double d_f, double dx, double dy, double *divU);
/* functions.py:1005-1014 _compute_divergence */
int rmt_divergence_central(rmt_ctx *ctx, const double *a, const double *b, double dx,
                           double dy, double *divU);
/* functions.py:1073-1089 _compute_pressure_gradient */
int rmt_pressure_gradient(rmt_ctx *ctx, const double *p, double dx, double dy, double *gx,
                          double *gy);
/* functions.py:1107-1119 _solve_poisson_dct: idctn(dctn(rhs,1)/eig,1) - mean, with eig
 * the DCT-I symbol of functions.py:1091-1104 for this grid (dx, dy). */
int rmt_solve_poisson_dct(rmt_ctx *ctx, const double *rhs, double dx, double dy, double *p);
/* functions.py:1255-1364 pressure_projection_amg, Neumann branch, constant density rho
 * (variable density: rmt_pressure_projection_variable).  p_prev may be NULL. */
int rmt_pressure_projection(rmt_ctx *ctx, const double *a_star, const double *b_star,
                            double dx, double dy, double dt, double rho, int bc_kind,
                            double lid, const double *p_prev, double *a, double *b, double *p);
/* The variable-density branch (rho a device (ny, nx) array with ptp > 1e-10),
 * functions.py:1296-1328 + :1350-1364: Rhie-Chow divergence with per-face dt/rho, rhs =
 * divU/dt - mean, preconditioned CG (scipy.sparse.linalg.cg semantics: x0 = 0, stop when
 * ||r|| < rtol ||rhs||, at most maxiter iterations; the reference passes tol = 1e-6,
 * maxiter = 200) on the matrix-free div((1/rho) grad) operator with the DCT-I solve as the
 * preconditioner, then a = a* - (dt/rho) grad p_c, BC, p = p_prev + p_c - mean.
 * *iters receives the iteration count (maxiter: not converged, as scipy's info > 0). */
int rmt_pressure_projection_variable(rmt_ctx *ctx, const double *a_star, const double *b_star,
                                     double dx, double dy, double dt, const double *rho,
                                     int bc_kind, double lid, const double *p_prev, double rtol,
                                     int maxiter, double *a, double *b, double *p, int *iters);
/* functions.py:1122-1168 _apply_variable_poisson: div((1/rho) grad p), face-averaged 1/rho,
 * mirror ghosts. */
int rmt_apply_variable_poisson(rmt_ctx *ctx, const double *p, double dx, double dy,
                               const double *inv_rho, double *out);
/* functions.py:1016-1070 _compute_divergence_rc with a variable rho array (per-face
 * d_f = dt * 0.5 * (1/rho_l + 1/rho_r)). */
int rmt_divergence_rc_variable(rmt_ctx *ctx, const double *a, const double *b, const double *p,
                               double dt, const double *rho, double dx, double dy,
                               double *divU);

/* functions.py:165-192 compute_timestep; host result, blocks. */
int rmt_compute_timestep(rmt_ctx *ctx, const double *a, const double *b, double dx, double dy,
                         double CFL, double dt_min_cap, double mu_s, double rho_s, double gamma,
                         double rho_f, double mu_f, double eta_s, double kappa, double *dt);

/* ---- standalone diagnostics and the blended RHS (pyRMT/__init__.py:16, :28-31) --------
 * Energies return a host scalar and block; the sum runs in np.sum's own order (pairwise over
 * 8192-element chunks), so a bit-exact density gives a bit-exact energy. */
/* output.py:6-39: sum(0.5 rho (a^2 + b^2)) dx dy, rho = (1-H) rho_s + H rho_f */
int rmt_compute_kinetic_energy(rmt_ctx *ctx, const double *a, const double *b, double rho_f,
                               double rho_s, const double *phi, double w_t, double dx, double dy,
                               double *ke);
/* output.py:41-134: neo-Hookean + volumetric strain energy over phi <= 0 (edge-padded grads) */
int rmt_compute_strain_energy(rmt_ctx *ctx, const double *X1, const double *X2, const double *phi,
                              double mu_s, double dx, double dy, double kappa, double *se);
/* output.py:136-193: viscous dissipation rate, mu = H mu_f + (1-H) eta_s */
int rmt_compute_viscous_dissipation(rmt_ctx *ctx, const double *a, const double *b, double mu_f,
                                    const double *phi, double w_t, double dx, double dy,
                                    double eta_s, double *diss);
/* output.py:195-211 divergence_2d_interior (the div_vel dataset of output_simulation_data,
 * pad = 4 there): central differences on the cells >= pad from every edge, 0 elsewhere */
int rmt_divergence_2d_interior(rmt_ctx *ctx, const double *u, const double *v, double dx,
                               double dy, int pad, double *div);
/* functions.py:897-944 velocity_rhs_blended_optimized: H, rho_local device arrays; the
 * surface-tension force fx, fy device arrays or both NULL (the scalar 0.0 of the gamma = 0
 * path).  (phi, dH_dx, dH_dy of the reference signature are unused by its body.) */
int rmt_velocity_rhs_blended(rmt_ctx *ctx, const double *u, const double *v, const double *p,
                             const double *sxx, const double *sxy, const double *syy, double dx,
                             double dy, double mu_f, const double *H, const double *rho,
                             const double *fx, const double *fy, double *rhs_u, double *rhs_v);

/* ---- fused, device-resident time step (the loop body of the benchmark drivers) ----- */
typedef enum {
    RMT_SHAPE_NONE = 0,   /* pure fluid (lid_driven_cavity.py): phi = 1, no solid       */
    RMT_SHAPE_DISC = 1    /* one disc: phi = |xi - (x0,y0)| - R                         */
} rmt_shape_kind;

typedef struct {
    int ny, nx;
    double dx, dy;
    const double *xs, *ys;   /* HOST node coordinates, length nx and ny (create_grid) */
    int scheme;              /* rmt_scheme                                            */
    int bc_kind;             /* rmt_bc_kind                                           */
    double lid;
    int shape;               /* rmt_shape_kind                                        */
    double x0, y0, R;
    double mu_s, kappa, rho_s, eta_s, mu_f, rho_f, w_t;
    int layers;              /* extrapolation layers                                  */
    double cfl, dt_cap;      /* compute_timestep CFL and dt_min_cap                   */
    int stress_band;
    double detg_clamp;
    int energies;            /* per-step KE / SE / dissipation (disc_in_taylor_green) */
} rmt_sim_params;

typedef struct rmt_sim rmt_sim;

/* Per-step diagnostics, one record per completed step (soft_disc_in_lid_driven.py:233
 * traj tuple, disc_in_taylor_green.py:243 hist tuple). */
typedef struct {
    double t, dt, cx, cy, minJ, maxJ, umax;
    double ke, se, diss, integ, ry;
} rmt_diag;

int rmt_sim_create(rmt_ctx *ctx, const rmt_sim_params *prm, rmt_sim **out);
int rmt_sim_destroy(rmt_sim *sim);
/* how often (steps, 1 .. 64) rmt_sim_step reads the device diagnostics back (see below) */
int rmt_sim_set_sync_every(rmt_sim *sim, int k);
/* field ids: 0 u (a), 1 v (b), 2 p, 3 X1, 4 X2, 5 phi (last rebuilt), 6 J, 7 sigma_xx,
 * 8 sigma_xy, 9 sigma_yy (the solid stress of the last momentum step) */
int rmt_sim_field(rmt_sim *sim, int field, double **dev_ptr);
/* Run nsteps loop bodies.  dt comes from compute_timestep on device and is clipped to
 * t_end - t as the drivers do; steps after t >= t_end are no-ops.  Blocks: the diagnostics
 * and flags of the enqueued steps are read back every rmt_sim_set_sync_every steps (64 by
 * default) and at the end of the call, and errors (non-finite velocity, extrapolation abort)
 * are returned then: the diagnostics and t stop at the last good step, while the fields are
 * those after the last ENQUEUED step (up to sync_every - 1 steps past the failing one; with
 * sync_every = 1, or a finite t_end, they are the failing step's).  The call returns once the
 * last step has finished on the stream. */
int rmt_sim_step(rmt_sim *sim, int nsteps, double t_end);
/* Carry (off by default): with on != 0, a call's last step also prepares what the next
 * step needs from the final state alone (the extrapolation geometry of its known plane, the
 * prep planes' constant-segment marks, max |u|^2 from the projection), and the next
 * rmt_sim_step starts from it -- its first step then costs what every later step costs.
 * The caller promises to call rmt_sim_invalidate after writing any field between calls; any
 * other use of the context's workspace between calls ends the carry by itself.  Results
 * are bit-identical either way. */
int rmt_sim_set_carry(rmt_sim *sim, int on);
int rmt_sim_invalidate(rmt_sim *sim);
/* Phase timers (HIP events on the context stream, accumulated over steps while on):
 * ms[0] dt reduction, [1] advection, [2] extrapolation, [3] momentum (prep + 4 stages +
 * BC), [4] projection, [5] diagnostics, [6] the four RK4 stage kernels alone,
 * [7] the extrapolation sweep kernel alone; calls[k] = number of timed intervals. */
int rmt_sim_set_profiling(rmt_sim *sim, int on);
int rmt_sim_phase_times(rmt_sim *sim, double *ms8, long *calls8);
/* Copy the diagnostics of all completed steps since creation (blocks). */
int rmt_sim_diagnostics(rmt_sim *sim, rmt_diag *out, int max_records, int *n_records);

/* ---- periodic branch (functions.py:1177-1290; tests/test_poisson.py:24-78) -----------
 * Overlap grid (x[-1] == x[0]): operators on the reduced (N-1)^2 sub-grid, tiled back.
 * lamx / lamy: HOST per-axis symbols -(sin(2 pi k / m) / h)^2, length m = N - 1. */
int rmt_divergence_periodic(rmt_ctx *ctx, const double *a, const double *b, double dx, double dy,
                            double *divU);                           /* functions.py:1236 */
int rmt_pressure_gradient_periodic(rmt_ctx *ctx, const double *p, double dx, double dy,
                                   double *gx, double *gy);          /* functions.py:1246 */
int rmt_solve_poisson_fft(rmt_ctx *ctx, const double *rhs, const double *lamx,
                          const double *lamy, double *p);            /* functions.py:1216 */
/* pressure_projection_amg(bc_type='periodic') (functions.py:1277-1290): rho_bar = mean rho
 * in the Poisson rhs; rho_cells (device, nullable) the local density of the correction */
int rmt_pressure_projection_periodic(rmt_ctx *ctx, const double *a_star, const double *b_star,
                                     double dx, double dy, double dt, double rho_bar,
                                     const double *rho_cells, int bc_kind, double lid,
                                     const double *lamx, const double *lamy,
                                     const double *p_prev, double *a, double *b, double *p);

/* ---- slab-decomposed step (the fused step over G GPUs, 1D row slabs) ----
 * One rmt_slab = rows [r0, r1) of the global ny x nx grid (row_splits[rank] ..
 * row_splits[rank+1]) plus RMT_SLAB_HALO resident rows on each side, and the column block
 * [col_splits[rank], col_splits[rank+1]) of the transposed DCT pass.  The caller
 * (pyrmt_amd/distributed.py) runs the phases below on every slab, in this order, and
 * performs the collectives named between them (torch.distributed over RCCL, or in-process
 * copies); the result is bit-identical to rmt_sim_step when every slab holds 2^m rows at a
 * multiple of 2^m (the row-tree means), and equal to rounding otherwise.
 * The ctx must be created for the GLOBAL grid; splits must be even and slabs >= HALO rows.
 * Replaces the loop body of soft_disc_in_lid_driven.py:206-235 (semi-Lagrangian, one disc).
 *   buffers: 0-6 u v p X1 X2 phi J (resident (hi-lo) x nx planes), 7 p_c plane,
 *            8 known bits (ny x W u64), 9 rim entries (3 doubles each), 10 DCT slab buffer
 *            (owned x nx), 11 DCT column buffer (ny x nc), 12 scalars (16 doubles:
 *            [0] max|u|^2 owned, [1..10] diag partials, [11] flags (1 non-finite velocity,
 *            2 halo overrun, 4 extrapolation abort), [12] rim count, [13] row-tree root,
 *            [14] cells fitted)
 *   info: r0, r1, lo, hi, c0, c1, W (64-cell words per row), HALO; and the constant dt. */
#define RMT_SLAB_HALO 12
typedef struct rmt_slab rmt_slab;
int rmt_slab_create(rmt_ctx *ctx, const rmt_sim_params *prm, int G, int rank,
                    const int *row_splits, const int *col_splits, rmt_slab **out);
int rmt_slab_destroy(rmt_slab *slab);
int rmt_slab_info(rmt_slab *slab, int *ints8, double *dt_const);
int rmt_slab_buffer(rmt_slab *slab, int id, void **dev_ptr);
int rmt_slab_begin(rmt_slab *slab);                      /* scal[0] of the initial state  */
/* optional, while the halo exchange is in flight: the advection of the rows that read no
 * halo row; rmt_slab_advect (after the halo) then does the remaining rows */
int rmt_slab_advect_interior(rmt_slab *slab, double dt);
int rmt_slab_advect(rmt_slab *slab, double dt);          /* then: allgather known bit rows */
int rmt_slab_rim_pack(rmt_slab *slab);                   /* then: allgather rim entries    */
int rmt_slab_extrapolate(rmt_slab *slab, const double *gathered, const long long *counts,
                         long long cap);                 /* gathered: G x cap x 3 (device) */
int rmt_slab_momentum(rmt_slab *slab, double dt);
int rmt_slab_project_rows(rmt_slab *slab, double dt);    /* then: all_to_all 10 -> 11      */
int rmt_slab_project_cols(rmt_slab *slab);               /* then: all_to_all 11 -> 10      */
int rmt_slab_project_unrows(rmt_slab *slab);             /* then: allgather scal[13]       */
int rmt_slab_sub_mean(rmt_slab *slab, int which, const double *roots_dev);  /* 0 p_c, 1 p */
int rmt_slab_project_correct(rmt_slab *slab, double dt); /* after halo(p_c); then roots   */
int rmt_slab_finish(rmt_slab *slab);                     /* then: allgather scal          */
/* Device-dt step (no host round trip inside the step; distributed.py's asynchronous path):
 * with on != 0 every phase reads dt from the slab's device scalar instead of its dt argument.
 * rmt_slab_next_dt: after the scalar allgather (G x 16 doubles, device), record
 * {dt, max|u|^2, the gathered blocks} into ring_slot (nullable, 2 + 16 G doubles) and set the
 * next dt from the gathered max|u|^2 -- the host's expression, NaN-propagating max.
 * rmt_slab_rim_pack + rmt_slab_rim_cap: the rim allgather moves a fixed `cap` entries per slab
 * (flag 8 in the scalar block's flags when a slab's rim is larger; the host raises);
 * rmt_slab_extrapolate_dev reads the counts from the gathered scalar blocks. */
int rmt_slab_set_device_dt(rmt_slab *slab, int on);
int rmt_slab_next_dt(rmt_slab *slab, const double *gathered_scal, int G, double *ring_slot);
int rmt_slab_rim_cap(rmt_slab *slab, long long cap);
/* The next step's extrapolation geometry beside this step's projection (as rmt_sim_step's
 * early geometry): after rmt_slab_momentum, rmt_slab_next_bits writes the owned rows of the
 * next known plane into buffer 13 (bits_next); the caller allgathers its rows; then
 * rmt_slab_geometry runs the value-independent extrapolation passes on the slab's second
 * stream, and the next step's rmt_slab_advect / rmt_slab_extrapolate* use them (no bits
 * allgather, no geometry on the critical path).  rmt_slab_drop_geometry forgets it (a step
 * that will not run).  Replaces the geometry half of extrapolate_reference_map
 * (functions.py:78-99: targets, acceptance, weights depend on the known set only). */
int rmt_slab_next_bits(rmt_slab *slab);
int rmt_slab_geometry(rmt_slab *slab);
int rmt_slab_drop_geometry(rmt_slab *slab);
int rmt_slab_extrapolate_dev(rmt_slab *slab, const double *gathered, const double *gathered_scal,
                             long long cap);

/* ---- MAC path (config 5): pyRMT/mac.py operators on an N x N cell grid -----------
 * ctx created for (N, N) cells; u is (N, N+1) x-faces, v (N+1, N) y-faces, p / phi (N, N). */
int rmt_mac_divergence(rmt_ctx *ctx, const double *u, const double *v, double dx, double dy,
                       double *out);                                       /* mac.py:81-84  */
int rmt_mac_gradient_p(rmt_ctx *ctx, const double *p, double dx, double dy, double *gu,
                       double *gv);                                        /* mac.py:87-101 */
/* lamx (nx) / lamy (ny): HOST per-axis eigenvalues (eig = lamx[None,:] + lamy[:,None], the
 * (0,0) mode zeroed), or both NULL for poisson_eigs_neumann's own (mac.py:104-115) */
int rmt_mac_solve_poisson_neumann(rmt_ctx *ctx, const double *rhs, double dx, double dy,
                                  const double *lamx, const double *lamy,
                                  double *out);                           /* mac.py:118-123 */
int rmt_mac_project(rmt_ctx *ctx, const double *u_star, const double *v_star, double dx,
                    double dy, double dt, double rho, const double *lamx, const double *lamy,
                    double *u, double *v, double *phi);                   /* mac.py:126-139 */
/* fu / fv: face forces or both NULL                                       mac.py:196-232 */
int rmt_mac_momentum_predictor(rmt_ctx *ctx, const double *u, const double *v, double nu,
                               double dx, double dy, double dt, double U_lid, const double *fu,
                               const double *fv, double rho, double *u_star, double *v_star);
int rmt_mac_contact_stress(rmt_ctx *ctx, const double *phi_a, const double *phi_b, double eta,
                           double Gsum, double eps, double dx, double dy, double *txx,
                           double *txy, double *tyy);                     /* mac.py:729-749 */
/* MAC IMEX tier (imex.hip), square N x N cell grid (ctx ny = nx = N).  kind 0: u faces, full
 * (N, N+1), interior (N, N-1); kind 1: v faces, full (N+1, N), interior (N-1, N).
 * rmt_mac_lap_lid_hom: the homogeneous-BC Laplacian of a full field on the interior faces,
 *   mac.py:243-250 _lap_u_lid_hom (kind 0) / :253-260 _lap_v_lid_hom (kind 1).
 * rmt_mac_helmholtz: (I - coef Lap_hom) x = rhs on the interior faces by scipy's cg
 *   (x0 = rhs, atol = rtol ||rhs||), precond 0: mac.py:263-275 _cg_helmholtz, precond 1:
 *   mac.py:287-316 _pcg_helmholtz (DST-II preconditioner); *iters = iterations run.
 * rmt_mac_momentum_predictor_lid_imex: mac.py:319-369; fu / fv full face forces or NULL;
 *   iters[2] (optional): the u and v PCG iteration counts. */
int rmt_mac_lap_lid_hom(rmt_ctx *ctx, int kind, const double *f, double dx, double dy,
                        double *out);
int rmt_mac_helmholtz(rmt_ctx *ctx, int kind, const double *rhs, double coef, double dx,
                      double dy, double rtol, int maxiter, int precond, double *x, int *iters);
int rmt_mac_momentum_predictor_lid_imex(rmt_ctx *ctx, const double *u, const double *v,
                                        double nu, double dx, double dy, double dt,
                                        double U_lid, const double *fu, const double *fv,
                                        double rho, double rtol, double cs2, double *u_star,
                                        double *v_star, int *iters);
/* mac.py:381-442 momentum_predictor_lid_semilag, its semi-Lagrangian branch (the caller
 * checked CFL > cfl_switch, mac.py:387-390): midpoint backtrace through cubic-spline
 * interpolation (scipy.ndimage.map_coordinates order 3, mode 'nearest', mac.py:374-378),
 * then the implicit viscosity by PCG; iters as above. */
int rmt_mac_momentum_predictor_lid_semilag(rmt_ctx *ctx, const double *u, const double *v,
                                           double nu, double dx, double dy, double dt,
                                           double U_lid, const double *fu, const double *fv,
                                           double rho, double cs2, double rtol, double *u_star,
                                           double *v_star, int *iters);

/* The loop body of benchmarks/mac_multi_disc_lid.py:62-98 (K soft discs with contact, lid
 * U_lid, fixed dt), device-resident.  Fields: 0 u, 1 v, 2 p (disc ignored); 3 X1, 4 X2,
 * 5 phi of disc `disc`. */
#define RMT_MAC_MAXD 8
typedef struct {
    int N;                   /* cells per side, dx = 1 / N                               */
    double dx;
    int n_discs;
    double R[RMT_MAC_MAXD], cx[RMT_MAC_MAXD], cy[RMT_MAC_MAXD];
    double U_lid, mu_s, mu_f, rho, eta;
    int layers;              /* extrapolation layers (3 in the driver)                   */
    double dt;               /* the driver's fixed step (mac_multi_disc_lid.py:58)        */
} rmt_mac_params;
typedef struct {
    double t, dt, minJ, maxJ, umax;
    int n_discs;
    double cx[RMT_MAC_MAXD], cy[RMT_MAC_MAXD];   /* centroid of phi_k <= 0 (:104)        */
    int diverged;   /* mac_multi_disc_lid.py:100-103: u non-finite, min J < 0, max J > 20 or a
                       disc with no phi <= 0 cell after this step; the sim stops stepping     */
} rmt_mac_diag;
typedef struct rmt_mac_sim rmt_mac_sim;
/* rmt_mac_sim_step stops after a step whose record has diverged set (the reference driver
 * breaks out of its loop there); later calls are no-ops.  RMT_EDEVICE on an extrapolation
 * abort, RMT_ENONFINITE on a non-finite velocity fed to the advection. */
int rmt_mac_sim_create(rmt_ctx *ctx, const rmt_mac_params *prm, rmt_mac_sim **out);
int rmt_mac_sim_destroy(rmt_mac_sim *sim);
int rmt_mac_sim_field(rmt_mac_sim *sim, int field, int disc, double **dev_ptr);
int rmt_mac_sim_step(rmt_mac_sim *sim, int nsteps, double t_end);
int rmt_mac_sim_diagnostics(rmt_mac_sim *sim, rmt_mac_diag *out, int max_records,
                            int *n_records);

/* The MAC step decomposed into row slabs (config 5 on several GPUs).
 * No reference interface: pyRMT runs mac_multi_disc_lid.py:62-98 in one process.  Slab
 * `rank` of G owns cell rows [row_splits[rank], row_splits[rank+1]) (even, > RMT_SLAB_HALO
 * rows each) and column block [col_splits[rank], col_splits[rank+1]) of the transposed
 * Poisson solve; ctx is the global N x N context.  The caller drives the phases and the
 * collectives between them (order in mac.hip; pyrmt_amd/distributed.py MacDistributedSim).
 * Buffers (rmt_mac_slab_buffer ids): 0 u ((hi-lo) x (N+1)), 1 v ((hi-lo+1) x N, face rows
 * lo..hi), 2 p, 3 X1[disc], 4 X2[disc], 5 phi[disc] ((hi-lo) x N), 6 known bits[disc]
 * (N x W words), 7 rim[disc] (owned cells x 3), 8 A, 9 B (transpose blocks), 10 scalars
 * (RMT_MAC_SLAB_SCALARS doubles: [0] flags 1 non-finite / 2 halo / 4 extrapolation abort,
 * [1] min J, [2] max J, [3] max|u|, [4 + 3k ..] disc k centroid sums (x, y, count),
 * [28 + k] rim count of disc k, [36] row-tree root, [37] cells fitted, [38 + k] 1 if
 * an extrapolation target of disc k in the owned rows fits (0 on every slab: the disc's
 * extrapolation is the identity, rmt_mac_slab_extrapolate_identity replaces the rim
 * allgather + rmt_mac_slab_extrapolate)). */
#define RMT_MAC_SLAB_SCALARS 48
typedef struct rmt_mac_slab rmt_mac_slab;
int rmt_mac_slab_create(rmt_ctx *ctx, const rmt_mac_params *prm, int G, int rank,
                        const int *row_splits, const int *col_splits, rmt_mac_slab **out);
int rmt_mac_slab_destroy(rmt_mac_slab *slab);
int rmt_mac_slab_info(rmt_mac_slab *slab, int *ints8);   /* r0 r1 lo hi c0 c1 W halo */
int rmt_mac_slab_buffer(rmt_mac_slab *slab, int id, int disc, void **dev_ptr);
int rmt_mac_slab_advect(rmt_mac_slab *slab, double dt);
int rmt_mac_slab_rim_pack(rmt_mac_slab *slab);
int rmt_mac_slab_extrapolate(rmt_mac_slab *slab, int disc, const double *gathered_rims,
                             const long long *counts, long long cap);
int rmt_mac_slab_extrapolate_identity(rmt_mac_slab *slab, int disc);
int rmt_mac_slab_predict(rmt_mac_slab *slab, double dt);
int rmt_mac_slab_project_rows(rmt_mac_slab *slab, const double *dev_roots);
int rmt_mac_slab_project_cols(rmt_mac_slab *slab);
int rmt_mac_slab_project_unrows(rmt_mac_slab *slab);
int rmt_mac_slab_correct(rmt_mac_slab *slab, double dt);

#ifdef __cplusplus
}
#endif
#endif /* RMT_H */
