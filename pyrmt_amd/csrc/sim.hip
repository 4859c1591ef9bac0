// sim.hip -- the RMT loop body of the reference drivers as one device-resident step.
//
// benchmarks/soft_disc_in_lid_driven.py:206-235 (configs 2/4), disc_in_taylor_green.py
// :206-242 (config 3) and lid_driven_cavity.py:58-80 (config 1):
//   dt = compute_timestep(u);  clip to t_end
//   phi = rebuild(X1, X2); mask = phi <= 0
//   X1, X2 = advect(X1, X2) * mask;  extrapolate(X1, X2, phi)
//   phi = rebuild(X1, X2)
//   u*, v* = momentum_step_rk4(...);  u, v, p = pressure_projection(u*, v*, p)
//   diagnostics: centroid of phi <= 0, J min/max (+ KE, SE, dissipation)
// State (u, v, p, X1, X2) stays in HBM; one host sync per step reads dt.
#include "rmt_internal.hpp"
#include <utility>
#include <vector>

namespace rmt {

// Test switches RMT_TEST_DELAY_SIDE / RMT_TEST_DELAY_MAIN = <n>: a one-thread kernel that
// sleeps ~3.4 us x n on the second stream as it starts this step's work beside the chain, or
// on the critical stream right after the chain.  Every cross-stream dependency is an event,
// so shifting either stream's timing must leave the results bit-identical
// (tests/test_gpu_env_variants.py: the regression test for stream hazards).
__global__ void k_delay(int n) {
    for (int k = 0; k < n; ++k) __builtin_amdgcn_s_sleep(127);
}



constexpr int DIAG_VALS = 10, DIAG_BLOCKS = 512, DIAG_T = 256;
// ring record: [0, DIAG_VALS) the diagnostics, then max |u|^2, dt, the 4 step flags
constexpr int RING_N = 64, RING_VALS = DIAG_VALS + 6;

}  // namespace rmt

struct rmt_sim {
    rmt_ctx *ctx = nullptr;
    rmt_sim_params P{};
    double *xs = nullptr, *ys = nullptr;
    // fields
    double *u = nullptr, *v = nullptr, *p = nullptr, *X1 = nullptr, *X2 = nullptr;
    double *phi = nullptr, *phi_pre = nullptr, *J = nullptr;
    double *X1n = nullptr, *X2n = nullptr, *us = nullptr, *vs = nullptr;
    double *X1h = nullptr, *X2h = nullptr;   // the map buffers rmt_sim_field hands out
    double *sxx = nullptr, *sxy = nullptr, *syy = nullptr;
    double *mw = nullptr;            // momentum workspace (8 planes)
    unsigned long long *kbits = nullptr;   // known plane (phi_pre < 0) from k_sim_sl
    unsigned char *mbytes = nullptr; // solid mask + flag
    double *dscr = nullptr;          // diag partials + scalars
    int *flag = nullptr;             // non-finite flag
    double dt_const = 0, t = 0, integ = 0;
    std::vector<rmt_diag> diag;
    void *block = nullptr;
    // overlap of the (one-CU) extrapolation chain with a speculative momentum pass
    hipStream_t st2 = nullptr;
    // the step's own stream at the highest priority (RMT_SIM_HIPRIO, default on), joined to the
    // caller's stream at entry and exit: the critical path's kernels are dispatched ahead of
    // the second stream's whenever both have work ready
    hipStream_t st1 = nullptr;
    hipEvent_t e_in = nullptr, e_out = nullptr;
    hipEvent_t e_sl = nullptr, e_mom = nullptr, e_rows = nullptr;
    int *tiles = nullptr, *tcount = nullptr, max_tiles = 0;
    // device-resident dt and diagnostics (rmt_sim_step's asynchronous path): per-block
    // max |u|^2 partials from the projection, and a ring of per-step records read back once
    // per RING_N steps
    double *m2part = nullptr, *ring = nullptr;
    int m2n = 0;
    // the projection's row pass runs beside the chain; only the rows of the fix-up tiles
    // (+-1 for the Rhie-Chow stencil) are redone after it
    unsigned char *rowmark = nullptr;
    // per 64 x 16 fix-up tile: listed this step (k_mark_rows; the diagnostics read those tiles
    // whole, k_diag_seg)
    unsigned char *tmark = nullptr;
    bool split_proj = false;
    // the advection split: the rim cells (within 7 of the known/unknown interface, all the
    // extrapolation reads) before the chain, the rest beside it on the second stream
    unsigned long long *rimw = nullptr;
    int *rimcnt = nullptr;
    hipEvent_t e_bits = nullptr, e_proj = nullptr, e_tail = nullptr, e_kb = nullptr, e_geo = nullptr;
    hipEvent_t e_tailp = nullptr;   // the pressure update done (tail_stream)
    // the next step's known plane, written by the phi kernels of this step (nx % 64 == 0):
    // double-buffered with kbits, valid from the second step of a call on
    unsigned long long *kbits_next = nullptr;
    bool bits_ready = false;
    // k_mom_prep's per-segment skip flags (MomWork::prep_const), cleared at each call's start
    unsigned char *pconst = nullptr;
    // zero-tile flags of the two map buffers (k_sim_sl_t, sl_zero_flags): zf[zcur] belongs to
    // the buffer X1 / X2 point at, zf[zcur ^ 1] to X1n / X2n; zv: written in this call
    unsigned char *zf[2] = {nullptr, nullptr};
    int zcur = 0;
    bool zv[2] = {false, false};
    int *segs = nullptr;     // rim row segments (k_rim_segments): ny * ceil(nx / 256) + count
    unsigned long long *m2acc = nullptr;   // k_dt_part's atomic max + block counter (zeroed)
    bool prof = false;
    int sync_every = rmt::RING_N;   // rmt_sim_set_sync_every
    // rmt_sim_set_carry: a call's last step also prepares the next step's geometry (and its
    // projection's max |u|^2 partials stay valid), and the next call starts from them unless
    // rmt_sim_invalidate or another user of the context's workspace came in between
    bool carry_on = false, carry_valid = false, m2_valid = false;
    unsigned long carry_gen = 0, carry_cfg = 0;   // workspace / extrapolation config generations
    hipEvent_t pev[7] = {};
    double ms[8] = {};
    long calls[8] = {};
};

namespace rmt {

// SL advection of (X1, X2) with the pre-advection level set and mask (one pass).
// One 256-cell row segment (j, i0) of the SL advection of (X1, X2) with the pre-advection
// level set and mask.  A wave covers 64 cells of one row, so the extrapolation's known plane
// (phi_pre < 0, 64-cell words) comes out of the same pass (kbits optional).  mode 1: only the
// rim cells (rimw), mode 2: every other cell -- the same per-cell result, split so that the
// extrapolation can start after the (small) rim part.  Block-uniform control flow (the zero
// test is a block reduction).
__device__ __forceinline__ void sl_segment(
    const double *__restrict__ X1, const double *__restrict__ X2, const double *__restrict__ a,
    const double *__restrict__ b, const double *__restrict__ xs, const double *__restrict__ ys,
    int ny, int nx, double dt, const DivK &Kx, const DivK &Ky, double x0, double y0, double R,
    double *__restrict__ X1n, double *__restrict__ X2n, double *__restrict__ phi_pre, int *bad,
    unsigned long long *__restrict__ kbits, const double *m2, int mode,
    const unsigned long long *__restrict__ rimw, int j, int i0) {
    const int i = i0 + threadIdx.x;
    const bool in = i < nx;
    const long c = (long)j * nx + i;
    bool mine = true;
    if (mode) {
        const bool rim = in && ((rimw[(long)j * ((nx + 63) / 64) + (i >> 6)] >> (i & 63)) & 1);
        mine = (mode == 1) == rim;
    }
    // (a rim segment -- mode 1 -- borders the solid: its map is never +0.0 throughout, so
    // the zero test's extra global round trip is skipped there)
    const bool zero = mode != 1 && sl_skip_ok(m2, dt, fmin(Kx.d, Ky.d)) &&
                      sl_zero_block(X1, X2, ny, nx, j, i0, 256, 0, ny);
    bool known = false;
    if (in && zero) {
        // the map is +0.0 here: phi of the origin, advected map +0.0 (no loads); phi_pre
        // only when no known plane is produced (its only reader is then the extrapolation)
        const double ph = disc_phi(0.0, 0.0, x0, y0, R);
        if (!kbits && !mode) phi_pre[c] = ph;
        known = ph < 0;
        if (mine) { X1n[c] = 0.0; X2n[c] = 0.0; }
    } else if (in && mine) {
        bool fin = isfinite(a[c]) && isfinite(b[c]);
        if (!fin) atomicOr(bad, 1);
        double ph = disc_phi(X1[c], X2[c], x0, y0, R);
        if (!kbits && !mode) phi_pre[c] = ph;
        known = ph < 0;
        {
            double m = ph <= 0 ? 1.0 : 0.0;
            double xb, yb;
            sl_backtrace_t<false>(a, b, xs[i], ys[j], dt, Kx, Ky, nx, ny, 0, ny, nullptr, xb, yb);
            X1n[c] = bilinear_t<false>(X1, xb, yb, Kx, Ky, nx, ny, 0, ny, nullptr) * m;
            X2n[c] = bilinear_t<false>(X2, xb, yb, Kx, Ky, nx, ny, 0, ny, nullptr) * m;
        }
    }
    if (kbits) {
        const unsigned long long w = __ballot(known);
        if ((threadIdx.x & 63) == 0 && (i >> 6) < (nx + 63) / 64)
            kbits[(long)j * ((nx + 63) / 64) + (i >> 6)] = w;
    }
}

// grid (ceil(nx / 256), ny)
__global__ void k_sim_sl(const double *__restrict__ X1, const double *__restrict__ X2,
                         const double *__restrict__ a, const double *__restrict__ b,
                         const double *__restrict__ xs, const double *__restrict__ ys, int ny,
                         int nx, double dt_arg, DivK Kx, DivK Ky, int shape, double x0,
                         double y0, double R, double *__restrict__ X1n, double *__restrict__ X2n,
                         double *__restrict__ phi_pre, int *bad,
                         unsigned long long *__restrict__ kbits, const double *m2,
                         const double *__restrict__ dtp = nullptr, int mode = 0,
                         const unsigned long long *__restrict__ rimw = nullptr) {
    (void)shape;
    const double dt = dtp ? *dtp : dt_arg;
    sl_segment(X1, X2, a, b, xs, ys, ny, nx, dt, Kx, Ky, x0, y0, R, X1n, X2n, phi_pre, bad, kbits,
               m2, mode, rimw, blockIdx.y, blockIdx.x * 256);
}

// Tiled SL advection (modes 0 and 2 of sl_segment, same per-cell arithmetic): a 64 x 4 tile
// stages X1, X2 and -- unless the tile is certified +0.0 -- the velocity on the tile + (1, 2)
// in LDS, so the RK4 backtrace's four dependent velocity gathers and the foot's map samples
// are LDS reads instead of four-plus-one dependent global round trips.  The staged region is
// exactly the union of the tile cells' zero-test neighbourhoods (rows j-1 .. j+2, columns
// i-1 .. i+2 of sl_zero_block), which holds every bilinear stencil when dt sqrt(m2) <= 0.9 h;
// a stencil outside it (a larger velocity) reads global memory: the same values either way.
constexpr int SLT_X = 64, SLT_Y = 4, SLT_SX = SLT_X + 3, SLT_SY = SLT_Y + 3;

// interpolators.py:4-61 at one query point (bilinear_t<false>), corners from the staged
// tile s (origin row sj0, column si0) when they lie in it, else from g
// FACE: g is a MAC face plane and a cell's value the mean of its two faces (mac.py's cell
// centre velocity, k_mac_centres_m2's expression): V 0 = u (nx + 1 faces a row), 1 = v (a
// row of nx faces, one row more)
template <int FACE, int V>
__device__ __forceinline__ double cell_vel(const double *__restrict__ g, int jj, int ii, int nx) {
    if constexpr (!FACE) return g[(long)jj * nx + ii];
    else if constexpr (V == 0) {
        const long f = (long)jj * (nx + 1) + ii;
        return 0.5 * (g[f] + g[f + 1]);
    } else {
        const long f = (long)jj * nx + ii;
        return 0.5 * (g[f] + g[f + nx]);
    }
}
template <int FACE = 0, int V = 0>
__device__ __forceinline__ double bl_tile(const double *__restrict__ s,
                                          const double *__restrict__ g, double xq, double yq,
                                          const DivK &Kx, const DivK &Ky, int nx, int ny,
                                          int sj0, int si0) {
    double x = divk(xq, Kx), y = divk(yq, Ky);
    if (!(isfinite(x) && isfinite(y))) return __builtin_nan("");
    if (x < 0.0) x = 0.0; else if (x > nx - 1.0) x = nx - 1.0;
    if (y < 0.0) y = 0.0; else if (y > ny - 1.0) y = ny - 1.0;
    int ix = (int)floor(x), iy = (int)floor(y);
    if (ix >= nx - 1) ix = nx - 2;
    if (iy >= ny - 1) iy = ny - 2;
    const double fx = x - ix, fy = y - iy;
    const int lx = ix - si0, ly = iy - sj0;
    double v00, v10, v01, v11;
    if ((unsigned)lx < (unsigned)(SLT_SX - 1) && (unsigned)ly < (unsigned)(SLT_SY - 1)) {
        const double *r0 = s + ly * SLT_SX + lx, *r1 = r0 + SLT_SX;
        v00 = r0[0]; v10 = r0[1]; v01 = r1[0]; v11 = r1[1];
    } else if constexpr (FACE) {
        v00 = cell_vel<FACE, V>(g, iy, ix, nx); v10 = cell_vel<FACE, V>(g, iy, ix + 1, nx);
        v01 = cell_vel<FACE, V>(g, iy + 1, ix, nx); v11 = cell_vel<FACE, V>(g, iy + 1, ix + 1, nx);
    } else {
        const double *r0 = g + (long)iy * nx + ix, *r1 = r0 + nx;
        v00 = r0[0]; v10 = r0[1]; v01 = r1[0]; v11 = r1[1];
    }
    return (1 - fx) * (1 - fy) * v00 + fx * (1 - fy) * v10 + (1 - fx) * fy * v01 + fx * fy * v11;
}

// grid ((nx + 63) / 64, (ny + 3) / 4); mode 0 (kbits optional) or 2 (the non-rim cells).
// FACE: a, b are the MAC u / v face planes (cell_vel), nx == ny
template <int FACE>
__device__ __forceinline__ void sl_tile(
    const double *__restrict__ X1, const double *__restrict__ X2, const double *__restrict__ a,
    const double *__restrict__ b, const double *__restrict__ xs, const double *__restrict__ ys,
    int ny, int nx, double dt, const DivK &Kx, const DivK &Ky, double x0, double y0, double R,
    double *__restrict__ X1n, double *__restrict__ X2n, double *__restrict__ phi_pre, int *bad,
    unsigned long long *__restrict__ kbits, const double *m2, int mode,
    const unsigned long long *__restrict__ rimw, double *__restrict__ phi, double thr,
    unsigned char *__restrict__ fbits, unsigned long long *__restrict__ nbits,
    const unsigned char *__restrict__ zin, unsigned char *__restrict__ zout, int zout_ok,
    int tcol, int trow, double *s1, double *s2, double *sa, double *sb) {
    const int i0 = tcol * SLT_X, j0 = trow * SLT_Y;
    const int tx = threadIdx.x & (SLT_X - 1), ty = threadIdx.x / SLT_X;
    const int i = i0 + tx, j = j0 + ty, sj0 = j0 - 1, si0 = i0 - 1;
    const bool in = i < nx && j < ny;
    const long c = (long)j * nx + i;
    // Zero-tile flags (mode 2 with phi, nx % 64 == 0; sl_zero_flags).  zout[t] = 1 when this
    // pass took the zero branch on tile t and the tile holds no rim cell: only this pass writes
    // its non-rim cells, so after the step the tile's map is +0.0 in every cell and its phi is
    // disc_phi(0, 0) (the fix-up prep recomputes the same value from the same +0.0).  zin: those
    // flags of the input map (the previous step's output buffer), zout_ok: zout still holds the
    // output buffer's flags from the step that last wrote it.  When the 3 x 3 tiles around a
    // tile (every cell the staged region reads) are flagged in zin, the tile holds no rim cell
    // and the velocity bound holds, the zero test's answer is known without its loads; the
    // advected map's +0.0 and phi's constant are then written only where the buffers may hold
    // something else.  The bits of every plane are those of the pass without the flags.
    const int TW = (nx + SLT_X - 1) / SLT_X, TH = (ny + SLT_Y - 1) / SLT_Y;
    const long tid = (long)trow * TW + tcol;
    bool tile_rim = false, z = false, dst_zero = false;
    if (zout) {
        // every flag load issued at once (one round trip): the tile's rim words, the input
        // flags of the 3 x 3 tiles around it (off the grid: +0.0, as the staging reads them),
        // the output buffer's flag
        const int W = (nx + 63) / 64;
        unsigned long long rw = 0;
#pragma unroll
        for (int r = 0; r < SLT_Y; ++r)
            rw |= j0 + r < ny ? rimw[(long)(j0 + r) * W + (i0 >> 6)] : 0ull;
        unsigned zf = 1;
        if (zin) {
#pragma unroll
            for (int dr = -1; dr <= 1; ++dr)
#pragma unroll
                for (int dc = -1; dc <= 1; ++dc) {
                    const int r = trow + dr, cc = tcol + dc;
                    zf &= (r >= 0 && r < TH && cc >= 0 && cc < TW) ? zin[(long)r * TW + cc] : 1u;
                }
        }
        dst_zero = zout_ok && zout[tid];
        tile_rim = rw != 0;
        z = zin && zf && !tile_rim;
    }
    if (z && sl_skip_ok(m2, dt, fmin(Kx.d, Ky.d))) {
        {
            const double ph = disc_phi(0.0, 0.0, x0, y0, R);
            if (in) {
                if (!dst_zero) { X1n[c] = 0.0; X2n[c] = 0.0; }
                if (!zin[tid]) phi[c] = ph;
            }
            if (kbits) {
                const unsigned long long w = __ballot(in && ph < 0);
                if (tx == 0 && j < ny) kbits[(long)j * ((nx + 63) / 64) + (i0 >> 6)] = w;
            }
            if (nbits) {
                const unsigned long long wn = __ballot(in && ph < 0);
                if (tx == 0 && j < ny) nbits[(long)j * (nx >> 6) + (i0 >> 6)] = wn;
            }
            const unsigned long long w = __ballot(!in || ph > thr);
            if (tx == 0 && j < ny)
                fbits[(long)j * (nx >> 6) + (i0 >> 6)] =
                    (unsigned char)((w == ~0ull) | (((w & 3ull) == 3ull) << 1) | (((w >> 62) == 3ull) << 2));
            __syncthreads();   // (every wave has read zout[tid])
            if (threadIdx.x == 0) zout[tid] = 1;
            return;
        }
    }
    unsigned long long bits = 0;
    for (int q = threadIdx.x; q < SLT_SY * SLT_SX; q += SLT_X * SLT_Y) {
        const int jj = sj0 + q / SLT_SX, ii = si0 + q % SLT_SX;
        double v1 = 0.0, v2 = 0.0;
        if (jj >= 0 && jj < ny && ii >= 0 && ii < nx) {
            const long g = (long)jj * nx + ii;
            v1 = X1[g]; v2 = X2[g];
        }
        s1[q] = v1; s2[q] = v2;
        bits |= (unsigned long long)__double_as_longlong(v1) |
                (unsigned long long)__double_as_longlong(v2);
    }
    // the staged region is the zero test's (clipped to the grid): rows j0-1 .. j0+5, columns
    // i0-1 .. i0+65 (sl_zero_block over the tile's cells)
    const bool nonzero = __syncthreads_or(bits != 0);
    const bool zero = sl_skip_ok(m2, dt, fmin(Kx.d, Ky.d)) && !nonzero;
    bool mine = true;
    if (mode) {
        const bool rim = in && ((rimw[(long)j * ((nx + 63) / 64) + (i >> 6)] >> (i & 63)) & 1);
        mine = !rim;
    }
    bool known = false;
    double o1 = 0.0, o2 = 0.0;   // this cell's advected map, when mine (phi below)
    if (zero) {
        if (in) {
            const double ph = disc_phi(0.0, 0.0, x0, y0, R);
            if (!kbits && !mode) phi_pre[c] = ph;
            known = ph < 0;
            if (mine) { X1n[c] = 0.0; X2n[c] = 0.0; }
        }
    } else {
        for (int q = threadIdx.x; q < SLT_SY * SLT_SX; q += SLT_X * SLT_Y) {
            const int jj = sj0 + q / SLT_SX, ii = si0 + q % SLT_SX;
            double va = 0.0, vb = 0.0;
            if (jj >= 0 && jj < ny && ii >= 0 && ii < nx) {
                va = cell_vel<FACE, 0>(a, jj, ii, nx); vb = cell_vel<FACE, 1>(b, jj, ii, nx);
            }
            sa[q] = va; sb[q] = vb;
        }
        __syncthreads();
        if (in) {
            const int o = (ty + 1) * SLT_SX + tx + 1;
            const double ph = disc_phi(s1[o], s2[o], x0, y0, R);
            if (!kbits && !mode) phi_pre[c] = ph;
            known = ph < 0;
            if (mine) {
                if (!(isfinite(sa[o]) && isfinite(sb[o]))) atomicOr(bad, 1);
                const double m = ph <= 0 ? 1.0 : 0.0;
#define BT_(S, G, X, Y) bl_tile(S, G, X, Y, Kx, Ky, nx, ny, sj0, si0)
#define BTA_(X, Y) bl_tile<FACE, 0>(sa, a, X, Y, Kx, Ky, nx, ny, sj0, si0)
#define BTB_(X, Y) bl_tile<FACE, 1>(sb, b, X, Y, Kx, Ky, nx, ny, sj0, si0)
                // functions.py:194-227 (sl_backtrace_t's operations, in order)
                const double x = xs[i], y = ys[j], hdt = 0.5 * dt, dt6 = dt / 6.0;
                const double k1x = BTA_(x, y), k1y = BTB_(x, y);
                const double x2 = x - hdt * k1x, y2 = y - hdt * k1y;
                const double k2x = BTA_(x2, y2), k2y = BTB_(x2, y2);
                const double x3 = x - hdt * k2x, y3 = y - hdt * k2y;
                const double k3x = BTA_(x3, y3), k3y = BTB_(x3, y3);
                const double x4 = x - dt * k3x, y4 = y - dt * k3y;
                const double k4x = BTA_(x4, y4), k4y = BTB_(x4, y4);
                const double xb = x - dt6 * (k1x + 2 * k2x + 2 * k3x + k4x);
                const double yb = y - dt6 * (k1y + 2 * k2y + 2 * k3y + k4y);
                o1 = BT_(s1, X1, xb, yb) * m;
                o2 = BT_(s2, X2, xb, yb) * m;
                X1n[c] = o1;
                X2n[c] = o2;
#undef BT_
#undef BTA_
#undef BTB_
            }
        }
    }
    if (kbits) {
        const unsigned long long w = __ballot(known);
        if (tx == 0 && j < ny) kbits[(long)j * ((nx + 63) / 64) + (i0 >> 6)] = w;
    }
    if (phi) {
        // k_phi_rebuild_fluid's phi from the map this pass leaves (a rim cell's as the rim
        // pass and the chain have it: read back, as that kernel reads it), and the pure-fluid
        // test of each cell as bits per (row, 64-column tile): bit 0 every cell, bit 1 columns
        // 0-1, bit 2 columns 62-63 (k_fluid_rows_bits adds the neighbours' halo columns).
        // One wave is one row of the tile (nx % 64 == 0).
        // nbits (nullable): k_phi_rebuild_fluid's known-plane words of this map
        bool ok = true, neg = false;
        if (in) {
            const double a1 = mine ? o1 : X1n[c], a2 = mine ? o2 : X2n[c];
            const double ph = disc_phi(a1, a2, x0, y0, R);
            phi[c] = ph;
            ok = ph > thr;   // (NaN phi is not fluid)
            neg = ph < 0;
        }
        if (nbits) {
            const unsigned long long wn = __ballot(neg);
            if (tx == 0 && j < ny) nbits[(long)j * (nx >> 6) + (i0 >> 6)] = wn;
        }
        const unsigned long long w = __ballot(ok);
        if (tx == 0 && j < ny)
            fbits[(long)j * (nx >> 6) + (i0 >> 6)] =
                (unsigned char)((w == ~0ull) | (((w & 3ull) == 3ull) << 1) | (((w >> 62) == 3ull) << 2));
    }
    if (zout && threadIdx.x == 0) zout[tid] = zero && !tile_rim;
}

// grid ((nx + 63) / 64, (ny + 3) / 4): one tile per workgroup, (tbx0, tby0) the tile of block
// (0, 0) for a launch over a box of tiles.  mode 0 (kbits optional) or 2 (the non-rim cells).
// FACE: a, b are the MAC u / v face planes (cell_vel), nx == ny.  (A fixed grid walking the
// tiles measured slower: 89 VGPRs, 5 waves per SIMD.)
template <int FACE = 0>
__global__ void __launch_bounds__(SLT_X * SLT_Y) k_sim_sl_t(
    const double *__restrict__ X1, const double *__restrict__ X2, const double *__restrict__ a,
    const double *__restrict__ b, const double *__restrict__ xs, const double *__restrict__ ys,
    int ny, int nx, double dt_arg, DivK Kx, DivK Ky, double x0, double y0, double R,
    double *__restrict__ X1n, double *__restrict__ X2n, double *__restrict__ phi_pre, int *bad,
    unsigned long long *__restrict__ kbits, const double *m2, const double *__restrict__ dtp,
    int mode, const unsigned long long *__restrict__ rimw, double *__restrict__ phi = nullptr,
    double thr = 0.0, unsigned char *__restrict__ fbits = nullptr,
    unsigned long long *__restrict__ nbits = nullptr, int tbx0 = 0, int tby0 = 0,
    const unsigned char *__restrict__ zin = nullptr, unsigned char *__restrict__ zout = nullptr,
    int zout_ok = 0) {
    __shared__ double s1[SLT_SY * SLT_SX], s2[SLT_SY * SLT_SX];
    __shared__ double sa[SLT_SY * SLT_SX], sb[SLT_SY * SLT_SX];
    const double dt = dtp ? *dtp : dt_arg;
#define SLT_ARGS(TC, TR) X1, X2, a, b, xs, ys, ny, nx, dt, Kx, Ky, x0, y0, R, X1n, X2n, phi_pre, \
        bad, kbits, m2, mode, rimw, phi, thr, fbits, nbits, zin, zout, zout_ok, TC, TR, s1, s2, sa, sb
    sl_tile<FACE>(SLT_ARGS(blockIdx.x + tbx0, blockIdx.y + tby0));
#undef SLT_ARGS
}

// the row segments holding a rim cell, listed (any order)
__global__ void __launch_bounds__(256) k_rim_segments(const unsigned long long *__restrict__ rimw,
                                                      int ny, int nx, int *__restrict__ list,
                                                      int *__restrict__ count) {
    const int nbx = (nx + 255) / 256, W = (nx + 63) / 64;
    const long id = blockIdx.x * 256L + threadIdx.x;
    if (id >= (long)ny * nbx) return;
    const int j = (int)(id / nbx), bx = (int)(id % nbx);
    unsigned long long any = 0;
    for (int w = 4 * bx; w < min(4 * bx + 4, W); ++w) any |= rimw[(long)j * W + w];
    if (any) list[atomicAdd(count, 1)] = (int)id;
}
// mode 1 over the listed segments: a fixed grid walking the list (its length is on the
// device only)
__global__ void k_sim_sl_rim(const double *__restrict__ X1, const double *__restrict__ X2,
                             const double *__restrict__ a, const double *__restrict__ b,
                             const double *__restrict__ xs, const double *__restrict__ ys,
                             int ny, int nx, double dt_arg, DivK Kx, DivK Ky, double x0,
                             double y0, double R, double *__restrict__ X1n,
                             double *__restrict__ X2n, int *bad, const double *m2,
                             const double *__restrict__ dtp,
                             const unsigned long long *__restrict__ rimw,
                             const int *__restrict__ list, const int *__restrict__ count) {
    const double dt = dtp ? *dtp : dt_arg;
    const int nbx = (nx + 255) / 256, cnt = *count;
    for (int k = blockIdx.x; k < cnt; k += gridDim.x) {
        const int id = list[k];
        sl_segment(X1, X2, a, b, xs, ys, ny, nx, dt, Kx, Ky, x0, y0, R, X1n, X2n, nullptr, bad,
                   nullptr, m2, 1, rimw, id / nbx, (id % nbx) * 256);
    }
}

// the known plane alone (phi of the pre-advection map < 0: k_sim_sl's `known`), 64-cell words
__global__ void __launch_bounds__(256) k_sim_bits(const double *__restrict__ X1,
                                                  const double *__restrict__ X2, int nx,
                                                  double x0, double y0, double R,
                                                  unsigned long long *__restrict__ kbits) {
    const int j = blockIdx.y, i = blockIdx.x * 256 + threadIdx.x;
    const long c = (long)j * nx + i;
    const bool known = i < nx && disc_phi(X1[c], X2[c], x0, y0, R) < 0;
    const unsigned long long w = __ballot(known);
    if ((threadIdx.x & 63) == 0 && (i >> 6) < (nx + 63) / 64)
        kbits[(long)j * ((nx + 63) / 64) + (i >> 6)] = w;
}

// k_sim_sl with the bicubic interpolant (functions.py:228-251, scheme semilagrangian_cubic)
__global__ void k_sim_sl_cubic(const double *__restrict__ X1, const double *__restrict__ X2,
                               const double *__restrict__ a, const double *__restrict__ b,
                               const double *__restrict__ xs, const double *__restrict__ ys,
                               int ny, int nx, double dt, double dx, double dy, double x0,
                               double y0, double R, double *__restrict__ X1n,
                               double *__restrict__ X2n, double *__restrict__ phi_pre, int *bad) {
    long c = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (c >= (long)ny * nx) return;
    int j = (int)(c / nx), i = (int)(c % nx);
    bool fin = isfinite(a[c]) && isfinite(b[c]);
    if (__any(!fin) && (threadIdx.x & 63) == 0) atomicOr(bad, 1);
    double ph = disc_phi(X1[c], X2[c], x0, y0, R);
    phi_pre[c] = ph;
    double m = ph <= 0 ? 1.0 : 0.0;
    double xb, yb;
    sl_backtrace_cubic(a, b, xs[i], ys[j], dt, dx, dy, nx, ny, xb, yb);
    X1n[c] = bicubic(X1, xb, yb, dx, dy, nx, ny) * m;
    X2n[c] = bicubic(X2, xb, yb, dx, dy, nx, ny) * m;
}

__global__ void k_sim_phi_mask(const double *__restrict__ X1, const double *__restrict__ X2,
                               const double *__restrict__ a, const double *__restrict__ b,
                               long n, double x0, double y0, double R,
                               double *__restrict__ phi_pre, int *bad) {
    long c = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (c >= n) return;
    bool fin = isfinite(a[c]) && isfinite(b[c]);
    if (__any(!fin) && (threadIdx.x & 63) == 0) atomicOr(bad, 1);
    phi_pre[c] = disc_phi(X1[c], X2[c], x0, y0, R);
}

__global__ void k_mask_mul(double *__restrict__ X1, double *__restrict__ X2,
                           const double *__restrict__ phi, long n) {
    long c = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (c >= n) return;
    double m = phi[c] <= 0 ? 1.0 : 0.0;
    X1[c] = X1[c] * m;
    X2[c] = X2[c] * m;
}

// phi = rebuild(X1n, X2n) (functions.py:1366) fused with the copy of the extrapolated
// map back into the state planes (keeps rmt_sim_field pointers stable).
// nbits (nullable; nx % 64 == 0): the known plane of the NEXT step's advection, phi < 0 of
// this map (k_sim_bits' bits), one 64-cell word per wave
__global__ void k_phi_rebuild(const double *__restrict__ X1n, const double *__restrict__ X2n,
                              long n, int shape, double x0, double y0, double R,
                              double *__restrict__ phi, double *__restrict__ X1,
                              double *__restrict__ X2, unsigned long long *__restrict__ nbits) {
    long c = blockIdx.x * (long)blockDim.x + threadIdx.x;
    bool known = false;
    if (c < n) {
        if (shape == RMT_SHAPE_DISC) {
            double a = X1n[c], b = X2n[c];
            if (X1) { X1[c] = a; X2[c] = b; }
            const double ph = disc_phi(a, b, x0, y0, R);
            phi[c] = ph;
            known = ph < 0;
        } else {
            phi[c] = 1.0;
        }
    }
    if (nbits) {
        const unsigned long long w = __ballot(known);
        if ((threadIdx.x & 63) == 0 && c < n) nbits[c >> 6] = w;
    }
}

// k_phi_rebuild (disc, nx % 64 == 0) that also writes k_fluid_rows' pure-fluid flags: a wave
// holds 64 cells of one row, i.e. one stage tile's columns; lanes 0-3 add the 2-column halo
// on each side (phi recomputed from the same map, the same disc_phi) -- the flags equal
// k_fluid_rows' on this phi, and the momentum's pass over the phi plane is saved
__global__ void __launch_bounds__(256) k_phi_rebuild_fluid(
    const double *__restrict__ X1n, const double *__restrict__ X2n, long n, int nx, int tiles_x,
    double x0, double y0, double R, double *__restrict__ phi, double *__restrict__ X1,
    double *__restrict__ X2, unsigned long long *__restrict__ nbits, double thr,
    unsigned char *__restrict__ frows) {
    const long c = blockIdx.x * (long)blockDim.x + threadIdx.x;
    const int lane = threadIdx.x & 63;
    if (c - lane >= n) return;   // wave-uniform (n is a multiple of 64)
    const double a = X1n[c], b = X2n[c];
    if (X1) { X1[c] = a; X2[c] = b; }
    const double ph = disc_phi(a, b, x0, y0, R);
    phi[c] = ph;
    if (nbits) {
        const unsigned long long w = __ballot(ph < 0);
        if (lane == 0) nbits[c >> 6] = w;
    }
    const long j = c / nx;
    const int i = (int)(c - j * nx), tx = i >> 6;
    bool ok = ph > thr;   // (k_fluid_rows: NaN phi is not fluid)
    if (lane < 4) {
        const int e = lane < 2 ? 64 * tx - 2 + lane : 64 * tx + 62 + lane;
        if (e >= 0 && e < nx) {
            const long ce = j * nx + e;
            ok = ok && disc_phi(X1n[ce], X2n[ce], x0, y0, R) > thr;
        }
    }
    const unsigned long long all = __ballot(ok);
    if (lane == 0) frows[j * tiles_x + tx] = all == ~0ull;
}

// k_phi_rebuild on the listed tiles (after the chain: the targets all lie inside them)
__global__ void __launch_bounds__(256) k_phi_tiles(const double *__restrict__ X1n,
                                                   const double *__restrict__ X2n, int ny, int nx,
                                                   double x0, double y0, double R,
                                                   double *__restrict__ phi,
                                                   double *__restrict__ X1,
                                                   double *__restrict__ X2,
                                                   const int *__restrict__ tiles,
                                                   const int *__restrict__ count, int tiles_x,
                                                   unsigned long long *__restrict__ nbits) {
    const int cnt = *count;
    for (int b = blockIdx.x; b < cnt; b += gridDim.x)   // list_grid launch
    for (int q = threadIdx.x; q < MOM_TX * MOM_TY; q += 256) {
        const int t = tiles[b];
        const int i0 = (t % tiles_x) * MOM_TX, j0 = (t / tiles_x) * MOM_TY;
        const int j = j0 + q / MOM_TX, i = i0 + q % MOM_TX;
        bool known = false;
        if (j < ny && i < nx) {
            const long c = (long)j * nx + i;
            const double a = X1n[c], b = X2n[c];
            if (X1) { X1[c] = a; X2[c] = b; }
            const double ph = disc_phi(a, b, x0, y0, R);
            phi[c] = ph;
            known = ph < 0;
        }
        if (nbits) {   // a wave is one 64-cell word of row j (tile columns are word-aligned)
            const unsigned long long w = __ballot(known);
            if ((threadIdx.x & 63) == 0 && j < ny) nbits[(long)j * (nx >> 6) + (i0 >> 6)] = w;
        }
    }
}

// dt on device-ready scalars: returned to the host (one sync per step).
__global__ void k_dt(const double *m2, double dt_const, double cfl, double dx, double *out) {
    *out = fmin(dt_const, cfl * dx / (sqrt(*m2) + 1e-6));
}
// the same dt with max |u|^2 folded from the projection's per-block partials (NaN-propagating
// max, exact in any order): DTP_BLOCKS blocks fold their share and merge with a 64-bit atomic
// max on the bit patterns (values are +0.0 .. +inf or NaN, which orders them as doubles with
// every NaN on top); the last block writes sc[0] = max |u|^2, sc[1] = dt and re-arms acc.
// With e, block 0 first completes the previous step's ring record (k_ring_put's work, one
// launch fewer between the projection and the next chain): it reads sc before its atomic
// ticket, so before the last block overwrites sc.
constexpr int DTP_BLOCKS = 64;
__device__ __forceinline__ void ring_record(const double *sc, int *flag, double *e);
__global__ void __launch_bounds__(256) k_dt_part(const double *__restrict__ part, int np,
                                                 double dt_const, double cfl, double dx,
                                                 double *__restrict__ sc,
                                                 unsigned long long *__restrict__ acc,
                                                 int *__restrict__ flag = nullptr,
                                                 double *__restrict__ e = nullptr) {
    __shared__ double s[256];
    __shared__ bool last;
    if (e && blockIdx.x == 0 && threadIdx.x == 0) ring_record(sc, flag, e);
    double m = 0.0;
    for (int k = blockIdx.x * 256 + threadIdx.x; k < np; k += DTP_BLOCKS * 256) {
        const double y = part[k];
        if (y > m || y != y) m = y;
    }
    s[threadIdx.x] = m;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) {
            const double y = s[threadIdx.x + w];
            if (y > s[threadIdx.x] || y != y) s[threadIdx.x] = y;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        atomicMax(acc, (unsigned long long)__double_as_longlong(s[0]));
        __threadfence();
        last = atomicAdd((unsigned long long *)(acc + 1), 1ull) == DTP_BLOCKS - 1;
    }
    __syncthreads();
    if (last && threadIdx.x == 0) {
        __threadfence();
        const double m2 = __longlong_as_double((long long)atomicExch(acc, 0ull));
        atomicExch((unsigned long long *)(acc + 1), 0ull);
        sc[0] = m2;
        sc[1] = fmin(dt_const, cfl * dx / (sqrt(m2) + 1e-6));
    }
}
// rows [16 ty - 1, 16 ty + 17) of every listed fix-up tile: the rows whose Rhie-Chow rhs
// (u*, v* at j-1 .. j+1) the tile re-run can change
// (tmark, nullable: the listed tiles themselves, one byte per tile)
__global__ void k_mark_rows(const int *__restrict__ tiles, const int *__restrict__ count,
                            int tiles_x, int ny, unsigned char *__restrict__ rowmark,
                            unsigned char *__restrict__ tmark = nullptr) {
    const int cnt = *count;
    for (int b = blockIdx.x; b < cnt; b += gridDim.x) {   // list_grid launch
        const int j = (tiles[b] / tiles_x) * MOM_TY - 1 + (int)threadIdx.x;
        if (threadIdx.x < MOM_TY + 2 && j >= 0 && j < ny) rowmark[j] = 1;
        if (tmark && threadIdx.x == 0) tmark[tiles[b]] = 1;
    }
}
// completes a ring record after k_diag_p2 wrote its diagnostics: max |u|^2, dt, flags
// and clears the non-finite flag for the next step (in place of a memset launch)
__device__ __forceinline__ void ring_record(const double *sc, int *flag, double *e) {
    e[DIAG_VALS] = sc[0];
    e[DIAG_VALS + 1] = sc[1];
    for (int k = 0; k < 4; ++k) e[DIAG_VALS + 2 + k] = flag ? (double)flag[k] : 0.0;
    if (flag) flag[0] = 0;
}
__global__ void k_ring_put(const double *__restrict__ sc, int *__restrict__ flag,
                           double *__restrict__ e) {
    if (threadIdx.x == 0) ring_record(sc, flag, e);
}

struct DiagArgs {
    const double *phi, *J, *xs, *ys, *u, *v, *X1, *X2;
    int ny, nx, energies;
    double dx, dy, w_t, rho_s, rho_f, mu_f, eta_s, mu_s, kappa;
    int jb, je;   // rows reduced (global indices; the whole grid: 0, ny)
    // k_diag_seg (both set, energies off, nx % 64 == 0): this step's pure-fluid bits per
    // (row, 64-column segment) from the SL pass and its fix-up tile marks
    const unsigned char *fbits = nullptr, *tmark = nullptr;
};
// partial [sx, sy, cnt, Jmin, Jmax, ke, se, diss, ymin, ymax] per block
__global__ void __launch_bounds__(DIAG_T) k_diag_p1(DiagArgs A, double *__restrict__ part) {
    __shared__ double s[DIAG_VALS][DIAG_T];
    double v[DIAG_VALS] = {0, 0, 0, INFINITY, -INFINITY, 0, 0, 0, INFINITY, -INFINITY};
    // Each thread visits c0, c0 + S, c0 + 2S, ... (S = grid size) in that order; the loads
    // of DIAG_U consecutive visits are issued together and (j, i) advance by (S / nx, S % nx)
    // without a 64-bit division per cell.  Same cells, same accumulation order as one visit
    // per iteration.
    constexpr int DIAG_U = 4;
    const long n = (long)A.je * A.nx, S = (long)DIAG_BLOCKS * DIAG_T;
    const int dj = (int)(S / A.nx), di = (int)(S % A.nx);
    long c = (long)A.jb * A.nx + blockIdx.x * (long)DIAG_T + threadIdx.x;
    int j = (int)(c / A.nx), i = (int)(c % A.nx);
    while (c < n) {
        double phq[DIAG_U], Jq[DIAG_U];
#pragma unroll
        for (int k = 0; k < DIAG_U; ++k) {
            const long ck = c + k * S;
            phq[k] = ck < n ? A.phi[ck] : 0.0;
            Jq[k] = ck < n ? A.J[ck] : 0.0;
        }
#pragma unroll
        for (int k = 0; k < DIAG_U; ++k) {
        if (c >= n) break;
        const double ph = phq[k];
        const bool solid = ph <= 0.0;
        if (solid) {
            v[0] += A.xs[i]; v[1] += A.ys[j]; v[2] += 1.0;
            v[8] = fmin(v[8], A.ys[j]); v[9] = fmax(v[9], A.ys[j]);
        }
        const double Jc = Jq[k];
        v[3] = fmin(v[3], Jc); v[4] = fmax(v[4], Jc);
        if (A.energies) {
            double H = heaviside(ph, A.w_t);
            double rho = (1 - H) * A.rho_s + H * A.rho_f;
            double uc = A.u[c], vc = A.v[c];
            v[5] += 0.5 * rho * (uc * uc + vc * vc);
            if (solid) v[6] += se_density(A.X1, A.X2, c, j, i, A.ny, A.nx, A.dx, A.dy, A.mu_s, A.kappa);
            const double h2x = 2 * A.dx, h2y = 2 * A.dy;
            double dudx = grad2(A.u + c, 1, i, A.nx, h2x), dvdy = grad2(A.v + c, A.nx, j, A.ny, h2y);
            double dxy = 0.5 * (grad2(A.u + c, A.nx, j, A.ny, h2y) + grad2(A.v + c, 1, i, A.nx, h2x));
            double mu = H * A.mu_f + (1 - H) * A.eta_s;
            v[7] += 2.0 * mu * (dudx * dudx + dvdy * dvdy + 2.0 * (dxy * dxy));
        }
        c += S; j += dj; i += di;
        if (i >= A.nx) { i -= A.nx; ++j; }
        }
    }
    for (int k = 0; k < DIAG_VALS; ++k) s[k][threadIdx.x] = v[k];
    __syncthreads();
    for (int w = DIAG_T / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w)
            for (int k = 0; k < DIAG_VALS; ++k) {
                double x = s[k][threadIdx.x], y = s[k][threadIdx.x + w];
                s[k][threadIdx.x] = (k == 3 || k == 8) ? fmin(x, y) : (k == 4 || k == 9) ? fmax(x, y) : x + y;
            }
        __syncthreads();
    }
    if (threadIdx.x < DIAG_VALS) part[blockIdx.x * DIAG_VALS + threadIdx.x] = s[threadIdx.x][0];
}
// k_diag_p1 (energies off) over the (row, 64-column segment) pieces that can hold a solid cell
// or J != 1.  A segment whose cells are all fluid (phi > max(w_t, w_cut, 0), bit 0 of the SL
// pass's fbits; NaN is not fluid) and that lies in no fix-up tile (where the fix-up prep
// rewrote phi and J after that pass) holds no phi <= 0 cell and J == 1 in every cell (the
// prep's value outside the stress region), so it adds nothing to the centroid sums and 1 to
// the J extrema; its phi and J are not read.  Every other cell is visited once, as in
// k_diag_p1: segments dealt to (block, wave, lane) round robin over the grid (64 flags per
// wave by ballot, then up to 8 needed segments' loads in flight), a lane one column of each;
// then k_diag_p1's block tree, so
// k_diag_p2 reduces the same DIAG_BLOCKS partials.  The centroid sums add the same terms in
// another order than k_diag_p1 (rounding-level differences of cx, cy; J extrema exact).
__global__ void __launch_bounds__(DIAG_T) k_diag_seg(DiagArgs A, double *__restrict__ part) {
    __shared__ double s[DIAG_VALS][DIAG_T];
    double v[DIAG_VALS] = {0, 0, 0, INFINITY, -INFINITY, 0, 0, 0, INFINITY, -INFINITY};
    const int W = A.nx >> 6, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int tiles_x = W;   // 64-column stage tiles: one segment wide
    const long nseg = (long)(A.je - A.jb) * W, s0 = (long)A.jb * W;
    // segment q of this block (q = 4 (64 c + lane) + wave, chunk c) is s0 + block + DIAG_BLOCKS q:
    // every block and wave takes an even share of the grid (and of the disc's segments)
    constexpr long STR = (long)DIAG_BLOCKS * DIAG_T;   // one chunk of every wave of every block
    bool skipped = false;
    for (long base = s0 + blockIdx.x + (long)DIAG_BLOCKS * wv; base < s0 + nseg; base += STR) {
        const long sg = base + (long)DIAG_BLOCKS * 4 * lane;
        bool need = false;
        if (sg < s0 + nseg) {
            const int j = (int)(sg / W), sx = (int)(sg - (long)j * W);
            need = !A.fbits || !(A.fbits[sg] & 1) || A.tmark[(j / MOM_TY) * tiles_x + sx];
            skipped = skipped || !need;
        }
        unsigned long long m = __ballot(need);
        while (m) {
            // up to 8 segments' loads in flight
            long sq[8];
            int nq = 0;
            for (; nq < 8 && m; ++nq, m &= m - 1)
                sq[nq] = base + (long)DIAG_BLOCKS * 4 * __builtin_ctzll(m);
            double phq[8], Jq[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const long c = k < nq ? sq[k] * 64 + lane : 0;
                phq[k] = k < nq ? A.phi[c] : 0.0;
                Jq[k] = k < nq ? A.J[c] : 0.0;
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                if (k >= nq) break;
                const int j = (int)(sq[k] / W), i = (int)(sq[k] - (long)j * W) * 64 + lane;
                if (phq[k] <= 0.0) {
                    v[0] += A.xs[i]; v[1] += A.ys[j]; v[2] += 1.0;
                    v[8] = fmin(v[8], A.ys[j]); v[9] = fmax(v[9], A.ys[j]);
                }
                v[3] = fmin(v[3], Jq[k]); v[4] = fmax(v[4], Jq[k]);
            }
        }
    }
    if (__ballot(skipped)) { v[3] = fmin(v[3], 1.0); v[4] = fmax(v[4], 1.0); }
    for (int k = 0; k < DIAG_VALS; ++k) s[k][threadIdx.x] = v[k];
    __syncthreads();
    for (int w = DIAG_T / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w)
            for (int k = 0; k < DIAG_VALS; ++k) {
                double x = s[k][threadIdx.x], y = s[k][threadIdx.x + w];
                s[k][threadIdx.x] = (k == 3 || k == 8) ? fmin(x, y) : (k == 4 || k == 9) ? fmax(x, y) : x + y;
            }
        __syncthreads();
    }
    if (threadIdx.x < DIAG_VALS) part[blockIdx.x * DIAG_VALS + threadIdx.x] = s[threadIdx.x][0];
}
// the step's diagnostics partials.  Energies off and nx % 64 == 0: k_diag_seg, whether or
// not a step's fluid bits let it skip segments (fbits null: every segment) -- a skipped
// segment adds nothing to any lane's sums, so every schedule gives the same bits; else (and
// with the diag_seg switch off) k_diag_p1
static void diag_partials(const DiagArgs &D, double *part, hipStream_t st, bool seg_on) {
    if (seg_on && !D.energies && D.nx % 64 == 0 && MOM_TX == 64)
        k_diag_seg<<<DIAG_BLOCKS, DIAG_T, 0, st>>>(D, part);
    else
        k_diag_p1<<<DIAG_BLOCKS, DIAG_T, 0, st>>>(D, part);
}
__global__ void __launch_bounds__(DIAG_T) k_diag_p2(const double *__restrict__ part,
                                                    double *__restrict__ out) {
    __shared__ double s[DIAG_VALS][DIAG_T];
    double v[DIAG_VALS] = {0, 0, 0, INFINITY, -INFINITY, 0, 0, 0, INFINITY, -INFINITY};
    for (int b = threadIdx.x; b < DIAG_BLOCKS; b += DIAG_T)
        for (int k = 0; k < DIAG_VALS; ++k) {
            double y = part[b * DIAG_VALS + k];
            v[k] = (k == 3 || k == 8) ? fmin(v[k], y) : (k == 4 || k == 9) ? fmax(v[k], y) : v[k] + y;
        }
    for (int k = 0; k < DIAG_VALS; ++k) s[k][threadIdx.x] = v[k];
    __syncthreads();
    for (int w = DIAG_T / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w)
            for (int k = 0; k < DIAG_VALS; ++k) {
                double x = s[k][threadIdx.x], y = s[k][threadIdx.x + w];
                s[k][threadIdx.x] = (k == 3 || k == 8) ? fmin(x, y) : (k == 4 || k == 9) ? fmax(x, y) : x + y;
            }
        __syncthreads();
    }
    if (threadIdx.x < DIAG_VALS) out[threadIdx.x] = s[threadIdx.x][0];
}

// k_sim_sl for other drivers (mac.hip: one disc's map on the MAC cell-centre velocity)
int sl_disc_map(rmt_ctx *ctx, const double *X1, const double *X2, const double *a,
                const double *b, const double *xs, const double *ys, double dt, double dx,
                double dy, double x0, double y0, double R, double *X1n, double *X2n,
                double *phi_pre, int *bad, const double *dev_m2, unsigned long long *kbits,
                const int *cbox, bool faces) {
    // cbox {j0, j1, i0, i1}: only the tiles meeting those cells (kbits words outside them
    // are left alone: the caller clears them)
    int ty0 = 0, ty1 = (ctx->ny + SLT_Y - 1) / SLT_Y, tx0 = 0, tx1 = (ctx->nx + SLT_X - 1) / SLT_X;
    if (cbox) {
        ty0 = cbox[0] / SLT_Y; ty1 = (cbox[1] + SLT_Y - 1) / SLT_Y;
        tx0 = cbox[2] / SLT_X; tx1 = (cbox[3] + SLT_X - 1) / SLT_X;
        if (ty1 <= ty0 || tx1 <= tx0) return RMT_OK;
    }
    // faces: a, b are MAC face planes (k_sim_sl_t<1>)
    RMT_CHECK(!faces || ctx->nx == ctx->ny, RMT_EINVAL, "sl_disc_map: faces need a square grid");
    auto *kern = faces ? k_sim_sl_t<1> : k_sim_sl_t<0>;
    kern<<<dim3(tx1 - tx0, ty1 - ty0), SLT_X * SLT_Y, 0, ctx->stream>>>(
        X1, X2, a, b, xs, ys, ctx->ny, ctx->nx, dt, divk_make(dx), divk_make(dy), x0, y0, R, X1n,
        X2n, phi_pre, bad, kbits, dev_m2, nullptr, 0, nullptr, nullptr, 0.0, nullptr, nullptr,
        tx0, ty0, nullptr, nullptr, 0);
    RMT_LAUNCHED();
    return RMT_OK;
}

// slab-decomposed step: the 10 diagnostic partials of rows [jb, je) into out (device)
int diag_rows(rmt_ctx *ctx, const double *phi, const double *J, const double *xs,
              const double *ys, const double *u, const double *v, const double *X1,
              const double *X2, const rmt_sim_params &P, int jb, int je, double *part,
              double *out) {
    DiagArgs D{phi, J, xs, ys, u, v, X1, X2, P.ny, P.nx, P.energies, P.dx, P.dy, P.w_t,
               P.rho_s, P.rho_f, P.mu_f, P.eta_s, P.mu_s, P.kappa, jb, je};
    k_diag_p1<<<DIAG_BLOCKS, DIAG_T, 0, ctx->stream>>>(D, part);
    k_diag_p2<<<1, DIAG_T, 0, ctx->stream>>>(part, out);
    RMT_LAUNCHED();
    return RMT_OK;
}

}  // namespace rmt

using namespace rmt;

extern "C" {

int rmt_sim_create(rmt_ctx *ctx, const rmt_sim_params *prm, rmt_sim **out) {
    RMT_CHECK(ctx && prm && out, RMT_EINVAL, "null argument");
    RMT_CHECK(prm->ny == ctx->ny && prm->nx == ctx->nx, RMT_EINVAL, "sim grid != ctx grid");
    RMT_CHECK(prm->scheme >= RMT_SCHEME_SEMILAGRANGIAN &&
                  prm->scheme <= RMT_SCHEME_SEMILAGRANGIAN_CUBIC,
              RMT_EINVAL, "unknown advection scheme");
    RMT_CHECK(prm->bc_kind >= 0 && prm->bc_kind <= 3, RMT_EINVAL, "unknown bc kind");
    RMT_CHECK(prm->shape == RMT_SHAPE_NONE || prm->shape == RMT_SHAPE_DISC, RMT_EINVAL,
              "unknown shape");
    RMT_CHECK(prm->shape == RMT_SHAPE_NONE || prm->rho_s == prm->rho_f, RMT_ENOTSUP,
              "rho_s != rho_f needs the variable-density CG projection (not on this path)");
    rmt_sim *S = new rmt_sim;
    S->ctx = ctx;
    S->P = *prm;
    S->P.xs = S->P.ys = nullptr;
    const int ny = prm->ny, nx = prm->nx;
    const size_t n = (size_t)ny * nx;
    const int nplanes = 16 + MOM_WORK_PLANES;
    size_t bytes = (nplanes * n + nx + ny + DIAG_BLOCKS * DIAG_VALS + 64) * sizeof(double) + n + 256;
    RMT_HIP(hipMalloc(&S->block, bytes));
    RMT_HIP(hipMemsetAsync(S->block, 0, bytes, ctx->stream));
    double *q = (double *)S->block;
    double **planes[] = {&S->u, &S->v, &S->p, &S->X1, &S->X2, &S->phi, &S->phi_pre, &S->J,
                         &S->X1n, &S->X2n, &S->us, &S->vs, &S->sxx, &S->sxy, &S->syy};
    for (auto pp : planes) { *pp = q; q += n; }
    S->X1h = S->X1; S->X2h = S->X2;
    S->kbits = (unsigned long long *)q; q += n;   // ny * ceil(nx / 64) words fit a plane
    S->mw = q; q += MOM_WORK_PLANES * n;
    S->xs = q; q += nx;
    S->ys = q; q += ny;
    S->dscr = q; q += DIAG_BLOCKS * DIAG_VALS + 64;
    S->mbytes = (unsigned char *)q;
    S->flag = (int *)(S->mbytes + n + 64);
    RMT_HIP(hipMemcpyAsync(S->xs, prm->xs, nx * 8, hipMemcpyHostToDevice, ctx->stream));
    RMT_HIP(hipMemcpyAsync(S->ys, prm->ys, ny * 8, hipMemcpyHostToDevice, ctx->stream));
    // constant part of functions.py:165-192 (everything but the advective limit); the
    // reference's h**2 on a numpy float64 scalar is libm pow.
    const double dx = prm->dx, CFL = prm->cfl;
    double cs = std::sqrt((prm->kappa + prm->mu_s * 4.0 / 3.0) / (prm->rho_s + 1e-12));
    double d = std::fmin(CFL * dx / (cs + 1e-14), 1.0);
    double mu_max = std::fmax(prm->mu_f, prm->eta_s), rho_min = std::fmin(prm->rho_s, prm->rho_f);
    if (mu_max > 1e-12 && rho_min > 1e-12)
        d = std::fmin(d, CFL * rho_min * std::pow(dx, 2.0) / (4.0 * mu_max));
    S->dt_const = std::fmin(d, prm->dt_cap);
    // size the shared scratch once (WENO5: 3 planes, projection: 2) and the extrapolation's
    // byte workspace, so nothing is reallocated while kernels are queued
    RMT_TRY(ensure_scratch(ctx, 3 * n * sizeof(double)));
    RMT_TRY(ensure_bytes(ctx, extrap_workspace(ny, nx, prm->layers, extrap_par_enabled())));
    if (prm->shape == RMT_SHAPE_DISC && prm->scheme == RMT_SCHEME_SEMILAGRANGIAN &&
        prm->layers >= 1 && prm->layers <= 12) {
        // the speculative momentum stream at the lowest priority: the extrapolation's own
        // kernels (chip-wide passes, then the chain) are dispatched first when both are ready
        int least = 0, greatest = 0;
        RMT_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest));
        RMT_HIP(hipStreamCreateWithPriority(&S->st2, hipStreamNonBlocking, least));
        if (ctx->opt.sim_hiprio && greatest != least) {
            RMT_HIP(hipStreamCreateWithPriority(&S->st1, hipStreamNonBlocking, greatest));
            RMT_HIP(hipEventCreateWithFlags(&S->e_in, hipEventDisableTiming));
            RMT_HIP(hipEventCreateWithFlags(&S->e_out, hipEventDisableTiming));
        }
        RMT_HIP(hipEventCreateWithFlags(&S->e_sl, hipEventDisableTiming));
        RMT_HIP(hipEventCreateWithFlags(&S->e_mom, hipEventDisableTiming));
        RMT_HIP(hipEventCreateWithFlags(&S->e_rows, hipEventDisableTiming));
        S->max_tiles = ((nx + MOM_TX - 1) / MOM_TX) * ((ny + MOM_TY - 1) / MOM_TY);
        RMT_HIP(hipMalloc(&S->tiles, (S->max_tiles + 64) * sizeof(int)));
        S->tcount = S->tiles + S->max_tiles;
    }
    S->m2n = ((nx + 255) / 256) * ny;
    const size_t Wn = (size_t)(nx + 63) / 64;
    RMT_HIP(hipMalloc(&S->m2part, ((size_t)S->m2n + (size_t)RING_N * RING_VALS + ny / 8 + 8 +
                                   (size_t)ny * Wn + ny / 2 + 8 + (size_t)ny * Wn +
                                   (size_t)ny * ((nx + 255) / 256) / 2 + 8 + 8 +
                                   (size_t)S->max_tiles / 8 + 8) * sizeof(double)));
    S->ring = S->m2part + S->m2n;
    S->rowmark = (unsigned char *)(S->ring + (size_t)RING_N * RING_VALS);
    S->rimw = (unsigned long long *)(S->ring + (size_t)RING_N * RING_VALS + ny / 8 + 8);
    S->rimcnt = (int *)(S->rimw + (size_t)ny * Wn);
    S->kbits_next = (unsigned long long *)((double *)S->rimcnt + ny / 2 + 8);
    S->segs = (int *)(S->kbits_next + (size_t)ny * Wn);
    S->m2acc = (unsigned long long *)(S->segs + (((size_t)ny * ((nx + 255) / 256) + 3) & ~(size_t)1));
    S->tmark = (unsigned char *)(S->m2acc + 8);   // max_tiles bytes
    RMT_HIP(hipMemsetAsync(S->m2acc, 0, 2 * sizeof(unsigned long long), ctx->stream));
    if (nx % 64 == 0) RMT_HIP(hipMalloc(&S->pconst, (size_t)ny * (nx / 64)));
    if (S->st2 && nx % 64 == 0) {
        const size_t ntl = (size_t)(nx / SLT_X) * ((ny + SLT_Y - 1) / SLT_Y);
        RMT_HIP(hipMalloc(&S->zf[0], 2 * ntl));
        S->zf[1] = S->zf[0] + ntl;
    }
    if (S->st2) {
        RMT_HIP(hipEventCreateWithFlags(&S->e_bits, hipEventDisableTiming));
        RMT_HIP(hipEventCreateWithFlags(&S->e_proj, hipEventDisableTiming));
        RMT_HIP(hipEventCreateWithFlags(&S->e_tail, hipEventDisableTiming));
        RMT_HIP(hipEventCreateWithFlags(&S->e_tailp, hipEventDisableTiming));
        RMT_HIP(hipEventCreateWithFlags(&S->e_kb, hipEventDisableTiming));
        RMT_HIP(hipEventCreateWithFlags(&S->e_geo, hipEventDisableTiming));
    }
    if (S->st2 && prm->rho_f > 0) {
        RMT_TRY(dct_plan(ctx, prm->dx, prm->dy));
        S->split_proj = dct_lds_ready(ctx) && ny <= ctx->rsum_len;
    }
    RMT_HIP(hipStreamSynchronize(ctx->stream));
    *out = S;
    return RMT_OK;
}

int rmt_sim_destroy(rmt_sim *S) {
    if (!S) return RMT_OK;
    (void)hipFree(S->block);
    if (S->m2part) (void)hipFree(S->m2part);
    if (S->pconst) (void)hipFree(S->pconst);
    if (S->zf[0]) (void)hipFree(S->zf[0]);
    if (S->tiles) (void)hipFree(S->tiles);
    if (S->e_sl) (void)hipEventDestroy(S->e_sl);
    if (S->e_mom) (void)hipEventDestroy(S->e_mom);
    if (S->e_rows) (void)hipEventDestroy(S->e_rows);
    if (S->e_bits) (void)hipEventDestroy(S->e_bits);
    if (S->e_proj) (void)hipEventDestroy(S->e_proj);
    if (S->e_tail) (void)hipEventDestroy(S->e_tail);
    if (S->e_tailp) (void)hipEventDestroy(S->e_tailp);
    if (S->e_kb) (void)hipEventDestroy(S->e_kb);
    if (S->e_geo) (void)hipEventDestroy(S->e_geo);
    if (S->st2) (void)hipStreamDestroy(S->st2);
    if (S->st1) (void)hipStreamDestroy(S->st1);
    if (S->e_in) (void)hipEventDestroy(S->e_in);
    if (S->e_out) (void)hipEventDestroy(S->e_out);
    for (auto e : S->pev) if (e) (void)hipEventDestroy(e);
    S->ctx->prof = false;
    delete S;
    return RMT_OK;
}

int rmt_sim_field(rmt_sim *S, int field, double **ptr) {
    RMT_CHECK(S && ptr, RMT_EINVAL, "null argument");
    double *f[] = {S->u, S->v, S->p, S->X1, S->X2, S->phi, S->J, S->sxx, S->sxy, S->syy};
    RMT_CHECK(field >= 0 && field < 10, RMT_EINVAL, "unknown field id");
    *ptr = f[field];
    return RMT_OK;
}

// One step's host bookkeeping from its diagnostics record: error flags, t, the diag entry.
static int sim_record(rmt_sim *S, const double *dv, double m2, double dt, const int *fl) {
    const rmt_sim_params &P = S->P;
    RMT_CHECK(!fl[0], RMT_ENONFINITE, "advect_reference_map: non-finite velocity (the "
                                      "simulation diverged)");
    RMT_CHECK(!fl[3], RMT_EDEVICE, extrap_abort_detail(fl[3]));
    S->t += dt;
    rmt_diag r{};
    r.t = S->t; r.dt = dt;
    r.cx = dv[2] > 0 ? dv[0] / dv[2] : NAN;
    r.cy = dv[2] > 0 ? dv[1] / dv[2] : NAN;
    r.minJ = dv[3]; r.maxJ = dv[4]; r.umax = std::sqrt(m2);
    if (P.energies) {
        r.ke = dv[5] * P.dx * P.dy;
        r.se = dv[6] * P.dx * P.dy;
        r.diss = dv[7] * P.dx * P.dy;
        S->integ += r.diss * dt;
        r.integ = S->integ;
        r.ry = dv[2] > 0 ? 0.5 * (dv[9] - dv[8]) : NAN;
    }
    S->diag.push_back(r);
    return RMT_OK;
}

int rmt_sim_step(rmt_sim *S, int nsteps, double t_end) {
    RMT_CHECK(S, RMT_EINVAL, "null sim");
    rmt_ctx *ctx = S->ctx;
    const rmt_sim_params &P = S->P;
    const int ny = P.ny, nx = P.nx;
    const long n = (long)ny * nx;
    const unsigned g = grid1d(n, 256);
    // run on S->st1 (highest priority) when it exists: ordered after the caller's stream on
    // entry, the caller's stream ordered after it on every return
    struct OnHi {
        rmt_ctx *c; hipStream_t user; rmt_sim *S;
        ~OnHi() {
            if (!S->st1) return;
            (void)hipEventRecord(S->e_out, S->st1);
            (void)hipStreamWaitEvent(user, S->e_out, 0);
            c->stream = user;
        }
    } on_hi{ctx, ctx->stream, S};
    // the map buffers swap roles every step; at the call's end the state is copied back into
    // the buffers rmt_sim_field hands out (one copy per call instead of one per step).  Runs
    // on the step's stream before on_hi hands the stream back (destroyed first).
    struct MapHome {
        rmt_sim *S;
        ~MapHome() {
            if (S->X1 == S->X1h) return;
            const size_t b = (size_t)S->P.ny * S->P.nx * sizeof(double);
            (void)hipMemcpyAsync(S->X1h, S->X1, b, hipMemcpyDeviceToDevice, S->ctx->stream);
            (void)hipMemcpyAsync(S->X2h, S->X2, b, hipMemcpyDeviceToDevice, S->ctx->stream);
            std::swap(S->X1, S->X1n);
            std::swap(S->X2, S->X2n);
            S->zcur ^= 1;
        }
    } map_home{S};
    if (S->st1) {
        RMT_HIP(hipEventRecord(S->e_in, ctx->stream));
        RMT_HIP(hipStreamWaitEvent(S->st1, S->e_in, 0));
        ctx->stream = S->st1;
    }
    hipStream_t st = ctx->stream;
    double *sc = S->dscr + DIAG_BLOCKS * DIAG_VALS;   // [0] maxsq, [1] dt, [2..11] diag
    // Asynchronous path (no t_end: nothing to clip): dt is computed and consumed on the
    // device, max |u|^2 comes out of the projection, and the per-step diagnostics go to a
    // device ring read back every RING_N steps -- no host round trip inside the loop.  The
    // synchronous path (t_end clip, profiling, the Eulerian schemes) reads dt back each step.
    const bool force_sync = ctx->opt.sim_sync != 0;
    const bool async = !force_sync && !S->prof && std::isinf(t_end) && t_end > 0 &&
                       P.scheme == RMT_SCHEME_SEMILAGRANGIAN;
    int slot = 0;
    // the step's tail (p -= mean(p), the diagnostics) may run on the second stream beside the
    // next step's band passes; joined before the ring is read and when the call returns
    // Deferred to the second stream's next start (the next chain's launch), so that it does
    // not crowd the next step's rim advection and record values either.
    bool tail = false, pending = false;
    bool tail_p = false;   // the pending tail's pressure update ran on the edge-tile stream
    double *pend_e = nullptr;
    // the pending tail's diagnostics already ran (on the second stream after the next step's
    // geometry, beside the projection: they read phi and J only, final after the fix-up)
    bool pend_diag_done = false, diag_early = false, pend_seg = false;
    // after_sl: the second stream already waits for this step's e_sl, recorded on the main
    // stream after the tail's projection -- no event of its own (a record right after the
    // velocity correction cost the critical path ~5 us); else one recorded now
    auto emit_tail = [&](bool after_sl) -> int {
        if (!pending) return RMT_OK;
        pending = false;
        DiagArgs D{S->phi, S->J, S->xs, S->ys, S->u, S->v, S->X1, S->X2, ny, nx, P.energies,
                   P.dx, P.dy, P.w_t, P.rho_s, P.rho_f, P.mu_f, P.eta_s, P.mu_s, P.kappa, 0, ny};
        if (!after_sl) {
            RMT_HIP(hipEventRecord(S->e_proj, st));
            RMT_HIP(hipStreamWaitEvent(S->st2, S->e_proj, 0));
        }
        ctx->stream = S->st2;
        // beside the chain (after_sl), the pressure update runs on the edge-tile stream,
        // beside the second stream's SL and prep; that stream's momentum stages wait for it
        // (tail_p, MomWork::wait_p) before they read p, and nothing else of the step touches
        // p, pc or the root before then (RMT_TAIL_STREAM)
        hipStream_t ts_st = S->st2;
        if (after_sl && ctx->opt.tail_stream) {
            hipStream_t es = nullptr;
            const int e = edge_stream(ctx, &es);
            if (e != RMT_OK) { ctx->stream = st; return e; }
            if (es) {
                RMT_HIP(hipStreamWaitEvent(es, S->e_sl, 0));
                ts_st = es;
            }
        }
        ctx->stream = ts_st;
        // (the pending tail always follows a projection_finish that deferred the pressure
        // update: pc and its mean's root are still where that projection left them)
        const int ts = sub_mean_rows_upd(ctx, S->p, ctx->scratch + (long)ny * nx,
                                         ctx->red + RED_BLOCKS + 17, ny, nx);
        ctx->stream = st;
        RMT_TRY(ts);
        tail_p = ts_st != S->st2;
        if (tail_p) RMT_HIP(hipEventRecord(S->e_tailp, ts_st));
        if (!pend_diag_done) {
            // (this step's SL pass and fix-up marks come after this on the same stream)
            if (pend_seg) {
                D.fbits = fluid_bits_buf(mom_work(S->mw, (long)ny * nx, S->mbytes, S->flag + 1));
                D.tmark = S->tmark;
            }
            diag_partials(D, S->dscr, S->st2, ctx->opt.diag_seg != 0);
            k_diag_p2<<<1, DIAG_T, 0, S->st2>>>(S->dscr, pend_e);
            RMT_LAUNCHED();
        }
        RMT_HIP(hipEventRecord(S->e_tail, S->st2));
        tail = true;
        return RMT_OK;
    };
    auto join = [&]() -> int {
        RMT_TRY(emit_tail(false));
        if (tail) RMT_HIP(hipStreamWaitEvent(st, S->e_tail, 0));
        if (tail && tail_p) RMT_HIP(hipStreamWaitEvent(st, S->e_tailp, 0));
        tail = false;
        tail_p = false;
        return RMT_OK;
    };
    // the last step's ring record, completed by the next step's k_dt_part (or here)
    double *ring_e = nullptr;
    int *const ring_flag = P.shape != RMT_SHAPE_NONE ? S->flag : nullptr;
    auto flush = [&]() -> int {
        RMT_TRY(join());
        if (ring_e) {
            k_ring_put<<<1, 64, 0, st>>>(sc, ring_flag, ring_e);
            RMT_LAUNCHED();
            ring_e = nullptr;
        }
        if (!slot) return RMT_OK;
        std::vector<double> h((size_t)slot * RING_VALS);
        RMT_HIP(hipMemcpyAsync(h.data(), S->ring, h.size() * sizeof(double),
                               hipMemcpyDeviceToHost, st));
        RMT_HIP(hipStreamSynchronize(st));
        const int cnt = slot;
        slot = 0;
        for (int k = 0; k < cnt; ++k) {
            const double *e = h.data() + (size_t)k * RING_VALS;
            int fl[4];
            for (int q = 0; q < 4; ++q) fl[q] = (int)e[DIAG_VALS + 2 + q];
            RMT_TRY(sim_record(S, e, e[DIAG_VALS], e[DIAG_VALS + 1], fl));
        }
        return RMT_OK;
    };
    // a carried state (rmt_sim_set_carry): this call's first step uses the geometry, known
    // plane, prep planes and max |u|^2 partials the previous call's last step left
    const bool carry = S->carry_on && S->carry_valid && S->carry_gen == ctx->bytes_gen &&
                       S->carry_cfg == extrap_config_gen();
    const bool m2_ok = carry && S->m2_valid;
    S->carry_valid = false;
    // the zero-tile flags describe maps this call wrote (the caller may change them between calls)
    S->zv[0] = S->zv[1] = false;
    if (!carry) {
        S->bits_ready = false;   // the caller may have changed the map between calls
        // ... or the prep planes: the first prep of a call writes every segment
        if (S->pconst) RMT_HIP(hipMemsetAsync(S->pconst, 0, (size_t)ny * (nx / 64), st));
    }
    // the next step's rim words and extrapolation geometry, prepared on the second stream
    // beside this step's projection (they depend on the known plane alone)
    const bool geo_env = ctx->opt.early_geometry != 0;
    // the column pass's transpose of the row blocks without fix-up rows beside the chain
    // (RMT_EARLY_TRANSPOSE, default on)
    const bool early_t_env = ctx->opt.early_transpose != 0;
    bool early_t = false;
    // k_phi_rebuild writes the momentum's pure-fluid flags (RMT_FUSED_FLUID, default on)
    const bool fluid_env = ctx->opt.fused_fluid != 0;
    bool geo_ready = carry;
    bool m2_last = false;   // the last step's projection wrote the max |u|^2 partials
    for (int it = 0; it < nsteps; ++it) {
        if (!(S->t < t_end)) break;
        if (S->prof) RMT_HIP(hipEventRecord(S->pev[0], st));
        // 1. dt (compute_timestep + the drivers' clip to t_end); NaN-propagating max so it
        // also bounds the velocities for the SL block skip
        double hv[2] = {0.0, 0.0}, dt = NAN;
        if (async && (it > 0 || m2_ok)) {
            k_dt_part<<<DTP_BLOCKS, 256, 0, st>>>(S->m2part, S->m2n, S->dt_const, P.cfl, P.dx,
                                                  sc, S->m2acc, ring_e ? ring_flag : nullptr,
                                                  ring_e);
            RMT_LAUNCHED();
            ring_e = nullptr;
        } else {
            RMT_CHECK(!ring_e, RMT_EINVAL, "sim: ring record pending on a synchronous step");
            RMT_TRY(reduce_maxsq2_nan(ctx, S->u, S->v, n, sc));
            k_dt<<<1, 1, 0, st>>>(sc, S->dt_const, P.cfl, P.dx, sc + 1);
            RMT_LAUNCHED();
        }
        if (!async) {
            RMT_HIP(hipMemcpyAsync(hv, sc, 2 * sizeof(double), hipMemcpyDeviceToHost, st));
            RMT_HIP(hipStreamSynchronize(st));
            dt = hv[1];
            if (S->t + dt > t_end) dt = t_end - S->t;
        }
        const double *dtp = async ? sc + 1 : nullptr;
        const bool solid = P.shape != RMT_SHAPE_NONE;
        // this step's phi kernels also write the next step's known plane (split advection)
        unsigned long long *nb = (solid && P.scheme == RMT_SCHEME_SEMILAGRANGIAN && S->e_bits &&
                                  nx % 64 == 0) ? S->kbits_next : nullptr;
        rmt_momentum_params M{};
        M.bc_kind = P.bc_kind; M.lid = P.lid; M.mu_s = P.mu_s; M.kappa = P.kappa;
        M.eta_s = P.eta_s; M.rho_s = P.rho_s; M.rho_f = P.rho_f; M.mu_f = P.mu_f; M.w_t = P.w_t;
        M.dx = P.dx; M.dy = P.dy; M.dt = dt; M.stress_band = P.stress_band;
        M.detg_clamp = P.detg_clamp;
        MomWork W = mom_work(S->mw, n, S->mbytes, S->flag + 1);
        W.dtp = dtp;
        W.prep_const = S->pconst;
        // the extrapolation chain occupies one CU for milliseconds; everything it does not
        // feed runs beside it: the momentum of every cell, from the pre-extrapolation map, on
        // a second stream, re-run afterwards on the tiles within reach of a target
        const bool no_overlap = ctx->opt.no_overlap != 0;
        const bool side_tail = ctx->opt.side_tail != 0;
        // the parallel extrapolation: its values pass (~0.5 ms at N=4096, mostly the
        // one-workgroup combine) runs beside the speculative momentum too (RMT_PAR_OVERLAP=0:
        // in order, the momentum after it)
        const bool par = extrap_par_enabled();
        const bool par_ov = ctx->opt.par_overlap != 0;
        const bool overlap = solid && S->st2 && !no_overlap && (!par || par_ov);
        bool fixprep = false;   // the fused fix-up prep (set where the extrapolation runs)
        bool seg_diag = false;  // this step's fbits and fix-up tile marks are set (k_diag_seg)
        if (S->prof) RMT_HIP(hipEventRecord(S->pev[1], st));
        if (solid) {
            // (the output buffer's zero-tile flags hold only when the flagged pass writes it;
            // the flagged pass reads them first: the rim pass and the chain below write only rim
            // cells, and a tile with a rim cell never uses them)
            const bool zo_valid = S->zv[S->zcur ^ 1];
            S->zv[S->zcur ^ 1] = false;
            // 2. advect the reference map with the pre-advection level set and mask
            // (on the asynchronous path the previous step's ring record -- k_dt_part or k_ring_put --
            // cleared it)
            if (!(async && it > 0)) RMT_HIP(hipMemsetAsync(S->flag, 0, sizeof(int), st));
            if (P.scheme == RMT_SCHEME_SEMILAGRANGIAN && overlap && S->e_bits) {
                // known plane -> rim words -> the rim's advection here; the rest on the second
                // stream, beside the extrapolation (which reads rim cells only)
                const dim3 gsl((nx + 255) / 256, ny);
                if (!S->bits_ready) {
                    k_sim_bits<<<gsl, 256, 0, st>>>(S->X1, S->X2, nx, P.x0, P.y0, P.R, S->kbits);
                    RMT_LAUNCHED();
                }
                const long nseg = (long)ny * ((nx + 255) / 256);
                int *scount = S->segs + nseg;
                if (geo_ready) {
                    RMT_HIP(hipStreamWaitEvent(st, S->e_geo, 0));
                } else {
                    RMT_TRY(rim_words(ctx, S->kbits, ny, nx, (nx + 63) / 64, S->rimw, S->rimcnt));
                    RMT_HIP(hipMemsetAsync(scount, 0, sizeof(int), st));
                    k_rim_segments<<<grid1d(nseg, 256), 256, 0, st>>>(S->rimw, ny, nx, S->segs,
                                                                       scount);
                }
                k_sim_sl_rim<<<4096, 256, 0, st>>>(   // ~one rim segment per block
                    S->X1, S->X2, S->u, S->v, S->xs, S->ys, ny, nx, dt, divk_make(P.dx), divk_make(P.dy), P.x0, P.y0,
                    P.R, S->X1n, S->X2n, S->flag, sc, dtp, S->rimw, S->segs, scount);
            } else if (P.scheme == RMT_SCHEME_SEMILAGRANGIAN) {
                k_sim_sl_t<0><<<dim3((nx + SLT_X - 1) / SLT_X, (ny + SLT_Y - 1) / SLT_Y), SLT_X * SLT_Y,
                             0, st>>>(S->X1, S->X2, S->u, S->v, S->xs, S->ys, ny, nx, dt,
                                      divk_make(P.dx), divk_make(P.dy), P.x0, P.y0, P.R, S->X1n,
                                      S->X2n, S->phi_pre, S->flag, S->kbits, sc, dtp, 0, nullptr);
            } else if (P.scheme == RMT_SCHEME_SEMILAGRANGIAN_CUBIC) {
                k_sim_sl_cubic<<<g, 256, 0, st>>>(S->X1, S->X2, S->u, S->v, S->xs, S->ys, ny, nx,
                                                  dt, P.dx, P.dy, P.x0, P.y0, P.R, S->X1n,
                                                  S->X2n, S->phi_pre, S->flag);
            } else {
                // Eulerian schemes on the pre-advection level set, w_cut = 0 as the drivers
                k_sim_phi_mask<<<g, 256, 0, st>>>(S->X1, S->X2, S->u, S->v, n, P.x0, P.y0, P.R,
                                                  S->phi_pre, S->flag);
                for (int comp = 0; comp < 2; ++comp) {
                    const double *q = comp ? S->X2 : S->X1;
                    double *o = comp ? S->X2n : S->X1n;
                    if (P.scheme == RMT_SCHEME_WENO5)
                        RMT_TRY(rmt_advect_weno5_rk3(ctx, q, S->u, S->v, P.dx, P.dy, dt,
                                                     S->phi_pre, 0.0, o));
                    else
                        RMT_TRY(rmt_advect_central_rk3(ctx, q, S->u, S->v, P.dx, P.dy, dt,
                                                       S->phi_pre, 0.0,
                                                       P.scheme == RMT_SCHEME_CONSERVATIVE, o));
                }
                k_mask_mul<<<g, 256, 0, st>>>(S->X1n, S->X2n, S->phi_pre, n);
            }
            RMT_LAUNCHED();
            if (S->prof) RMT_HIP(hipEventRecord(S->pev[2], st));
            // 3. narrow-band extrapolation (exact raster-order semantics), in place; with the
            // overlap, the speculative phi + momentum start on the second stream once the
            // chip-wide passes are done and the one-workgroup chain kernel is launched
            if (overlap) ctx->ev_chain = S->e_sl;
            const bool kb = P.scheme == RMT_SCHEME_SEMILAGRANGIAN;   // k_sim_sl wrote kbits
            if (geo_ready && !overlap) RMT_HIP(hipStreamWaitEvent(st, S->e_geo, 0));
            // with the fused fix-up prep (below) the status words are copied by its kernel
            const bool fp_env = ctx->opt.fused_fixprep != 0;
            fixprep = overlap && fp_env && P.shape == RMT_SHAPE_DISC && nx % 64 == 0 &&
                      momentum_mode() != 2 && P.layers > 0;
            int *dstat = fixprep ? nullptr : S->flag + 2;
            // with the fused fix-up prep the fallback sweep runs on the second stream beside the
            // chain (the fix-up joins that stream before it reads the map or the status)
            ctx->ex_sweep_defer = fixprep;
            ctx->ev_chain_vals = fixprep;   // ev_chain completes with the values pass
            const int es = geo_ready && P.layers > 0
                               ? extrap_finish(ctx, P.dx, P.dy, P.layers, S->X1n, S->X2n, dstat)
                               : extrapolate(ctx, S->X1n, S->X2n, S->phi_pre, P.dx, P.dy, P.layers,
                                             S->X1n, S->X2n, dstat, kb ? S->kbits : nullptr);
            geo_ready = false;
            ctx->ev_chain = nullptr;
            ctx->ex_sweep_defer = false;
            ctx->ev_chain_vals = false;
            RMT_TRY(es);
            if (overlap) {
                RMT_HIP(hipStreamWaitEvent(S->st2, S->e_sl, 0));
                const int dly_side = ctx->opt.test_delay_side;
                if (dly_side) { k_delay<<<1, 1, 0, S->st2>>>(dly_side); RMT_LAUNCHED(); }
                if (fixprep && ctx->ex_chain && !ctx->ex_par)
                    RMT_TRY(extrap_sweep(ctx, P.dx, P.dy, P.layers, S->X1n, S->X2n, S->st2));
                // the previous step's tail, beside the chain (e_sl, recorded by this step's
                // extrapolation when it has layers, follows that step's projection)
                RMT_TRY(emit_tail(P.layers > 0));
                // the fix-up tiles and the rows they reach depend on the known plane only
                ctx->stream = S->st2;
                const int fs = extrap_fix_tiles(ctx, P.layers, 12, S->tiles, S->tcount);
                ctx->stream = st;
                RMT_TRY(fs);
                const bool tm = ctx->opt.diag_seg != 0;
                if (S->split_proj) {
                    RMT_HIP(hipMemsetAsync(S->rowmark, 0, ny, S->st2));
                    if (tm) RMT_HIP(hipMemsetAsync(S->tmark, 0, S->max_tiles, S->st2));
                    k_mark_rows<<<list_grid(S->max_tiles), 64, 0, S->st2>>>(
                        S->tiles, S->tcount, (nx + MOM_TX - 1) / MOM_TX, ny, S->rowmark,
                        tm ? S->tmark : nullptr);
                    RMT_LAUNCHED();
                }
                MomWork Wf = W;
                if (tail_p) Wf.wait_p = S->e_tailp;   // (emit_tail above: p on another stream)
                const bool fl_ok = fluid_env && P.shape == RMT_SHAPE_DISC && nx % 64 == 0 &&
                                   MOM_TX == 64;
                // the SL pass also leaves phi, the known-plane words and per-tile fluid bits
                // (RMT_SL_PHI, default on): k_phi_rebuild_fluid's outputs without its pass
                const bool sl_phi = P.scheme == RMT_SCHEME_SEMILAGRANGIAN && S->e_bits &&
                                    fl_ok && ctx->opt.sl_phi;
                if (P.scheme == RMT_SCHEME_SEMILAGRANGIAN && S->e_bits) {
                    // the advection of every non-rim cell, once the chain has started (earlier
                    // its blocks would crowd out the one-workgroup band passes); with the
                    // zero-tile flags (sl_zero_flags, with sl_phi) the tiles that stay +0.0 move
                    // no map or phi bytes
                    const bool zon = sl_phi && S->zf[0] && ctx->opt.sl_zero_flags;
                    const int zi = S->zcur, zo = S->zcur ^ 1;
                    k_sim_sl_t<0><<<dim3((nx + SLT_X - 1) / SLT_X, (ny + SLT_Y - 1) / SLT_Y),
                                 SLT_X * SLT_Y, 0, S->st2>>>(
                        S->X1, S->X2, S->u, S->v, S->xs, S->ys, ny, nx, dt, divk_make(P.dx),
                        divk_make(P.dy), P.x0, P.y0, P.R, S->X1n, S->X2n, S->phi_pre, S->flag,
                        nullptr, sc, dtp, 2, S->rimw, sl_phi ? S->phi : nullptr,
                        fluid_threshold(&M), sl_phi ? fluid_bits_buf(W) : nullptr,
                        sl_phi ? nb : nullptr, 0, 0, zon && S->zv[zi] ? S->zf[zi] : nullptr,
                        zon ? S->zf[zo] : nullptr, zon && zo_valid);
                    RMT_LAUNCHED();
                    S->zv[zo] = zon;
                }
                seg_diag = sl_phi && S->split_proj && tm && !P.energies;
                if (sl_phi) {
                    Wf.fluid_bits = fluid_bits_buf(W);
                } else if (fl_ok) {
                    // phi and the stage kernels' pure-fluid flags in one pass
                    k_phi_rebuild_fluid<<<g, 256, 0, S->st2>>>(
                        S->X1n, S->X2n, n, nx, (nx + 63) / 64, P.x0, P.y0, P.R, S->phi, nullptr,
                        nullptr, nb, fluid_threshold(&M), fluid_rows_buf(W, 0, nx));
                    Wf.fluid_rows_ready = true;
                    RMT_LAUNCHED();
                } else {
                    k_phi_rebuild<<<g, 256, 0, S->st2>>>(S->X1n, S->X2n, n, P.shape, P.x0, P.y0,
                                                          P.R, S->phi, nullptr, nullptr, nb);
                    RMT_LAUNCHED();
                }
                ctx->stream = S->st2;
                int ms = momentum_rk4(ctx, &M, S->u, S->v, S->p, S->X1n, S->X2n, S->phi,
                                      S->us, S->vs, S->sxx, S->sxy, S->syy, S->J, Wf);
                if (ms == RMT_OK) ms = hipEventRecord(S->e_mom, S->st2) ? RMT_EDEVICE : RMT_OK;
                // and the projection's rows from the speculative u*, v* (the fix-up tiles the
                // main stream re-runs meanwhile only feed rows it redoes afterwards)
                if (ms == RMT_OK && S->split_proj)
                    ms = projection_rows(ctx, S->us, S->vs, P.dx, P.dy, dtp, dt, P.rho_f, S->p,
                                         nullptr, nullptr, nullptr, 0,
                                         ctx->opt.skip_marked_rows ? S->rowmark : nullptr);
                // and the row blocks no fix-up row falls in, transposed for the column pass
                if (ms == RMT_OK && S->split_proj && early_t_env) {
                    ms = dct_transpose_unmarked(ctx, ctx->scratch + n, S->rowmark);
                    early_t = ms == RMT_OK;
                }
                ctx->stream = st;
                RMT_TRY(ms);
                RMT_HIP(hipEventRecord(S->e_rows, S->st2));
            }
            if (S->prof) RMT_HIP(hipEventRecord(S->pev[3], st));
            // the flags (non-finite velocity, sweep aborted) are read with the diagnostics at
            // the end of the step: no host round trip between the chain and the projection
        }
        if (S->prof && !solid) {
            RMT_HIP(hipEventRecord(S->pev[2], st));
            RMT_HIP(hipEventRecord(S->pev[3], st));
        }
        // one join of the second stream instead of two (RMT_MERGED_JOIN, default on; not in
        // the parallel mode, whose values pass ends long before that stream's row passes):
        // e_rows, after the speculative momentum AND the projection's rows, here -- beside the
        // ~3 ms chain both are done -- and no second wait before the projection
        const bool mj_env = ctx->opt.merged_join != 0;
        const bool mjoin = overlap && mj_env && !par;
        if (overlap) {
            const int dly_main = ctx->opt.test_delay_main;
            if (dly_main) { k_delay<<<1, 1, 0, st>>>(dly_main); RMT_LAUNCHED(); }
            // 4 + 5 on the tiles the extrapolation can reach
            RMT_HIP(hipStreamWaitEvent(st, mjoin ? S->e_rows : S->e_mom, 0));
            const int tiles_x = (nx + MOM_TX - 1) / MOM_TX;
            // phi on the tiles and the momentum's prep there in one kernel (RMT_FUSED_FIXPREP,
            // default on where nx % 64 == 0), which also copies the extrapolation's status
            // the next step's geometry below starts once the known plane is final (e_kb)
            const bool geo_next = async && geo_env && nb && P.layers > 0 &&
                                  (it + 1 < nsteps || S->carry_on);
            if (fixprep) {
                RMT_TRY(fixup_phi_prep(ctx, &M, W, S->X1n, S->X2n, P.x0, P.y0, P.R, nullptr, nullptr,
                                       S->phi, nb, S->sxx, S->sxy, S->syy, S->J, S->tiles,
                                       S->tcount, S->max_tiles, extrap_status(ctx, P.layers),
                                       S->flag + 2, geo_next ? S->e_kb : nullptr));
            } else {
                k_phi_tiles<<<list_grid(S->max_tiles), 256, 0, st>>>(S->X1n, S->X2n, ny, nx, P.x0, P.y0, P.R,
                                                           S->phi, nullptr, nullptr, S->tiles, S->tcount,
                                                           tiles_x, nb);
                RMT_LAUNCHED();
            }
            if (geo_next) {
                // the next step's known plane is final (the phi kernel above): its rim words, rim
                // segments and extrapolation geometry on the second stream, beside the rest of
                // this step (nothing there uses them or the extrapolation workspace).  Issued
                // before the fix-up stages: after them its few-block kernels would share the CUs
                // with the projection's FFT passes (measured: the step no faster)
                hipStream_t sg = S->st2;
                if (!fixprep) RMT_HIP(hipEventRecord(S->e_kb, st));   // (else: with the prep)
                RMT_HIP(hipStreamWaitEvent(sg, S->e_kb, 0));
                // this step's diagnostics (phi, J: final after the fix-up prep) on the second
                // stream, beside the projection, instead of in the tail beside the next chain;
                // they land in the ring slot this step's record takes below.  diag_first: ahead
                // of the geometry, beside the latency-bound fix-up stages (behind it they
                // overlapped the projection's DCT passes)
                // J is final here only with the fused fix-up prep (it writes J and records e_kb
                // on completion); without it momentum_fixup's prep writes J on the main stream
                // later, so the diagnostics stay in the tail
                const bool early_diag = fixprep && side_tail && S->split_proj && !P.energies;
                auto diag_now = [&]() {
                    DiagArgs D{S->phi, S->J, S->xs, S->ys, S->u, S->v, S->X1n, S->X2n, ny, nx,
                               P.energies, P.dx, P.dy, P.w_t, P.rho_s, P.rho_f, P.mu_f, P.eta_s,
                               P.mu_s, P.kappa, 0, ny};
                    if (seg_diag) { D.fbits = fluid_bits_buf(W); D.tmark = S->tmark; }
                    diag_partials(D, S->dscr, sg, ctx->opt.diag_seg != 0);
                    k_diag_p2<<<1, DIAG_T, 0, sg>>>(S->dscr, S->ring + (size_t)slot * RING_VALS);
                    diag_early = true;
                };
                if (early_diag && ctx->opt.diag_first) { diag_now(); RMT_LAUNCHED(); }
                const long nseg = (long)ny * ((nx + 255) / 256);
                int *scount = S->segs + nseg;
                ctx->stream = sg;
                int gs = rim_words(ctx, nb, ny, nx, (nx + 63) / 64, S->rimw, S->rimcnt);
                if (gs == RMT_OK)
                    gs = hipMemsetAsync(scount, 0, sizeof(int), sg) ? RMT_EDEVICE : RMT_OK;
                if (gs == RMT_OK) {
                    k_rim_segments<<<grid1d(nseg, 256), 256, 0, sg>>>(S->rimw, ny, nx,
                                                                       S->segs, scount);
                    gs = extrap_geometry(ctx, S->X1n, S->X2n, nullptr, P.dx, P.dy, P.layers,
                                         S->X1n, S->X2n, nb);
                }
                ctx->stream = st;
                RMT_TRY(gs);
                RMT_HIP(hipEventRecord(S->e_geo, sg));
                geo_ready = true;
                if (early_diag && !ctx->opt.diag_first) { diag_now(); RMT_LAUNCHED(); }
            }
            RMT_TRY(momentum_fixup(ctx, &M, S->u, S->v, S->p, S->X1n, S->X2n, S->phi, S->us, S->vs,
                                   S->sxx, S->sxy, S->syy, S->J, W, S->tiles, S->tcount,
                                   S->max_tiles, nullptr, fixprep));
        } else {
            // 4. phi from the advected + extrapolated map (and the momentum's pure-fluid flags)
            if (fluid_env && P.shape == RMT_SHAPE_DISC && nx % 64 == 0 && MOM_TX == 64) {
                k_phi_rebuild_fluid<<<g, 256, 0, st>>>(
                    S->X1n, S->X2n, n, nx, (nx + 63) / 64, P.x0, P.y0, P.R, S->phi, nullptr,
                    nullptr, nb, fluid_threshold(&M), fluid_rows_buf(W, 0, nx));
                W.fluid_rows_ready = true;
            } else {
                k_phi_rebuild<<<g, 256, 0, st>>>(S->X1n, S->X2n, n, P.shape, P.x0, P.y0, P.R,
                                                  S->phi, nullptr, nullptr, nb);
            }
            RMT_LAUNCHED();
            if (par && async && geo_env && nb && P.layers > 0 && S->st2 && it + 1 < nsteps) {
                // the next step's extrapolation geometry (known plane nb) beside this step's
                // momentum and projection
                RMT_HIP(hipEventRecord(S->e_kb, st));
                RMT_HIP(hipStreamWaitEvent(S->st2, S->e_kb, 0));
                ctx->stream = S->st2;
                const int gs = extrap_geometry(ctx, S->X1n, S->X2n, nullptr, P.dx, P.dy,
                                               P.layers, S->X1n, S->X2n, nb);
                ctx->stream = st;
                RMT_TRY(gs);
                RMT_HIP(hipEventRecord(S->e_geo, S->st2));
                geo_ready = true;
            }
            // 5. momentum (RK4)
            RMT_TRY(momentum_rk4(ctx, &M, S->u, S->v, S->p, S->X1n, S->X2n, S->phi, S->us, S->vs,
                                 S->sxx, S->sxy, S->syy, S->J, W));
        }
        if (S->prof) RMT_HIP(hipEventRecord(S->pev[4], st));
        // 6. projection (constant density rho_f; Neumann DCT-I)
        if (overlap && S->split_proj) {
            // redo the rhs on the fix-up tiles (+1 cell) and the row DCT of the rows they
            // reach, then the column pass and the rest
            if (!mjoin) RMT_HIP(hipStreamWaitEvent(st, S->e_rows, 0));
            RMT_TRY(projection_rows(ctx, S->us, S->vs, P.dx, P.dy, dtp, dt, P.rho_f, S->p,
                                    S->rowmark, S->tiles, S->tcount, S->max_tiles));
            RMT_TRY(projection_finish(ctx, S->us, S->vs, P.dx, P.dy, dtp, dt, P.rho_f, P.bc_kind,
                                      P.lid, S->p, S->u, S->v, S->p,
                                      async ? S->m2part : nullptr, !(async && side_tail),
                                      early_t ? S->rowmark : nullptr));
            early_t = false;
        } else if (async)
            RMT_TRY(projection_dev(ctx, S->us, S->vs, P.dx, P.dy, dtp, P.rho_f, P.bc_kind, P.lid,
                                   S->p, S->u, S->v, S->p, S->m2part));
        else
            RMT_TRY(rmt_pressure_projection(ctx, S->us, S->vs, P.dx, P.dy, dt, P.rho_f,
                                            P.bc_kind, P.lid, S->p, S->u, S->v, S->p));
        if (S->prof) RMT_HIP(hipEventRecord(S->pev[5], st));
        m2_last = async;
        // the advected + extrapolated map (X1n, X2n) is the state from here on: the two map
        // buffers swap roles instead of copying the map back (restored at the call's end)
        std::swap(S->X1, S->X1n);
        std::swap(S->X2, S->X2n);
        S->zcur ^= 1;
        // 7. diagnostics (running them beside the projection on the second stream measured
        // no gain: both are HBM-bound)
        DiagArgs D{S->phi, S->J, S->xs, S->ys, S->u, S->v, S->X1, S->X2, ny, nx, P.energies,
                   P.dx, P.dy, P.w_t, P.rho_s, P.rho_f, P.mu_f, P.eta_s, P.mu_s, P.kappa, 0, ny};
        if (async && overlap && S->split_proj && side_tail) {
            // p -= mean(p) and the diagnostics on the second stream: nothing before the next
            // step's chain reads p or writes what they read (that stream's next work -- the
            // speculative phi, momentum -- is queued behind them)
            double *e = S->ring + (size_t)slot * RING_VALS;
            pend_e = e;
            pending = true;
            pend_seg = seg_diag;
            pend_diag_done = diag_early;
            diag_early = false;
            ring_e = e;
            if (nb) { std::swap(S->kbits, S->kbits_next); S->bits_ready = true; }
            if (++slot == S->sync_every) RMT_TRY(flush());
            continue;
        }
        diag_partials(D, S->dscr, st, ctx->opt.diag_seg != 0);
        if (async) {
            double *e = S->ring + (size_t)slot * RING_VALS;
            k_diag_p2<<<1, DIAG_T, 0, st>>>(S->dscr, e);
            RMT_LAUNCHED();
            ring_e = e;
            if (nb) { std::swap(S->kbits, S->kbits_next); S->bits_ready = true; }
            if (++slot == S->sync_every) RMT_TRY(flush());
            continue;
        }
        k_diag_p2<<<1, DIAG_T, 0, st>>>(S->dscr, sc + 2);
        RMT_LAUNCHED();
        double dv[DIAG_VALS];
        int fl[4] = {0, 0, 0, 0};   // non-finite, (momentum), fitted, sweep aborted
        RMT_HIP(hipMemcpyAsync(dv, sc + 2, sizeof(dv), hipMemcpyDeviceToHost, st));
        if (solid) RMT_HIP(hipMemcpyAsync(fl, S->flag, sizeof(fl), hipMemcpyDeviceToHost, st));
        if (S->prof) RMT_HIP(hipEventRecord(S->pev[6], st));
        RMT_HIP(hipStreamSynchronize(st));
        if (S->prof) {
            float f;
            for (int k = 0; k < 6; ++k) {
                RMT_HIP(hipEventElapsedTime(&f, S->pev[k], S->pev[k + 1]));
                S->ms[k] += f; S->calls[k] += 1;
            }
            RMT_HIP(hipEventElapsedTime(&f, ctx->ev[0], ctx->ev[1]));
            S->ms[6] += f; S->calls[6] += 4;
            if (solid) {
                RMT_HIP(hipEventElapsedTime(&f, ctx->ev[2], ctx->ev[3]));
                S->ms[7] += f; S->calls[7] += 1;
            }
        }
        if (nb) { std::swap(S->kbits, S->kbits_next); S->bits_ready = true; }
        RMT_TRY(sim_record(S, dv, hv[0], dt, fl));
    }
    // the geometry prepared for a next call is joined here: nothing of this call stays in
    // flight on the second stream (the caller may reuse the context's workspace)
    if (geo_ready) RMT_HIP(hipStreamWaitEvent(st, S->e_geo, 0));
    RMT_TRY(flush());
    S->carry_valid = S->carry_on && geo_ready;
    S->m2_valid = m2_last;
    S->carry_gen = ctx->bytes_gen;
    S->carry_cfg = extrap_config_gen();
    return RMT_OK;
}

int rmt_sim_set_carry(rmt_sim *S, int on) {
    RMT_CHECK(S, RMT_EINVAL, "null sim");
    S->carry_on = on != 0;
    S->carry_valid = false;
    return RMT_OK;
}

int rmt_sim_invalidate(rmt_sim *S) {
    RMT_CHECK(S, RMT_EINVAL, "null sim");
    S->carry_valid = false;
    return RMT_OK;
}

int rmt_sim_set_sync_every(rmt_sim *S, int k) {
    RMT_CHECK(S, RMT_EINVAL, "null sim");
    RMT_CHECK(k >= 1 && k <= RING_N, RMT_EINVAL, "rmt_sim_set_sync_every: k must be 1 .. 64");
    S->sync_every = k;
    return RMT_OK;
}

int rmt_sim_set_profiling(rmt_sim *S, int on) {
    RMT_CHECK(S, RMT_EINVAL, "null sim");
    if (on && !S->pev[0]) {
        for (auto &e : S->pev) RMT_HIP(hipEventCreate(&e));
        if (!S->ctx->ev[0])
            for (auto &e : S->ctx->ev) RMT_HIP(hipEventCreate(&e));
    }
    S->prof = on != 0;
    S->ctx->prof = on != 0;
    for (int k = 0; k < 8; ++k) { S->ms[k] = 0; S->calls[k] = 0; }
    return RMT_OK;
}

int rmt_sim_phase_times(rmt_sim *S, double *ms8, long *calls8) {
    RMT_CHECK(S && ms8, RMT_EINVAL, "null argument");
    for (int k = 0; k < 8; ++k) {
        ms8[k] = S->ms[k];
        if (calls8) calls8[k] = S->calls[k];
    }
    return RMT_OK;
}

int rmt_sim_diagnostics(rmt_sim *S, rmt_diag *out, int max_records, int *n_records) {
    RMT_CHECK(S && n_records, RMT_EINVAL, "null argument");
    int m = (int)std::min<size_t>(S->diag.size(), (size_t)std::max(0, max_records));
    for (int k = 0; k < m; ++k) out[k] = S->diag[S->diag.size() - m + k];
    *n_records = (int)S->diag.size();
    return RMT_OK;
}

}  // extern "C"
