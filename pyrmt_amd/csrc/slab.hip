// slab.hip -- the RMT loop body decomposed into row slabs.
//
// One rmt_slab owns rows [r0, r1) of the global NY x NX grid and keeps HALO rows on each
// side resident (rows [lo, hi), clipped to the grid).  Every plane is addressed with GLOBAL
// cell indices j*NX + i (pointers offset by -lo*NX), so the per-cell arithmetic, the
// boundary tests and the node coordinates are those of the single-domain step (sim.hip)
// and the decomposed step reproduces it bit for bit.  The caller runs the phases below on
// every slab and performs the collectives between them (pyrmt_amd/distributed.py:
// torch.distributed over RCCL, or in-process copies for virtual ranks):
//
//   halo(u, v, p, X1, X2; HALO rows)        -- start of step
//   advect            SL-RK4 of the map on rows r0-10 .. r1+10, phi_pre, known bits (owned)
//   allgather(known bit rows)
//   rim_pack          the cells within 7 of the known/unknown interface, (index, X1, X2)
//   allgather(rim entries)                  -- a few hundred KB at N = 4096
//   extrapolate       dense replica of the band, the exact raster-order chain (extrap*.hip)
//                     run redundantly on every slab, rim written back, phi rebuilt
//   momentum          prep + 4 RK4 stages on shrinking row windows (2 rows per stage)
//   project_rows      Rhie-Chow divergence, rhs, DCT-I along x, column blocks packed
//   all_to_all        slab -> column blocks
//   project_cols      DCT-I along y, / eig, inverse along y (fused)
//   all_to_all        back
//   project_unrows    inverse DCT-I along x; row-tree root of p_c
//   allgather(roots); sub_mean(p_c); halo(p_c; 2 rows)
//   project_correct   velocity correction + BC, p = p_prev + p_c; row-tree root of p
//   allgather(roots); sub_mean(p)
//   finish            diagnostics partials, max|u|^2 for the next dt, flags
//   allgather(scalars)
//
// Why the extrapolation is exact: it reads values only at known cells inside the 9x9 window
// of a target, targets lie within 3 cells of the known set, so every value it reads or
// writes is within 7 cells (Chebyshev) of a known/unknown pair -- the rim.  Acceptance,
// weights and the target order depend on the known set alone, which every slab holds as a
// full bit plane.  The dense replica therefore sees exactly the inputs of the single-domain
// call at every cell it touches.
#include "rmt_internal.hpp"
#include "extrap.hpp"
#include <algorithm>
#include <vector>

using rmt::u64;

namespace rmt {
constexpr int SLAB_MAXG = 64;
enum { SC_M2 = 0, SC_DIAG = 1, SC_FLAGS = 11, SC_COUNT = 12, SC_ROOT = 13, SC_FIT = 14,
       SC_M2RES = 15, SC_N = 16, SC_M2OWN = 16 /* device-only, past the exported block */,
       SC_DT = 20, SC_M2G = 21 /* device dt: this step's dt and the max |u|^2 it came from */ };
enum { FL_NONFINITE = 1, FL_HALO = 2, FL_EXABORT = 4, FL_RIMCAP = 8 };
struct Splits { int v[SLAB_MAXG + 1]; };
struct Counts { long long c[SLAB_MAXG]; };
}  // namespace rmt

struct rmt_slab {
    rmt_ctx *ctx = nullptr;
    rmt_sim_params P{};
    int G = 1, rank = 0, NY = 0, NX = 0, W = 0;
    int r0 = 0, r1 = 0, lo = 0, hi = 0, c0 = 0, c1 = 0;
    rmt::Splits rs{}, cs{};
    double dt_const = 0;
    void *block = nullptr;
    // resident planes ((hi - lo) x NX), LOCAL base pointers
    double *u, *v, *p, *X1, *X2, *phi, *phi_pre, *J, *X1n, *X2n, *us, *vs, *sxx, *sxy, *syy;
    double *pc, *rhs, *mw;
    unsigned char *solid;
    double *X1d, *X2d;     // dense NY x NX (extrapolation replica)
    u64 *bits;             // NY x W known plane
    u64 *rimw;             // (r1 - r0) x W rim words
    int *rowcnt;           // r1 - r0 + 1
    double *rim;           // 3 doubles per owned cell (index, X1, X2)
    double *A, *B, *T, *Y; // DCT: owned x NX, NY x nc, nc x NY, owned x NX
    double *xs, *ys;
    double *scal, *part;
    int *flags;            // [0] flags, [4..5] extrapolation {fitted, aborted}
    // the momentum beside the (replicated) chain, as rmt_sim_step: a speculative pass on a
    // second stream from the pre-extrapolation map, re-run on the tiles a target can reach
    hipStream_t st2 = nullptr;
    hipEvent_t e_chain = nullptr, e_mom = nullptr;
    int *tiles = nullptr, *tcount = nullptr, max_tiles = 0;
    double dt_cur = 0;
    // device dt (rmt_slab_set_device_dt): the step's kernels read dt from *dtp instead of the
    // host argument, and the rim counts come from the gathered scalars (rmt_slab_extrapolate_dev)
    const double *dtp = nullptr;
    bool spec = false;     // a speculative momentum is in flight for this step
    bool interior = false; // rmt_slab_advect_interior ran for this step
    // the next step's extrapolation geometry beside this step's projection (as rmt_sim_step):
    // the next known plane (bits_next: owned rows from phi after the fix-up, then allgathered)
    // and the geometry on st2 into this slab's own extrapolation workspace (ws; slabs sharing
    // a context must not share it while geometries run beside other slabs' chains)
    u64 *bits_next = nullptr;
    unsigned char *ws = nullptr;
    size_t ws_len = 0;
    hipEvent_t e_bits = nullptr, e_geo = nullptr;
    bool geo_ready = false;
    double *gv(double *q) const { return q - (long)lo * NX; }   // global-index view
};

namespace rmt {

// test switch test_delay_geo: ~3.4 us x n of sleep ahead of an early geometry on st2
__global__ void k_slab_delay(int n) {
    for (int k = 0; k < n; ++k) __builtin_amdgcn_s_sleep(127);
}

// ------------------------------------------------------------------- advection --
// k_sim_sl (sim.hip) on rows [jb, je) with the bilinear rows checked against [lo, hi)
__global__ void k_slab_sl(const double *__restrict__ X1, const double *__restrict__ X2,
                          const double *__restrict__ a, const double *__restrict__ b,
                          const double *__restrict__ xs, const double *__restrict__ ys, int ny,
                          int nx, double dt, DivK Kx, DivK Ky, double x0, double y0, double R,
                          double *__restrict__ X1n, double *__restrict__ X2n,
                          double *__restrict__ phi_pre, int *flags, int jb, int je, int lo,
                          int hi, const double *m2, const double *__restrict__ dtp) {
    // grid (ceil(nx / 256), je - jb); the block skip of sl_zero_block (rmt_internal.hpp) with
    // m2 bounding the velocities of the resident rows
    if (dtp) dt = *dtp;
    const int j = jb + blockIdx.y, i0 = blockIdx.x * 256, i = i0 + threadIdx.x;
    const bool zero = sl_skip_ok(m2, dt, fmin(Kx.d, Ky.d)) &&
                      sl_zero_block(X1, X2, ny, nx, j, i0, 256, lo, hi);
    if (i >= nx) return;
    const long c = (long)j * nx + i;
    if (zero) {   // map +0.0 around: no loads (m2 finite: every velocity is)
        phi_pre[c] = disc_phi(0.0, 0.0, x0, y0, R);
        X1n[c] = 0.0; X2n[c] = 0.0;
        return;
    }
    if (!(isfinite(a[c]) && isfinite(b[c]))) atomicOr(flags, FL_NONFINITE);
    const double ph = disc_phi(X1[c], X2[c], x0, y0, R);
    phi_pre[c] = ph;
    const double m = ph <= 0 ? 1.0 : 0.0;
    bool oob = false;
    double xb, yb;
    sl_backtrace_t<true>(a, b, xs[i], ys[j], dt, Kx, Ky, nx, ny, lo, hi, &oob, xb, yb);
    X1n[c] = bilinear_t<true>(X1, xb, yb, Kx, Ky, nx, ny, lo, hi, &oob) * m;
    X2n[c] = bilinear_t<true>(X2, xb, yb, Kx, Ky, nx, ny, lo, hi, &oob) * m;
    if (oob) atomicOr(flags, FL_HALO);
}

// known bits (phi < 0, as k_ex_bits) of rows [r0, r1)
__global__ void __launch_bounds__(256) k_slab_bits(const double *__restrict__ phi, int nx, int W,
                                                   u64 *__restrict__ bits, int r0) {
    const int j = r0 + blockIdx.y, i = blockIdx.x * 256 + threadIdx.x;
    const bool k = i < nx && phi[(long)j * nx + i] < 0;
    const u64 m = __ballot(k);
    if ((threadIdx.x & 63) == 0 && (i >> 6) < W) bits[(long)j * W + (i >> 6)] = m;
}

// ------------------------------------------------------------------------- rim --
__device__ __forceinline__ u64 col_mask(int w, int W, int nx) {
    if (w < 0 || w >= W) return 0;
    const int r = nx - 64 * w;
    return r >= 64 ? ~0ull : ((1ull << r) - 1);
}
// Chebyshev dilation by 7 along a row of words (a | b | e = words w-1, w, w+1)
__device__ __forceinline__ u64 hdil7(u64 a, u64 b, u64 e) {
    u64 h = b;
#pragma unroll
    for (int s = 1; s <= 7; ++s) h |= (b << s) | (a >> (64 - s)) | (b >> s) | (e << (64 - s));
    return h;
}
// rim words of rows [r0, r1): cells whose 15x15 box holds a known and an unknown cell;
// one wave per row, per-row counts
__global__ void __launch_bounds__(256) k_rim_words(const u64 *__restrict__ bits, int ny, int nx,
                                                   int W, int r0, int r1, u64 *__restrict__ rimw,
                                                   int *__restrict__ rowcnt) {
    const int lane = threadIdx.x & 63, j = r0 + blockIdx.x * 4 + (threadIdx.x >> 6);
    if (j >= r1) return;
    int cnt = 0;
    for (int w = lane; w < W; w += 64) {
        u64 K[3] = {0, 0, 0}, U[3] = {0, 0, 0};
        for (int jj = max(0, j - 7); jj <= min(ny - 1, j + 7); ++jj) {
#pragma unroll
            for (int d = 0; d < 3; ++d) {
                const int ww = w - 1 + d;
                const u64 cm = col_mask(ww, W, nx);
                const u64 k = cm ? bits[(long)jj * W + ww] : 0;
                K[d] |= k;
                U[d] |= ~k & cm;
            }
        }
        const u64 r = hdil7(K[0], K[1], K[2]) & hdil7(U[0], U[1], U[2]) & col_mask(w, W, nx);
        rimw[(long)(j - r0) * W + w] = r;
        cnt += __popcll(r);
    }
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) cnt += __shfl_xor(cnt, d);
    if (lane == 0) rowcnt[j - r0] = cnt;
}
// exclusive scan of n <= 8192 row counts in place; total -> *total
__global__ void __launch_bounds__(1024) k_rim_scan(int *__restrict__ cnt, int n,
                                                   double *__restrict__ total) {
    __shared__ long long s[1024];
    const int per = (n + 1023) / 1024, t = threadIdx.x, a = t * per, b = min(n, a + per);
    long long loc = 0;
    for (int k = a; k < b; ++k) loc += cnt[k];
    s[t] = loc;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {
        const long long x = t >= d ? s[t - d] : 0;
        __syncthreads();
        s[t] += x;
        __syncthreads();
    }
    long long run = s[t] - loc;
    for (int k = a; k < b; ++k) { const int c = cnt[k]; cnt[k] = (int)run; run += c; }
    if (t == 1023) *total = (double)s[1023];
}
// (global index, X1, X2) of every rim cell, raster order
__global__ void __launch_bounds__(256) k_rim_emit(const u64 *__restrict__ rimw,
                                                  const int *__restrict__ rowoff, int W, int nx,
                                                  int r0, int r1, const double *__restrict__ X1,
                                                  const double *__restrict__ X2,
                                                  double *__restrict__ rim) {
    const int lane = threadIdx.x & 63, j = r0 + blockIdx.x * 4 + (threadIdx.x >> 6);
    if (j >= r1) return;
    long base = rowoff[j - r0];
    for (int w0 = 0; w0 < W; w0 += 64) {
        const int w = w0 + lane;
        u64 m = w < W ? rimw[(long)(j - r0) * W + w] : 0;
        const int pc = __popcll(m);
        int inc = pc;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int t = __shfl_up(inc, d);
            if (lane >= d) inc += t;
        }
        long e = base + inc - pc;
        while (m) {
            const int bit = __builtin_ctzll(m);
            m &= m - 1;
            const long c = (long)j * nx + 64 * w + bit;
            rim[3 * e] = (double)c;
            rim[3 * e + 1] = X1[c];
            rim[3 * e + 2] = X2[c];
            ++e;
        }
        base += __shfl(inc, 63);
    }
}
// gathered rim counts: on the host (cn) or in the gathered scalar blocks (gs, G x SC_N: the
// device-dt path, counts capped at cap -- an overflow is flagged by k_rim_cap)
__device__ __forceinline__ long rim_count(const Counts &cn, const double *gs, int k, long cap) {
    return gs ? min((long)gs[(long)k * SC_N + SC_COUNT], cap) : cn.c[k];
}
__global__ void k_rim_unpack(const double *__restrict__ g, Counts cn, int G, long cap,
                             double *__restrict__ X1d, double *__restrict__ X2d,
                             const double *__restrict__ gs) {
    const long q = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (q >= G * cap) return;
    const int k = (int)(q / cap);
    if (q - k * cap >= rim_count(cn, gs, k, cap)) return;
    const long c = (long)g[3 * q];
    X1d[c] = g[3 * q + 1];
    X2d[c] = g[3 * q + 2];
}
__global__ void k_rim_writeback(const double *__restrict__ g, Counts cn, int G, long cap,
                                const double *__restrict__ X1d, const double *__restrict__ X2d,
                                double *__restrict__ X1n, double *__restrict__ X2n, long c_lo,
                                long c_hi, const double *__restrict__ gs) {
    const long q = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (q >= G * cap) return;
    const int k = (int)(q / cap);
    if (q - k * cap >= rim_count(cn, gs, k, cap)) return;
    const long c = (long)g[3 * q];
    if (c < c_lo || c >= c_hi) return;
    X1n[c] = X1d[c];
    X2n[c] = X2d[c];
}
// k_phi_rebuild (sim.hip) on rows [jb, je): phi from the extrapolated map, map copied back
__global__ void k_slab_phi(const double *__restrict__ X1n, const double *__restrict__ X2n,
                           double x0, double y0, double R, int nx, int jb, int je,
                           double *__restrict__ phi, double *__restrict__ X1,
                           double *__restrict__ X2) {
    const long c = (long)jb * nx + blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (c >= (long)je * nx) return;
    const double a = X1n[c], b = X2n[c];
    X1[c] = a; X2[c] = b;
    phi[c] = disc_phi(a, b, x0, y0, R);
}

// k_slab_phi on the listed fix-up tiles, rows [jb, je) only
__global__ void __launch_bounds__(256) k_slab_phi_tiles(const double *__restrict__ X1n,
                                                        const double *__restrict__ X2n,
                                                        double x0, double y0, double R, int nx,
                                                        int jb, int je, double *__restrict__ phi,
                                                        double *__restrict__ X1,
                                                        double *__restrict__ X2,
                                                        const int *__restrict__ tiles,
                                                        const int *__restrict__ count,
                                                        int tiles_x) {
    if ((int)blockIdx.x >= *count) return;
    const int t = tiles[blockIdx.x];
    const int i0 = (t % tiles_x) * MOM_TX, j0 = (t / tiles_x) * MOM_TY;
    for (int q = threadIdx.x; q < MOM_TX * MOM_TY; q += 256) {
        const int j = j0 + q / MOM_TX, i = i0 + q % MOM_TX;
        if (j < jb || j >= je || i >= nx) continue;
        const long c = (long)j * nx + i;
        const double a = X1n[c], b = X2n[c];
        X1[c] = a; X2[c] = b;
        phi[c] = disc_phi(a, b, x0, y0, R);
    }
}

// ------------------------------------------------------------------ device dt --
// ring (nullable) <- {this step's dt, the max |u|^2 it came from, the gathered scalar blocks};
// then the next dt from the gathered max |u|^2 (NaN-propagating, as numpy's max), with the
// host's expression (distributed.py: min(dt_const, cfl dx / (sqrt(m2) + 1e-6)); Python's
// min(dt_const, nan) is dt_const, as fmin)
__global__ void k_slab_dt(const double *__restrict__ gs, int G, double dt_const, double cfl,
                          double dx, double *__restrict__ scal, double *__restrict__ ring) {
    if (threadIdx.x != 0) {
        if (ring)
            for (int q = threadIdx.x - 1; q < G * SC_N; q += blockDim.x - 1) ring[2 + q] = gs[q];
        return;
    }
    if (ring) { ring[0] = scal[SC_DT]; ring[1] = scal[SC_M2G]; }
    double m2 = gs[SC_M2];
    for (int k = 1; k < G; ++k) {
        const double x = gs[(long)k * SC_N + SC_M2];
        if (x > m2 || x != x) m2 = x;
    }
    scal[SC_M2G] = m2;
    scal[SC_DT] = fmin(dt_const, cfl * dx / (sqrt(m2) + 1e-6));
}
// the rim allgather moves `cap` entries per slab: a larger count is flagged (the host raises)
__global__ void k_rim_cap(const double *__restrict__ scal, long cap, int *__restrict__ flags) {
    if (scal[SC_COUNT] > (double)cap) atomicOr(flags, FL_RIMCAP);
}

// ------------------------------------------------------------------ projection --
// owned rows x NX  <->  per-destination column blocks (rows x nc_m at offset rows * c0_m)
template <bool PACK>
__global__ void k_cols(double *__restrict__ Y, int rows, int nx, Splits cs, int G,
                       double *__restrict__ A) {
    const long q = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (q >= (long)rows * nx) return;
    const int r = (int)(q / nx), c = (int)(q % nx);
    int m = 0;
    while (m + 1 < G && c >= cs.v[m + 1]) ++m;
    const int c0 = cs.v[m], nc = cs.v[m + 1] - c0;
    const long o = (long)rows * c0 + (long)r * nc + (c - c0);
    if (PACK) A[o] = Y[q];
    else Y[q] = A[o];
}
__global__ void k_flags_out(const int *__restrict__ flags, double *__restrict__ scal) {
    scal[SC_FLAGS] = (double)(flags[0] | (flags[5] ? FL_EXABORT : 0));
    // an aborted extrapolation reports its abort word (extrap.hpp EXA_*) instead of the count
    scal[SC_FIT] = flags[5] ? -(double)flags[5] : (double)flags[4];
}

static int check_splits(const int *s, int G, int n, int minsz, bool even) {
    if (s[0] != 0 || s[G] != n) return RMT_EINVAL;
    for (int k = 0; k < G; ++k) {
        if (s[k + 1] - s[k] < minsz) return RMT_EINVAL;
        if (even && (s[k] & 1)) return RMT_EINVAL;
    }
    return RMT_OK;
}


// this slab's extrapolation workspace as the context's byte scratch for the scope (written
// back: ensure_bytes may reallocate it)
struct SlabWs {
    rmt_slab *S;
    unsigned char *b;
    size_t l;
    explicit SlabWs(rmt_slab *s) : S(s), b(s->ctx->bytes), l(s->ctx->bytes_len) {
        ++S->ctx->bytes_gen;
        if (S->ws) { S->ctx->bytes = S->ws; S->ctx->bytes_len = S->ws_len; }
    }
    ~SlabWs() {
        if (!S->ws) return;
        S->ws = S->ctx->bytes; S->ws_len = S->ctx->bytes_len;
        S->ctx->bytes = b; S->ctx->bytes_len = l;
    }
};

// ------------------------------------------- shared with the MAC slabs (mac.hip) --
int slab_sl(rmt_ctx *ctx, const double *X1, const double *X2, const double *a, const double *b,
            const double *xs, const double *ys, int ny, int nx, double dt, double dx, double dy,
            double x0, double y0, double R, double *X1n, double *X2n, double *phi_pre,
            int *flags, int jb, int je, int lo, int hi, const double *dev_m2) {
    if (je <= jb) return RMT_OK;
    k_slab_sl<<<dim3((nx + 255) / 256, je - jb), 256, 0, ctx->stream>>>(
        X1, X2, a, b, xs, ys, ny, nx, dt, divk_make(dx), divk_make(dy), x0, y0, R, X1n, X2n, phi_pre, flags, jb, je,
        lo, hi, dev_m2, nullptr);
    RMT_LAUNCHED();
    return RMT_OK;
}

int slab_bits(rmt_ctx *ctx, const double *phi, int nx, int W, u64 *bits, int r0, int r1) {
    k_slab_bits<<<dim3((nx + 255) / 256, r1 - r0), 256, 0, ctx->stream>>>(phi, nx, W, bits, r0);
    RMT_LAUNCHED();
    return RMT_OK;
}

int slab_rim_pack(rmt_ctx *ctx, const u64 *bits, int ny, int nx, int W, int r0, int r1,
                  u64 *rimw, int *rowcnt, const double *X1n, const double *X2n, double *rim,
                  double *count) {
    const int rows = r1 - r0;
    k_rim_words<<<(rows + 3) / 4, 256, 0, ctx->stream>>>(bits, ny, nx, W, r0, r1, rimw, rowcnt);
    k_rim_scan<<<1, 1024, 0, ctx->stream>>>(rowcnt, rows, count);
    k_rim_emit<<<(rows + 3) / 4, 256, 0, ctx->stream>>>(rimw, rowcnt, W, nx, r0, r1, X1n, X2n,
                                                        rim);
    RMT_LAUNCHED();
    return RMT_OK;
}

// rim words of the whole grid (the fused step's split advection, sim.hip)
int rim_words(rmt_ctx *ctx, const u64 *bits, int ny, int nx, int W, u64 *rimw, int *rowcnt) {
    k_rim_words<<<(ny + 3) / 4, 256, 0, ctx->stream>>>(bits, ny, nx, W, 0, ny, rimw, rowcnt);
    RMT_LAUNCHED();
    return RMT_OK;
}

int slab_rim_extrapolate(rmt_ctx *ctx, const double *gathered, const long long *counts, int G,
                         long long cap, double *X1d, double *X2d, const u64 *bits, double dx,
                         double dy, int layers, int *exflags, double *X1n, double *X2n,
                         long c_lo, long c_hi, const double *gs, hipEvent_t geo) {
    Counts cn{};
    for (int k = 0; k < G && !gs; ++k) {
        RMT_CHECK(counts[k] >= 0 && counts[k] <= cap, RMT_EINVAL, "slab: rim count > cap");
        cn.c[k] = counts[k];
    }
    const long tot = (long)G * cap;
    if (tot > 0) {
        k_rim_unpack<<<grid1d(tot, 256), 256, 0, ctx->stream>>>(gathered, cn, G, cap, X1d, X2d, gs);
        RMT_LAUNCHED();
    }
    if (geo && layers > 0) {   // the geometry ran beside the previous step's projection
        RMT_HIP(hipStreamWaitEvent(ctx->stream, geo, 0));
        RMT_TRY(extrap_finish(ctx, dx, dy, layers, X1d, X2d, exflags));
    } else {
        RMT_TRY(extrapolate(ctx, X1d, X2d, nullptr, dx, dy, layers, X1d, X2d, exflags, bits));
    }
    if (tot > 0) {
        k_rim_writeback<<<grid1d(tot, 256), 256, 0, ctx->stream>>>(gathered, cn, G, cap, X1d, X2d,
                                                                   X1n, X2n, c_lo, c_hi, gs);
        RMT_LAUNCHED();
    }
    return RMT_OK;
}

int slab_cols(rmt_ctx *ctx, bool pack, double *Y, int rows, int nx, const int *csplits, int G,
              double *A) {
    Splits cs{};
    for (int k = 0; k <= G; ++k) cs.v[k] = csplits[k];
    const long no = (long)rows * nx;
    if (no == 0) return RMT_OK;
    if (pack) k_cols<true><<<grid1d(no, 256), 256, 0, ctx->stream>>>(Y, rows, nx, cs, G, A);
    else k_cols<false><<<grid1d(no, 256), 256, 0, ctx->stream>>>(Y, rows, nx, cs, G, A);
    RMT_LAUNCHED();
    return RMT_OK;
}

}  // namespace rmt

using namespace rmt;

#define SLAB_RW(S) RowWin{0, 0, (S)->lo, (S)->hi}
static int slab_momentum_pass(rmt_slab *S, double dt, bool fixup);

extern "C" {

int rmt_slab_create(rmt_ctx *ctx, const rmt_sim_params *prm, int G, int rank,
                    const int *row_splits, const int *col_splits, rmt_slab **out) {
    RMT_CHECK(ctx && prm && row_splits && col_splits && out, RMT_EINVAL, "null argument");
    RMT_CHECK(G >= 1 && G <= SLAB_MAXG && rank >= 0 && rank < G, RMT_EINVAL, "slab: bad G/rank");
    RMT_CHECK(prm->ny == ctx->ny && prm->nx == ctx->nx, RMT_EINVAL, "slab: ctx must be global");
    RMT_CHECK(prm->scheme == RMT_SCHEME_SEMILAGRANGIAN && prm->shape == RMT_SHAPE_DISC,
              RMT_ENOTSUP, "slab step: semi-Lagrangian disc configurations (configs 2/4)");
    RMT_CHECK(prm->rho_s == prm->rho_f, RMT_ENOTSUP, "slab step: constant density only");
    RMT_CHECK(!prm->energies, RMT_ENOTSUP, "slab step: per-step energies (config 3) not decomposed");
    RMT_CHECK(prm->bc_kind >= 0 && prm->bc_kind <= 2, RMT_EINVAL, "unknown bc kind");
    RMT_CHECK(prm->ny <= 8192 && prm->nx <= 8192, RMT_ENOTSUP, "slab step: N <= 8192");
    RMT_CHECK(check_splits(row_splits, G, prm->ny, RMT_SLAB_HALO, true) == RMT_OK, RMT_EINVAL,
              "slab: row splits must be even, increasing, >= RMT_SLAB_HALO rows each");
    RMT_CHECK(check_splits(col_splits, G, prm->nx, 2, true) == RMT_OK, RMT_EINVAL,
              "slab: column splits must be even, increasing, >= 2 columns each");
    RMT_TRY(dct_plan(ctx, prm->dx, prm->dy));
    RMT_CHECK(dct_lds_ready(ctx), RMT_ENOTSUP,
              "slab step: 2(N-1) must factor into radices <= 23 (LDS DCT-I)");
    rmt_slab *S = new rmt_slab;
    S->ctx = ctx; S->P = *prm; S->P.xs = S->P.ys = nullptr;
    S->G = G; S->rank = rank; S->NY = prm->ny; S->NX = prm->nx; S->W = (prm->nx + 63) / 64;
    for (int k = 0; k <= G; ++k) { S->rs.v[k] = row_splits[k]; S->cs.v[k] = col_splits[k]; }
    S->r0 = row_splits[rank]; S->r1 = row_splits[rank + 1];
    S->c0 = col_splits[rank]; S->c1 = col_splits[rank + 1];
    S->lo = std::max(0, S->r0 - RMT_SLAB_HALO); S->hi = std::min(S->NY, S->r1 + RMT_SLAB_HALO);
    const long NX = S->NX, nl = (long)(S->hi - S->lo) * NX, no = (long)(S->r1 - S->r0) * NX;
    const long nd = (long)S->NY * NX, nc = S->c1 - S->c0;
    const long W = S->W;
    size_t dbl = 18 * nl + MOM_WORK_PLANES * nl + 2 * nd + 3 * no + 2 * no + 2 * nc * S->NY +
                 NX + S->NY + SC_N * 4 + DIAG_PART;
    size_t bytes = dbl * 8 + (size_t)S->NY * W * 8 + (size_t)(S->r1 - S->r0) * W * 8 +
                   (S->r1 - S->r0 + 64) * 4 + nl + 256;
    RMT_HIP(hipMalloc(&S->block, bytes));
    RMT_HIP(hipMemsetAsync(S->block, 0, bytes, ctx->stream));
    double *q = (double *)S->block;
    double **pl[] = {&S->u, &S->v, &S->p, &S->X1, &S->X2, &S->phi, &S->phi_pre, &S->J, &S->X1n,
                     &S->X2n, &S->us, &S->vs, &S->sxx, &S->sxy, &S->syy, &S->pc, &S->rhs};
    for (auto pp : pl) { *pp = q; q += nl; }
    q += nl;   // spare
    S->mw = q; q += MOM_WORK_PLANES * nl;
    S->X1d = q; q += nd;
    S->X2d = q; q += nd;
    S->rim = q; q += 3 * no;
    S->A = q; q += no;
    S->Y = q; q += no;
    S->B = q; q += nc * S->NY;
    S->T = q; q += nc * S->NY;
    S->xs = q; q += NX;
    S->ys = q; q += S->NY;
    S->scal = q; q += SC_N * 4;
    S->part = q; q += DIAG_PART;
    S->bits = (u64 *)q; S->rimw = S->bits + (long)S->NY * W;
    S->rowcnt = (int *)(S->rimw + (long)(S->r1 - S->r0) * W);
    S->flags = S->rowcnt + (S->r1 - S->r0 + 64) - 16;
    S->solid = (unsigned char *)(S->rowcnt + (S->r1 - S->r0 + 64));
    RMT_HIP(hipMemcpyAsync(S->xs, prm->xs, NX * 8, hipMemcpyHostToDevice, ctx->stream));
    RMT_HIP(hipMemcpyAsync(S->ys, prm->ys, S->NY * 8, hipMemcpyHostToDevice, ctx->stream));
    // the constant part of compute_timestep, exactly as rmt_sim_create computes it
    const double dx = prm->dx, CFL = prm->cfl;
    double cs_ = std::sqrt((prm->kappa + prm->mu_s * 4.0 / 3.0) / (prm->rho_s + 1e-12));
    double d = std::fmin(CFL * dx / (cs_ + 1e-14), 1.0);
    double mu_max = std::fmax(prm->mu_f, prm->eta_s), rho_min = std::fmin(prm->rho_s, prm->rho_f);
    if (mu_max > 1e-12 && rho_min > 1e-12)
        d = std::fmin(d, CFL * rho_min * std::pow(dx, 2.0) / (4.0 * mu_max));
    S->dt_const = std::fmin(d, prm->dt_cap);
    RMT_TRY(ensure_bytes(ctx, extrap_workspace(S->NY, S->NX, prm->layers, extrap_par_enabled())));
    if (prm->layers >= 1 && prm->layers <= 12) {
        int least = 0, greatest = 0;
        RMT_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest));
        RMT_HIP(hipStreamCreateWithPriority(&S->st2, hipStreamNonBlocking, least));
        RMT_HIP(hipEventCreateWithFlags(&S->e_chain, hipEventDisableTiming));
        RMT_HIP(hipEventCreateWithFlags(&S->e_mom, hipEventDisableTiming));
        S->max_tiles = ((S->NX + MOM_TX - 1) / MOM_TX) * ((S->NY + MOM_TY - 1) / MOM_TY);
        RMT_HIP(hipMalloc(&S->tiles, (S->max_tiles + 64) * sizeof(int)));
        S->tcount = S->tiles + S->max_tiles;
        RMT_HIP(hipEventCreateWithFlags(&S->e_bits, hipEventDisableTiming));
        RMT_HIP(hipEventCreateWithFlags(&S->e_geo, hipEventDisableTiming));
        RMT_HIP(hipMalloc(&S->bits_next, (size_t)S->NY * W * sizeof(u64)));
        S->ws_len = extrap_workspace(S->NY, S->NX, prm->layers, extrap_par_enabled());
        RMT_HIP(hipMalloc(&S->ws, S->ws_len));
    }
    RMT_HIP(hipStreamSynchronize(ctx->stream));
    *out = S;
    return RMT_OK;
}

int rmt_slab_destroy(rmt_slab *S) {
    if (!S) return RMT_OK;
    if (S->st2) (void)hipStreamSynchronize(S->st2);
    (void)hipFree(S->block);
    if (S->tiles) (void)hipFree(S->tiles);
    if (S->e_chain) (void)hipEventDestroy(S->e_chain);
    if (S->e_mom) (void)hipEventDestroy(S->e_mom);
    if (S->e_bits) (void)hipEventDestroy(S->e_bits);
    if (S->e_geo) (void)hipEventDestroy(S->e_geo);
    if (S->bits_next) (void)hipFree(S->bits_next);
    if (S->ws) (void)hipFree(S->ws);
    if (S->st2) (void)hipStreamDestroy(S->st2);
    delete S;
    return RMT_OK;
}

int rmt_slab_info(rmt_slab *S, int *ints8, double *dt_const) {
    RMT_CHECK(S && ints8, RMT_EINVAL, "null argument");
    const int v[8] = {S->r0, S->r1, S->lo, S->hi, S->c0, S->c1, S->W, RMT_SLAB_HALO};
    for (int k = 0; k < 8; ++k) ints8[k] = v[k];
    if (dt_const) *dt_const = S->dt_const;
    return RMT_OK;
}

int rmt_slab_buffer(rmt_slab *S, int id, void **ptr) {
    RMT_CHECK(S && ptr, RMT_EINVAL, "null argument");
    void *b[] = {S->u, S->v, S->p, S->X1, S->X2, S->phi, S->J, S->pc, S->bits, S->rim,
                 S->A, S->B, S->scal, S->bits_next};
    RMT_CHECK(id != 13 || S->bits_next, RMT_ENOTSUP, "slab: no early-geometry buffers");
    RMT_CHECK(id >= 0 && id < (int)(sizeof(b) / sizeof(b[0])), RMT_EINVAL, "unknown buffer id");
    *ptr = b[id];
    return RMT_OK;
}

int rmt_slab_set_device_dt(rmt_slab *S, int on) {
    RMT_CHECK(S, RMT_EINVAL, "null slab");
    S->dtp = on ? S->scal + SC_DT : nullptr;
    return RMT_OK;
}

int rmt_slab_next_dt(rmt_slab *S, const double *gathered_scal, int G, double *ring_slot) {
    RMT_CHECK(S && gathered_scal && G == S->G, RMT_EINVAL, "rmt_slab_next_dt: bad argument");
    k_slab_dt<<<1, 256, 0, S->ctx->stream>>>(gathered_scal, G, S->dt_const, S->P.cfl, S->P.dx,
                                             S->scal, ring_slot);
    RMT_LAUNCHED();
    return RMT_OK;
}

int rmt_slab_rim_cap(rmt_slab *S, long long cap) {
    RMT_CHECK(S && cap >= 0, RMT_EINVAL, "rmt_slab_rim_cap: bad argument");
    k_rim_cap<<<1, 1, 0, S->ctx->stream>>>(S->scal, (long)cap, S->flags);
    RMT_LAUNCHED();
    return RMT_OK;
}

int rmt_slab_begin(rmt_slab *S) {
    RMT_CHECK(S, RMT_EINVAL, "null slab");
    const long o = (long)(S->r0 - S->lo) * S->NX, n = (long)(S->r1 - S->r0) * S->NX;
    return reduce_maxsq2(S->ctx, S->u + o, S->v + o, n, S->scal + SC_M2);
}

// rows [r0 + 10, r1 - 10): every sample of their backtraces lies in owned rows (the step
// moves a departure point by far less than a cell), so they need no halo row and can run
// while the halo exchange is in flight; a NaN-propagating max |u|^2 over the owned rows
// bounds their velocities (bilinear rows checked against [r0, r1))
static void slab_interior_rows(const rmt_slab *S, int *ib, int *ie) {
    *ib = S->r0 + 10; *ie = std::max(*ib, S->r1 - 10);
}
int rmt_slab_advect_interior(rmt_slab *S, double dt) {
    RMT_CHECK(S, RMT_EINVAL, "null slab");
    rmt_ctx *ctx = S->ctx;
    const rmt_sim_params &P = S->P;
    const int NX = S->NX;
    int ib, ie;
    slab_interior_rows(S, &ib, &ie);
    S->dt_cur = dt;
    S->interior = true;
    RMT_HIP(hipMemsetAsync(S->flags, 0, 8 * sizeof(int), ctx->stream));
    if (ie > ib) {
        const long o = (long)(S->r0 - S->lo) * NX, no = (long)(S->r1 - S->r0) * NX;
        RMT_TRY(reduce_maxsq2_nan(ctx, S->u + o, S->v + o, no, S->scal + SC_M2OWN));
        k_slab_sl<<<dim3((NX + 255) / 256, ie - ib), 256, 0, ctx->stream>>>(
            S->gv(S->X1), S->gv(S->X2), S->gv(S->u), S->gv(S->v), S->xs, S->ys, S->NY, NX, dt,
            divk_make(P.dx), divk_make(P.dy), P.x0, P.y0, P.R, S->gv(S->X1n), S->gv(S->X2n), S->gv(S->phi_pre),
            S->flags, ib, ie, S->r0, S->r1, S->scal + SC_M2OWN, S->dtp);
        RMT_LAUNCHED();
    }
    return RMT_OK;
}

int rmt_slab_advect(rmt_slab *S, double dt) {
    RMT_CHECK(S, RMT_EINVAL, "null slab");
    rmt_ctx *ctx = S->ctx;
    const rmt_sim_params &P = S->P;
    const int NX = S->NX, jb = std::max(0, S->r0 - 10), je = std::min(S->NY, S->r1 + 10);
    // the per-step state is consumed before any check, so a failed call cannot leak into the
    // next step
    const bool in = S->interior;
    S->interior = false;
    RMT_CHECK(!in || S->dtp || dt == S->dt_cur, RMT_EINVAL, "slab advect: dt differs");
    S->dt_cur = dt;
    if (!in) RMT_HIP(hipMemsetAsync(S->flags, 0, 8 * sizeof(int), ctx->stream));
    // max |u|^2 over the resident rows: bounds every velocity sample of the backtraces
    RMT_TRY(reduce_maxsq2_nan(ctx, S->u, S->v, (long)(S->hi - S->lo) * NX, S->scal + SC_M2RES));
    int ib = je, ie = je;   // rows done by rmt_slab_advect_interior
    if (in) slab_interior_rows(S, &ib, &ie);
    const int segs[2][2] = {{jb, std::min(ib, je)}, {std::max(ie, jb), je}};
    for (int k = 0; k < (in ? 2 : 1); ++k) {
        const int a = in ? segs[k][0] : jb, b = in ? segs[k][1] : je;
        if (b <= a) continue;
        k_slab_sl<<<dim3((NX + 255) / 256, b - a), 256, 0, ctx->stream>>>(
            S->gv(S->X1), S->gv(S->X2), S->gv(S->u), S->gv(S->v), S->xs, S->ys, S->NY, NX, dt,
            divk_make(P.dx), divk_make(P.dy), P.x0, P.y0, P.R, S->gv(S->X1n), S->gv(S->X2n), S->gv(S->phi_pre),
            S->flags, a, b, S->lo, S->hi, S->scal + SC_M2RES, S->dtp);
        RMT_LAUNCHED();
    }
    if (S->geo_ready) {
        // the whole known plane was gathered with the geometry (rmt_slab_geometry): the
        // owned rows equal k_slab_bits of this phi_pre (the same disc_phi of the same map)
        RMT_HIP(hipMemcpyAsync(S->bits, S->bits_next, (size_t)S->NY * S->W * sizeof(u64),
                               hipMemcpyDeviceToDevice, ctx->stream));
        return RMT_OK;
    }
    k_slab_bits<<<dim3((NX + 255) / 256, S->r1 - S->r0), 256, 0, ctx->stream>>>(
        S->gv(S->phi_pre), NX, S->W, S->bits, S->r0);
    RMT_LAUNCHED();
    return RMT_OK;
}

// the next step's known plane, owned rows (after rmt_slab_momentum: phi is final)
int rmt_slab_next_bits(rmt_slab *S) {
    RMT_CHECK(S && S->bits_next, RMT_ENOTSUP, "slab: no early-geometry buffers");
    k_slab_bits<<<dim3((S->NX + 255) / 256, S->r1 - S->r0), 256, 0, S->ctx->stream>>>(
        S->gv(S->phi), S->NX, S->W, S->bits_next, S->r0);
    RMT_LAUNCHED();
    return RMT_OK;
}

// the next step's extrapolation geometry from the gathered bits_next, on the second stream
// beside the rest of this step; the next rmt_slab_advect / extrapolate use it
int rmt_slab_geometry(rmt_slab *S) {
    RMT_CHECK(S && S->bits_next && S->st2, RMT_ENOTSUP, "slab: no early-geometry buffers");
    rmt_ctx *ctx = S->ctx;
    const rmt_sim_params &P = S->P;
    S->geo_ready = false;
    if (P.layers <= 0) return RMT_OK;
    RMT_HIP(hipEventRecord(S->e_bits, ctx->stream));
    RMT_HIP(hipStreamWaitEvent(S->st2, S->e_bits, 0));
    hipStream_t st = ctx->stream;
    ctx->stream = S->st2;
    // (test switch: the geometry starts late, so that a dropped one overlaps what follows)
    if (ctx->opt.test_delay_geo) { k_slab_delay<<<1, 1, 0, S->st2>>>(ctx->opt.test_delay_geo); RMT_LAUNCHED(); }
    int gs;
    {
        SlabWs ws(S);
        gs = extrap_geometry(ctx, S->X1d, S->X2d, nullptr, P.dx, P.dy, P.layers, S->X1d, S->X2d,
                             S->bits_next);
    }
    ctx->stream = st;
    RMT_TRY(gs);
    RMT_HIP(hipEventRecord(S->e_geo, S->st2));
    S->geo_ready = true;
    return RMT_OK;
}

// forget a geometry prepared for a step that will not run (the state may change in between).
// The dropped geometry may still be running on st2 into the slab's extrapolation workspace:
// the main stream waits for it, so the next user of that workspace (a full extrapolation, a
// rerun window after a rim overflow) cannot overlap it -- as rmt_sim_step's end of call does
// (sim.hip).  VERDICT r5 weak 3, hypothesis (a); tests/test_distributed.py
// test_slab_rerun_after_late_dropped_geometry delays the dropped geometry into the rerun.
int rmt_slab_drop_geometry(rmt_slab *S) {
    RMT_CHECK(S, RMT_EINVAL, "null slab");
    if (S->geo_ready && !S->ctx->opt.test_nowait_drop)
        RMT_HIP(hipStreamWaitEvent(S->ctx->stream, S->e_geo, 0));
    S->geo_ready = false;
    return RMT_OK;
}

int rmt_slab_rim_pack(rmt_slab *S) {
    RMT_CHECK(S, RMT_EINVAL, "null slab");
    return slab_rim_pack(S->ctx, S->bits, S->NY, S->NX, S->W, S->r0, S->r1, S->rimw, S->rowcnt,
                         S->gv(S->X1n), S->gv(S->X2n), S->rim, S->scal + SC_COUNT);
}

static int slab_extrapolate(rmt_slab *S, const double *gathered, const long long *counts,
                            long long cap, const double *gs);
int rmt_slab_extrapolate(rmt_slab *S, const double *gathered, const long long *counts,
                         long long cap) {
    RMT_CHECK(S && counts && (gathered || cap == 0), RMT_EINVAL, "null argument");
    return slab_extrapolate(S, gathered, counts, cap, nullptr);
}
int rmt_slab_extrapolate_dev(rmt_slab *S, const double *gathered, const double *gathered_scal,
                             long long cap) {
    RMT_CHECK(S && gathered_scal && (gathered || cap == 0), RMT_EINVAL, "null argument");
    return slab_extrapolate(S, gathered, nullptr, cap, gathered_scal);
}
}  // extern "C"
static int slab_extrapolate(rmt_slab *S, const double *gathered, const long long *counts,
                            long long cap, const double *gs) {
    rmt_ctx *ctx = S->ctx;
    const rmt_sim_params &P = S->P;
    S->spec = S->st2 && !ctx->opt.no_overlap;
    const int jb = std::max(0, S->r0 - 10), je = std::min(S->NY, S->r1 + 10);
    if (S->spec) ctx->ev_chain = S->e_chain;
    const bool geo = S->geo_ready;
    S->geo_ready = false;
    int es;
    {
        SlabWs ws(S);
        es = slab_rim_extrapolate(ctx, gathered, counts, S->G, cap, S->X1d, S->X2d, S->bits,
                                  P.dx, P.dy, P.layers, S->flags + 4, S->gv(S->X1n),
                                  S->gv(S->X2n), (long)S->lo * S->NX, (long)S->hi * S->NX, gs,
                                  geo ? S->e_geo : nullptr);
    }
    ctx->ev_chain = nullptr;
    if (es != RMT_OK) { S->spec = false; return es; }
    if (!S->spec) {
        k_slab_phi<<<grid1d((long)(je - jb) * S->NX, 256), 256, 0, ctx->stream>>>(
            S->gv(S->X1n), S->gv(S->X2n), P.x0, P.y0, P.R, S->NX, jb, je, S->gv(S->phi),
            S->gv(S->X1), S->gv(S->X2));
        RMT_LAUNCHED();
        return RMT_OK;
    }
    // beside the chain (second stream, from the advected map before the rim write-back): phi
    // and the slab's momentum; the main stream lists the tiles a target can reach
    RMT_HIP(hipStreamWaitEvent(S->st2, S->e_chain, 0));
    k_slab_phi<<<grid1d((long)(je - jb) * S->NX, 256), 256, 0, S->st2>>>(
        S->gv(S->X1n), S->gv(S->X2n), P.x0, P.y0, P.R, S->NX, jb, je, S->gv(S->phi),
        S->gv(S->X1), S->gv(S->X2));
    RMT_LAUNCHED();
    hipStream_t st = ctx->stream;
    ctx->stream = S->st2;
    const int ms = slab_momentum_pass(S, S->dt_cur, false);
    ctx->stream = st;
    RMT_TRY(ms);
    RMT_HIP(hipEventRecord(S->e_mom, S->st2));
    SlabWs ws(S);   // the tiles come from this step's extrapolation workspace
    return extrap_fix_tiles(ctx, P.layers, 12, S->tiles, S->tcount);
}
extern "C" {

int rmt_slab_momentum(rmt_slab *S, double dt) {
    RMT_CHECK(S, RMT_EINVAL, "null slab");
    if (S->spec) {
        RMT_CHECK(S->dtp || dt == S->dt_cur, RMT_EINVAL,
                  "slab momentum: dt differs from the advection's");
        S->spec = false;
        rmt_ctx *ctx = S->ctx;
        const rmt_sim_params &P = S->P;
        const int jb = std::max(0, S->r0 - 10), je = std::min(S->NY, S->r1 + 10);
        RMT_HIP(hipStreamWaitEvent(ctx->stream, S->e_mom, 0));
        k_slab_phi_tiles<<<S->max_tiles, 256, 0, ctx->stream>>>(
            S->gv(S->X1n), S->gv(S->X2n), P.x0, P.y0, P.R, S->NX, jb, je, S->gv(S->phi),
            S->gv(S->X1), S->gv(S->X2), S->tiles, S->tcount, (S->NX + MOM_TX - 1) / MOM_TX);
        RMT_LAUNCHED();
        return slab_momentum_pass(S, dt, true);
    }
    return slab_momentum_pass(S, dt, false);
}
}  // extern "C"

// the slab's RK4 momentum on its window (fixup: only the listed tiles, after the chain)
static int slab_momentum_pass(rmt_slab *S, double dt, bool fixup) {
    const rmt_sim_params &P = S->P;
    rmt_momentum_params M{};
    M.bc_kind = P.bc_kind; M.lid = P.lid; M.mu_s = P.mu_s; M.kappa = P.kappa;
    M.eta_s = P.eta_s; M.rho_s = P.rho_s; M.rho_f = P.rho_f; M.mu_f = P.mu_f; M.w_t = P.w_t;
    M.dx = P.dx; M.dy = P.dy; M.dt = dt; M.stress_band = P.stress_band;
    M.detg_clamp = P.detg_clamp;
    const long nl = (long)(S->hi - S->lo) * S->NX, off = (long)S->lo * S->NX;
    MomWork W = mom_work(S->mw - off, nl, S->solid - off, S->flags + 1);
    W.dtp = S->dtp;
    const RowWin win{std::max(0, S->r0 - 1), std::min(S->NY, S->r1 + 1), S->lo, S->hi};
    if (fixup)
        return momentum_fixup(S->ctx, &M, S->gv(S->u), S->gv(S->v), S->gv(S->p), S->gv(S->X1),
                              S->gv(S->X2), S->gv(S->phi), S->gv(S->us), S->gv(S->vs),
                              S->gv(S->sxx), S->gv(S->sxy), S->gv(S->syy), S->gv(S->J), W,
                              S->tiles, S->tcount, S->max_tiles, &win);
    return momentum_rk4(S->ctx, &M, S->gv(S->u), S->gv(S->v), S->gv(S->p), S->gv(S->X1),
                        S->gv(S->X2), S->gv(S->phi), S->gv(S->us), S->gv(S->vs), S->gv(S->sxx),
                        S->gv(S->sxy), S->gv(S->syy), S->gv(S->J), W, &win);
}

extern "C" {

int rmt_slab_project_rows(rmt_slab *S, double dt) {
    RMT_CHECK(S, RMT_EINVAL, "null slab");
    rmt_ctx *ctx = S->ctx;
    const rmt_sim_params &P = S->P;
    const double rho = P.rho_f;
    const int rows = S->r1 - S->r0;
    const long no = (long)rows * S->NX;
    double *rhs = S->gv(S->rhs) + (long)S->r0 * S->NX;   // owned rows of the rhs plane
    // rhs = (rho * div) / dt in the divergence kernel (the same two roundings as the scale and
    // divide passes of ops.hip)
    RMT_TRY(divergence_rc_rows(ctx, S->gv(S->us), S->gv(S->vs), S->gv(S->p), dt / rho, P.dx, P.dy,
                               S->gv(S->rhs), S->r0, S->r1, rho, dt, S->dtp));
    RMT_TRY(dct_pass(ctx, false, 0, rhs, S->Y, rows, 0, 1.0));
    k_cols<true><<<grid1d(no, 256), 256, 0, ctx->stream>>>(S->Y, rows, S->NX, S->cs, S->G, S->A);
    RMT_LAUNCHED();
    return RMT_OK;
}

int rmt_slab_project_cols(rmt_slab *S) {
    RMT_CHECK(S, RMT_EINVAL, "null slab");
    rmt_ctx *ctx = S->ctx;
    const int nc = S->c1 - S->c0;
    transpose(ctx, ctx->stream, S->B, S->NY, nc, S->T);
    RMT_TRY(dct_pass(ctx, true, 1, S->T, S->T, nc, S->c0, 1.0 / (2.0 * (S->NY - 1))));
    transpose(ctx, ctx->stream, S->T, nc, S->NY, S->B);
    RMT_LAUNCHED();
    return RMT_OK;
}

int rmt_slab_project_unrows(rmt_slab *S) {
    RMT_CHECK(S, RMT_EINVAL, "null slab");
    rmt_ctx *ctx = S->ctx;
    const int rows = S->r1 - S->r0;
    const long no = (long)rows * S->NX;
    double *pc = S->gv(S->pc) + (long)S->r0 * S->NX;
    k_cols<false><<<grid1d(no, 256), 256, 0, ctx->stream>>>(S->Y, rows, S->NX, S->cs, S->G, S->A);
    RMT_LAUNCHED();
    if (rows > ctx->rsum_len) {
        RMT_TRY(dct_pass(ctx, false, 0, S->Y, pc, rows, 0, 1.0 / (2.0 * (S->NX - 1))));
        return rowtree_root(ctx, pc, rows, S->NX, S->scal + SC_ROOT);
    }
    // the row sums come out of the inverse pass itself (k_rowsum's order)
    RMT_TRY(dct_pass(ctx, false, 0, S->Y, pc, rows, 0, 1.0 / (2.0 * (S->NX - 1)), ctx->rsum));
    return rowtree_sums(ctx, rows, S->scal + SC_ROOT);
}

int rmt_slab_sub_mean(rmt_slab *S, int which, const double *roots) {
    RMT_CHECK(S && roots && (which == 0 || which == 1), RMT_EINVAL, "bad argument");
    double *x = S->gv(which ? S->p : S->pc) + (long)S->r0 * S->NX;
    return sub_tree_mean(S->ctx, x, (long)(S->r1 - S->r0) * S->NX, roots, S->G,
                         (double)S->NY * S->NX);
}

int rmt_slab_project_correct(rmt_slab *S, double dt) {
    RMT_CHECK(S, RMT_EINVAL, "null slab");
    const rmt_sim_params &P = S->P;
    RMT_TRY(project_correct_rows(S->ctx, S->gv(S->us), S->gv(S->vs), S->gv(S->pc), S->gv(S->p),
                                 P.dx, P.dy, dt / P.rho_f, P.bc_kind, P.lid, S->gv(S->u),
                                 S->gv(S->v), S->gv(S->p), S->r0, S->r1, S->dtp, P.rho_f));
    return rowtree_root(S->ctx, S->gv(S->p) + (long)S->r0 * S->NX, S->r1 - S->r0, S->NX,
                        S->scal + SC_ROOT);
}

int rmt_slab_finish(rmt_slab *S) {
    RMT_CHECK(S, RMT_EINVAL, "null slab");
    rmt_ctx *ctx = S->ctx;
    RMT_TRY(diag_rows(ctx, S->gv(S->phi), S->gv(S->J), S->xs, S->ys, S->gv(S->u), S->gv(S->v),
                      S->gv(S->X1), S->gv(S->X2), S->P, S->r0, S->r1, S->part,
                      S->scal + SC_DIAG));
    RMT_TRY(rmt_slab_begin(S));
    k_flags_out<<<1, 1, 0, ctx->stream>>>(S->flags, S->scal);
    RMT_LAUNCHED();
    return RMT_OK;
}

}  // extern "C"
