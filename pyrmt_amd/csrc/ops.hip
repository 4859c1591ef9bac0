// ops.hip -- context, reductions and the per-operator kernels of librmt.
// Each kernel restates one reference operator per cell (cited); launch shapes are
// 1D over cells with 256-thread workgroups (memory-bound elementwise / small-stencil
// work: reads coalesce along i, neighbours come from L2).
#include "rmt_internal.hpp"
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <vector>

namespace rmt {
static thread_local std::string g_err;
void set_error(const std::string &m) { g_err = m; }
// rmt_opts by name: (option name, environment variable, field)
static const struct { const char *name, *env; int rmt_opts::*f; } kOpts[] = {
    {"ext_events", "RMT_EXT_EVENTS", &rmt_opts::ext_events},
    {"ex_arena_bump", nullptr, &rmt_opts::ex_arena_bump},   // RMT_EX_ARENA=bump (below)
    {"ex_profile", "RMT_EX_PROFILE", &rmt_opts::ex_profile},
    {"fix_all", "RMT_FIX_ALL", &rmt_opts::fix_all},
    {"dct_rocfft", "RMT_DCT_ROCFFT", &rmt_opts::dct_rocfft},
    {"transpose2", "RMT_TRANSPOSE2", &rmt_opts::transpose2},
    {"sim_hiprio", "RMT_SIM_HIPRIO", &rmt_opts::sim_hiprio},
    {"sim_sync", "RMT_SIM_SYNC", &rmt_opts::sim_sync},
    {"early_geometry", "RMT_EARLY_GEOMETRY", &rmt_opts::early_geometry},
    {"early_transpose", "RMT_EARLY_TRANSPOSE", &rmt_opts::early_transpose},
    {"fused_fluid", "RMT_FUSED_FLUID", &rmt_opts::fused_fluid},
    {"no_overlap", "RMT_NO_OVERLAP", &rmt_opts::no_overlap},
    {"side_tail", "RMT_SIDE_TAIL", &rmt_opts::side_tail},
    {"par_overlap", "RMT_PAR_OVERLAP", &rmt_opts::par_overlap},
    {"fused_fixprep", "RMT_FUSED_FIXPREP", &rmt_opts::fused_fixprep},
    {"merged_join", "RMT_MERGED_JOIN", &rmt_opts::merged_join},
    {"test_delay_side", "RMT_TEST_DELAY_SIDE", &rmt_opts::test_delay_side},
    {"test_delay_main", "RMT_TEST_DELAY_MAIN", &rmt_opts::test_delay_main},
    {"test_delay_geo", "RMT_TEST_DELAY_GEO", &rmt_opts::test_delay_geo},
    {"test_nowait_drop", "RMT_TEST_NOWAIT_DROP", &rmt_opts::test_nowait_drop},
    {"chain_cols", "RMT_CH_PARTS", &rmt_opts::ch_cols},
    {"chain_layer_groups", "RMT_CH_LAYERS", &rmt_opts::ch_lgroups},
    {"edge_slots", "RMT_EDGE_SLOTS_USED", &rmt_opts::edge_slots},
    {"edge_stream", "RMT_EDGE_STREAM", &rmt_opts::edge_stream},
    {"sl_phi", "RMT_SL_PHI", &rmt_opts::sl_phi},
    {"mac_boxes", "RMT_MAC_BOXES", &rmt_opts::mac_boxes},
    {"skip_marked_rows", "RMT_SKIP_MARKED_ROWS", &rmt_opts::skip_marked_rows},
    {"tail_stream", "RMT_TAIL_STREAM", &rmt_opts::tail_stream},
    {"diag_first", "RMT_DIAG_FIRST", &rmt_opts::diag_first},
    {"mac_noop_host", "RMT_MAC_NOOP_HOST", &rmt_opts::mac_noop_host},
    {"mac_face_sl", "RMT_MAC_FACE_SL", &rmt_opts::mac_face_sl},
    {"mac_m2_bound", "RMT_MAC_M2_BOUND", &rmt_opts::mac_m2_bound},
    {"diag_seg", "RMT_DIAG_SEG", &rmt_opts::diag_seg},
    {"sl_zero_flags", "RMT_SL_ZERO_FLAGS", &rmt_opts::sl_zero_flags},
    {"dct_desc", "RMT_DCT_DESC", &rmt_opts::dct_desc},
};
int g_list_blocks = getenv("RMT_LIST_BLOCKS") ? std::max(1, atoi(getenv("RMT_LIST_BLOCKS")))
                                                : LIST_BLOCKS;
static rmt_opts opts_from_env() {
    rmt_opts o;
    for (const auto &k : kOpts)
        if (k.env)
            if (const char *e = getenv(k.env)) o.*(k.f) = atoi(e);
    if (const char *e = getenv("RMT_EX_ARENA")) o.ex_arena_bump = !strcmp(e, "bump");
    o.test_delay_side = std::max(0, o.test_delay_side);
    o.test_delay_main = std::max(0, o.test_delay_main);
    o.test_delay_geo = std::max(0, o.test_delay_geo);
    return o;
}

// Growing a context buffer frees the old one, which kernels queued on any of the context's
// streams may still read: the device is drained first (hipFree's implicit synchronisation,
// made explicit), and the new buffer's contents are written by stream-ordered kernels only.
int ensure_scratch(rmt_ctx *ctx, size_t bytes) {
    if (ctx->scratch_bytes >= bytes) return RMT_OK;
    RMT_HIP(hipDeviceSynchronize());
    if (ctx->scratch) RMT_HIP(hipFree(ctx->scratch));
    ctx->scratch = nullptr; ctx->scratch_bytes = 0;
    RMT_HIP(hipMalloc(&ctx->scratch, bytes));
    ctx->scratch_bytes = bytes;
    return RMT_OK;
}
int ensure_bytes(rmt_ctx *ctx, size_t bytes) {
    ++ctx->bytes_gen;   // (rmt_sim's carried geometry lives there: any other user ends it)
    if (ctx->bytes_len >= bytes) return RMT_OK;
    RMT_HIP(hipDeviceSynchronize());
    if (ctx->bytes) RMT_HIP(hipFree(ctx->bytes));
    ctx->bytes = nullptr; ctx->bytes_len = 0;
    RMT_HIP(hipMalloc(&ctx->bytes, bytes));
    ctx->bytes_len = bytes;
    return RMT_OK;
}

// ------------------------------------------------------------------ reductions ----
// Deterministic two-pass reductions: RED_BLOCKS fixed workgroups each fold a strided
// slice in a fixed order, then one workgroup folds the partials in a fixed tree.

template <int OP>  // 0 sum, 1 max, 2 max(a*a+b*b)
__global__ void __launch_bounds__(RED_T) k_reduce_p1(const double *__restrict__ a,
                                                     const double *__restrict__ b, long n,
                                                     double *__restrict__ part) {
    __shared__ double s[RED_T];
    double acc = OP == 0 ? 0.0 : -INFINITY;
    for (long k = blockIdx.x * (long)RED_T + threadIdx.x; k < n; k += (long)RED_BLOCKS * RED_T) {
        double x = OP >= 2 ? a[k] * a[k] + b[k] * b[k] : a[k];
        if (OP == 0) acc += x;
        else if (OP == 3) acc = (x > acc || x != x) ? x : acc;   // NaN propagates
        else acc = fmax(acc, x);   // NaN inputs are not on the path (guarded upstream)
    }
    s[threadIdx.x] = acc;
    __syncthreads();
    for (int w = RED_T / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w)
            s[threadIdx.x] = OP == 0 ? s[threadIdx.x] + s[threadIdx.x + w]
                             : OP == 3 ? ((s[threadIdx.x + w] > s[threadIdx.x] ||
                                           s[threadIdx.x + w] != s[threadIdx.x + w])
                                              ? s[threadIdx.x + w] : s[threadIdx.x])
                                       : fmax(s[threadIdx.x], s[threadIdx.x + w]);
        __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = s[0];
}

template <int OP>
__global__ void __launch_bounds__(RED_T) k_reduce_p2(const double *__restrict__ part, double *out,
                                                     double scale) {
    __shared__ double s[RED_T];
    double acc = OP == 0 ? 0.0 : -INFINITY;
    for (int k = threadIdx.x; k < RED_BLOCKS; k += RED_T) {
        const double y = part[k];
        acc = OP == 0 ? acc + y : OP == 3 ? ((y > acc || y != y) ? y : acc) : fmax(acc, y);
    }
    s[threadIdx.x] = acc;
    __syncthreads();
    for (int w = RED_T / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w) {
            const double y = s[threadIdx.x + w];
            s[threadIdx.x] = OP == 0 ? s[threadIdx.x] + y
                             : OP == 3 ? ((y > s[threadIdx.x] || y != y) ? y : s[threadIdx.x])
                                       : fmax(s[threadIdx.x], y);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) *out = OP == 0 ? s[0] * scale : s[0];
}

static int reduce_impl(rmt_ctx *ctx, int op, const double *a, const double *b, long n,
                       double *out, double scale) {
    if (op == 0) {
        k_reduce_p1<0><<<RED_BLOCKS, RED_T, 0, ctx->stream>>>(a, b, n, ctx->red);
        k_reduce_p2<0><<<1, RED_T, 0, ctx->stream>>>(ctx->red, out, scale);
    } else if (op == 1) {
        k_reduce_p1<1><<<RED_BLOCKS, RED_T, 0, ctx->stream>>>(a, b, n, ctx->red);
        k_reduce_p2<1><<<1, RED_T, 0, ctx->stream>>>(ctx->red, out, scale);
    } else if (op == 2) {
        k_reduce_p1<2><<<RED_BLOCKS, RED_T, 0, ctx->stream>>>(a, b, n, ctx->red);
        k_reduce_p2<1><<<1, RED_T, 0, ctx->stream>>>(ctx->red, out, scale);
    } else {
        k_reduce_p1<3><<<RED_BLOCKS, RED_T, 0, ctx->stream>>>(a, b, n, ctx->red);
        k_reduce_p2<3><<<1, RED_T, 0, ctx->stream>>>(ctx->red, out, scale);
    }
    RMT_LAUNCHED();
    return RMT_OK;
}
int reduce_sum(rmt_ctx *ctx, const double *x, long n, double *o) { return reduce_impl(ctx, 0, x, x, n, o, 1.0); }
int reduce_max(rmt_ctx *ctx, const double *x, long n, double *o) { return reduce_impl(ctx, 1, x, x, n, o, 1.0); }
int reduce_maxsq2(rmt_ctx *ctx, const double *a, const double *b, long n, double *o) {
    return reduce_impl(ctx, 2, a, b, n, o, 1.0);
}
int reduce_maxsq2_nan(rmt_ctx *ctx, const double *a, const double *b, long n, double *o) {
    return reduce_impl(ctx, 3, a, b, n, o, 1.0);
}
// the second pass of reduce_maxsq2_nan over RED_BLOCKS partials a fused kernel left in ctx->red
int reduce_max_partials_nan(rmt_ctx *ctx, double *o) {
    k_reduce_p2<3><<<1, RED_T, 0, ctx->stream>>>(ctx->red, o, 1.0);
    RMT_LAUNCHED();
    return RMT_OK;
}
int reduce_mean(rmt_ctx *ctx, const double *x, long n, double *o) {
    return reduce_impl(ctx, 0, x, x, n, o, 1.0 / (double)n);
}
// Row-tree sums (means of the projection): a fixed-order sum per row, then an aligned
// pairwise tree over the rows (level l node k covers rows [k 2^l, (k+1) 2^l)).  A slab of 2^m
// rows starting at a multiple of 2^m is one node of that tree, so the slab-decomposed step
// (slab.hip) combines its per-slab roots with the same tree and gets the same bits.
__global__ void __launch_bounds__(256) k_rowsum(const double *__restrict__ x, int nx,
                                                double *__restrict__ rs) {
    __shared__ double s[256];
    const double *r = x + (long)blockIdx.x * nx;
    double acc = 0.0;
    for (int i = threadIdx.x; i < nx; i += 256) acc += r[i];
    s[threadIdx.x] = acc;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w) s[threadIdx.x] = s[threadIdx.x] + s[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) rs[blockIdx.x] = s[0];
}
// k_rowsum of x = p + (pc - m) (m = *root / count, k_project_correct's mean of the raw solve),
// x written back to p: the deferred half of the projection's pressure update, fused into the
// mean removal's row pass (same expression and the same per-row summation order)
__global__ void __launch_bounds__(256) k_rowsum_upd(double *__restrict__ p,
                                                    const double *__restrict__ pc,
                                                    const double *__restrict__ root, double count,
                                                    int nx, double *__restrict__ rs) {
    __shared__ double s[256];
    const double m = *root / count;
    double *r = p + (long)blockIdx.x * nx;
    const double *q = pc + (long)blockIdx.x * nx;
    double acc = 0.0;
    for (int i = threadIdx.x; i < nx; i += 256) {
        const double v = r[i] + (q[i] - m);
        r[i] = v;
        acc += v;
    }
    s[threadIdx.x] = acc;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w) s[threadIdx.x] = s[threadIdx.x] + s[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) rs[blockIdx.x] = s[0];
}
constexpr int TREE_MAX = 8192, TREE_T = 1024;
__global__ void __launch_bounds__(TREE_T) k_rowtree(const double *__restrict__ rs, int m,
                                                    double *__restrict__ out) {
    __shared__ double s[TREE_MAX];
    for (int k = threadIdx.x; k < m; k += TREE_T) s[k] = rs[k];
    __syncthreads();
    while (m > 1) {
        const int h = (m + 1) / 2;
        double v[TREE_MAX / 2 / TREE_T];
#pragma unroll
        for (int q = 0; q < TREE_MAX / 2 / TREE_T; ++q) {
            const int k = threadIdx.x + q * TREE_T;
            if (k < h) v[q] = 2 * k + 1 < m ? s[2 * k] + s[2 * k + 1] : s[2 * k];
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < TREE_MAX / 2 / TREE_T; ++q) {
            const int k = threadIdx.x + q * TREE_T;
            if (k < h) s[k] = v[q];
        }
        __syncthreads();
        m = h;
    }
    if (threadIdx.x == 0) *out = s[0];
}
// x -= tree(roots) / count over n cells (numpy mean: sum / count); the same aligned tree
// over the G <= 64 slab roots, folded once per block in LDS
constexpr int STM_BLOCKS = 2048;
__global__ void __launch_bounds__(256) k_sub_tree_mean(double *__restrict__ x, long n,
                                                       const double *__restrict__ roots, int G,
                                                       double count) {
    __shared__ double s[64];
    __shared__ double mean;
    if (threadIdx.x < 64) s[threadIdx.x] = threadIdx.x < G ? roots[threadIdx.x] : 0.0;
    __syncthreads();
    if (threadIdx.x == 0) {
        int m = G;
        while (m > 1) {
            const int h = (m + 1) / 2;
            for (int k = 0; k < h; ++k) s[k] = 2 * k + 1 < m ? s[2 * k] + s[2 * k + 1] : s[2 * k];
            m = h;
        }
        mean = s[0] / count;
    }
    __syncthreads();
    const double m = mean;
    for (long k = blockIdx.x * 256L + threadIdx.x; k < n; k += (long)gridDim.x * 256)
        x[k] = x[k] - m;
}
int rowtree_root(rmt_ctx *ctx, const double *x, int nrows, int nx, double *dev_root) {
    RMT_CHECK(nrows >= 1 && nrows <= TREE_MAX && nrows <= ctx->rsum_len, RMT_EINVAL,
              "rowtree_root: rows out of range");
    k_rowsum<<<nrows, 256, 0, ctx->stream>>>(x, nx, ctx->rsum);
    k_rowtree<<<1, TREE_T, 0, ctx->stream>>>(ctx->rsum, nrows, dev_root);
    RMT_LAUNCHED();
    return RMT_OK;
}
int rowtree_sums(rmt_ctx *ctx, int nrows, double *dev_root) {
    RMT_CHECK(nrows >= 1 && nrows <= TREE_MAX && nrows <= ctx->rsum_len, RMT_EINVAL,
              "rowtree_sums: rows out of range");
    k_rowtree<<<1, TREE_T, 0, ctx->stream>>>(ctx->rsum, nrows, dev_root);
    RMT_LAUNCHED();
    return RMT_OK;
}
int sub_tree_mean(rmt_ctx *ctx, double *x, long n, const double *dev_roots, int G, double count) {
    RMT_CHECK(G >= 1 && G <= 64, RMT_EINVAL, "sub_tree_mean: 1..64 roots");
    if (n > 0)
        k_sub_tree_mean<<<std::min<long>(grid1d(n, 256), STM_BLOCKS), 256, 0, ctx->stream>>>(
            x, n, dev_roots, G, count);
    RMT_LAUNCHED();
    return RMT_OK;
}
// p = p + (pc - pc_root / (ny nx)), then p -= mean(p) (projection_finish's deferred update)
int sub_mean_rows_upd(rmt_ctx *ctx, double *p, const double *pc, const double *pc_root, int ny,
                      int nx) {
    RMT_CHECK(ny >= 1 && ny <= TREE_MAX && ny <= ctx->rsum_len, RMT_EINVAL,
              "sub_mean_rows_upd: rows out of range");
    double *root = ctx->red + RED_BLOCKS + 16;
    k_rowsum_upd<<<ny, 256, 0, ctx->stream>>>(p, pc, pc_root, (double)ny * nx, nx, ctx->rsum);
    k_rowtree<<<1, TREE_T, 0, ctx->stream>>>(ctx->rsum, ny, root);
    RMT_LAUNCHED();
    return sub_tree_mean(ctx, p, (long)ny * nx, root, 1, (double)ny * nx);
}
int sub_mean_rows(rmt_ctx *ctx, double *x, int ny, int nx) {
    double *root = ctx->red + RED_BLOCKS + 16;
    RMT_TRY(rowtree_root(ctx, x, ny, nx, root));
    return sub_tree_mean(ctx, x, (long)ny * nx, root, 1, (double)ny * nx);
}
int read_scalar(rmt_ctx *ctx, const double *dev, double *host) {
    RMT_HIP(hipMemcpyAsync(host, dev, sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
    RMT_HIP(hipStreamSynchronize(ctx->stream));
    return RMT_OK;
}

// ------------------------------------------------------------------ FD helpers ----
__global__ void k_grad_x(const double *__restrict__ f, int ny, int nx, double h2,
                         double *__restrict__ out) {
    long c = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (c >= (long)ny * nx) return;
    int i = (int)(c % nx);
    out[c] = grad2(f + c, 1, i, nx, h2);
}
__global__ void k_grad_y(const double *__restrict__ f, int ny, int nx, double h2,
                         double *__restrict__ out) {
    long c = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (c >= (long)ny * nx) return;
    int j = (int)(c / nx);
    out[c] = grad2(f + c, nx, j, ny, h2);
}
__global__ void k_upwind(const double *__restrict__ f, const double *__restrict__ vel, int ny,
                         int nx, double h, int axis, double *__restrict__ out) {
    long c = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (c >= (long)ny * nx) return;
    int j = (int)(c / nx), i = (int)(c % nx);
    out[c] = axis == 1 ? upwind3(f + c, 1, i, nx, vel[c], h) : upwind3(f + c, nx, j, ny, vel[c], h);
}

// ---------------------------------------------------------- interpolation / SL ----
__global__ void k_bilinear(const double *__restrict__ u, const double *__restrict__ xq,
                           const double *__restrict__ yq, long nq, double dx, double dy, int nx,
                           int ny, double *__restrict__ out) {
    long k = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (k < nq) out[k] = bilinear(u, xq[k], yq[k], dx, dy, nx, ny);
}
__global__ void k_sl_rk4(const double *__restrict__ q, const double *__restrict__ a,
                         const double *__restrict__ b, const double *__restrict__ X,
                         const double *__restrict__ Y, int ny, int nx, double dt, double dx,
                         double dy, double *__restrict__ out) {
    long c = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (c >= (long)ny * nx) return;
    double xb, yb;
    sl_backtrace(a, b, X[c], Y[c], dt, dx, dy, nx, ny, xb, yb);
    out[c] = bilinear(q, xb, yb, dx, dy, nx, ny);
}
__global__ void k_all_finite2(const double *__restrict__ a, const double *__restrict__ b, long n,
                              int *bad) {
    long k = blockIdx.x * (long)blockDim.x + threadIdx.x;
    bool ok = true;
    for (; k < n; k += (long)gridDim.x * blockDim.x) ok &= isfinite(a[k]) && isfinite(b[k]);
    if (!ok) atomicOr(bad, 1);
}
__global__ void k_phi_disc(const double *__restrict__ X1, const double *__restrict__ X2, long n,
                           double x0, double y0, double R, double *__restrict__ phi) {
    long k = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (k < n) phi[k] = disc_phi(X1[k], X2[k], x0, y0, R);
}

// ------------------------------------------------------------------------ WENO5 ----
__global__ void k_weno5_rhs(const double *__restrict__ q, const double *__restrict__ a,
                            const double *__restrict__ b, int ny, int nx, double dx, double dy,
                            const double *__restrict__ phi, double w_cut,
                            double *__restrict__ rhs) {
    long c = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (c >= (long)ny * nx) return;
    int j = (int)(c / nx), i = (int)(c % nx);
    double r = 0.0;
    if (j >= 2 && j < ny - 2 && i >= 2 && i < nx - 2 && !(phi[c] > w_cut)) {
        double u = a[c], v = b[c];
        double dqdx = weno5_diff(q + c, 1, i, nx, u) / dx;
        double dqdy = weno5_diff(q + c, nx, j, ny, v) / dy;
        r = -(u * dqdx + v * dqdy);
    }
    rhs[c] = r;
}
// functions.py:420-444 _central2_rhs (mode 0) and :466-489 _conservative_rhs (mode 1):
// interior cells with phi <= w_cut, +/-1 central stencils, zero elsewhere
__global__ void k_central_rhs(const double *__restrict__ q, const double *__restrict__ a,
                              const double *__restrict__ b, int ny, int nx, double dx, double dy,
                              const double *__restrict__ phi, double w_cut, int mode,
                              double *__restrict__ rhs) {
    const long c = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (c >= (long)ny * nx) return;
    const int j = (int)(c / nx), i = (int)(c % nx);
    double r = 0.0;
    if (j >= 1 && j < ny - 1 && i >= 1 && i < nx - 1 && !(phi[c] > w_cut)) {
        const double ix2 = 0.5 / dx, iy2 = 0.5 / dy;
        if (mode == 0) {
            const double dqdx = (q[c + 1] - q[c - 1]) * ix2, dqdy = (q[c + nx] - q[c - nx]) * iy2;
            r = -(a[c] * dqdx + b[c] * dqdy);
        } else {
            const double dux = (a[c + 1] * q[c + 1] - a[c - 1] * q[c - 1]) * ix2;
            const double dvy = (b[c + nx] * q[c + nx] - b[c - nx] * q[c - nx]) * iy2;
            r = -(dux + dvy);
        }
    }
    rhs[c] = r;
}
__global__ void k_bicubic(const double *__restrict__ u, const double *__restrict__ xq,
                          const double *__restrict__ yq, long nq, double dx, double dy, int nx,
                          int ny, double *__restrict__ out) {
    const long k = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (k < nq) out[k] = bicubic(u, xq[k], yq[k], dx, dy, nx, ny);
}
__global__ void k_sl_cubic(const double *__restrict__ q, const double *__restrict__ a,
                           const double *__restrict__ b, const double *__restrict__ X,
                           const double *__restrict__ Y, int ny, int nx, double dt, double dx,
                           double dy, double *__restrict__ out) {
    const long c = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (c >= (long)ny * nx) return;
    double xb, yb;
    sl_backtrace_cubic(a, b, X[c], Y[c], dt, dx, dy, nx, ny, xb, yb);
    out[c] = bicubic(q, xb, yb, dx, dy, nx, ny);
}

// SSP-RK3 stage combinations (functions.py:407-413); stage 0: q + dt r,
// stage 1: 0.75 q + 0.25 (q1 + dt r), stage 2: (1/3) q + (2/3) (q2 + dt r).
__global__ void k_ssprk3_combine(const double *__restrict__ q, const double *__restrict__ qs,
                                 const double *__restrict__ r, long n, double dt, int stage,
                                 double *__restrict__ out) {
    long k = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (k >= n) return;
    if (stage == 0) out[k] = q[k] + dt * r[k];
    else if (stage == 1) out[k] = 0.75 * q[k] + 0.25 * (qs[k] + dt * r[k]);
    else out[k] = (1.0 / 3.0) * q[k] + (2.0 / 3.0) * (qs[k] + dt * r[k]);
}

// ------------------------------------------------------------------ solid stress ----
__global__ void k_solid_stress(const double *__restrict__ X1, const double *__restrict__ X2,
                               const double *__restrict__ phi, int ny, int nx, double dx,
                               double dy, double mu_s, double kappa, double w_cut, double clamp,
                               int iso, double *__restrict__ sxx, double *__restrict__ sxy,
                               double *__restrict__ syy, double *__restrict__ J) {
    long c = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (c >= (long)ny * nx) return;
    int j = (int)(c / nx), i = (int)(c % nx);
    Stress s{0.0, 0.0, 0.0, 1.0};
    if (j >= 1 && j < ny - 1 && i >= 1 && i < nx - 1)
        solid_stress_cell(X1, X2, phi, c, nx, dx, dy, mu_s, kappa, w_cut, clamp, iso != 0, s);
    sxx[c] = s.sxx; sxy[c] = s.sxy; syy[c] = s.syy; J[c] = s.J;
}
__global__ void k_heaviside(const double *__restrict__ x, long n, double w_t,
                            double *__restrict__ H) {
    long k = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (k < n) H[k] = heaviside(x[k], w_t);
}

// ----------------------------------------------------------------------- BCs ----
__global__ void k_apply_bc(int kind, double lid, double *u, double *v, int ny, int nx) {
    // in place: boundary cells only read interior (never written) source cells
    long c = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (c >= (long)ny * nx) return;
    int j = (int)(c / nx), i = (int)(c % nx);
    if (!(i == 0 || i == nx - 1 || j == 0 || j == ny - 1)) return;
    BCSrc s = bc_source(kind, lid, j, i, ny, nx);
    double uu = s.u_const ? s.u_val : u[s.u_src];
    double vv = s.v_const ? s.v_val : v[s.v_src];
    u[c] = uu; v[c] = vv;
}

// -------------------------------------------------------------------- projection ----
// rows [jb, je) of an nx-wide plane: blockIdx.y = row - jb, 256 columns per block
static inline dim3 rows_grid(int nx, int jb, int je) { return dim3((nx + 255) / 256, je - jb); }
// rho > 0: the projection's rhs = (rho * divU) / dt (functions.py:1331, the same two
// roundings as the separate scale and divide passes)
struct RcDiv { DivK x2, y2, x1, y1; };   // 2dx, 2dy, dx, dy (divk.hpp)
static RcDiv rc_div(double dx, double dy) {
    return RcDiv{divk_make(2.0 * dx), divk_make(2.0 * dy), divk_make(dx), divk_make(dy)};
}
__device__ __forceinline__ void div_rc_cell(const double *__restrict__ a,
                                            const double *__restrict__ b,
                                            const double *__restrict__ p, int ny, int nx,
                                            double d_f, const RcDiv &K,
                                            double *__restrict__ divU, double rho, double dt,
                                            int j, int i) {
    const long c = (long)j * nx + i;
    if (j < 1 || j >= ny - 1 || i < 1 || i >= nx - 1) {
        divU[c] = rho > 0 ? (rho * 0.0) / dt : 0.0;
        return;
    }
    double gxl = grad2k(p + c - 1, 1, i - 1, nx, K.x2), gxc = grad2k(p + c, 1, i, nx, K.x2),
           gxr = grad2k(p + c + 1, 1, i + 1, nx, K.x2);
    double gyd = grad2k(p + c - nx, nx, j - 1, ny, K.y2), gyc = grad2k(p + c, nx, j, ny, K.y2),
           gyu = grad2k(p + c + nx, nx, j + 1, ny, K.y2);
    double ue = 0.5 * (a[c] + a[c + 1]) - d_f * (divk(p[c + 1] - p[c], K.x1) - 0.5 * (gxc + gxr));
    double uw = 0.5 * (a[c - 1] + a[c]) - d_f * (divk(p[c] - p[c - 1], K.x1) - 0.5 * (gxl + gxc));
    double vn = 0.5 * (b[c] + b[c + nx]) - d_f * (divk(p[c + nx] - p[c], K.y1) - 0.5 * (gyc + gyu));
    double vs = 0.5 * (b[c - nx] + b[c]) - d_f * (divk(p[c] - p[c - nx], K.y1) - 0.5 * (gyd + gyc));
    const double d = divk(ue - uw, K.x1) + divk(vn - vs, K.y1);
    divU[c] = rho > 0 ? (rho * d) / dt : d;
}
__global__ void k_divergence_rc(const double *__restrict__ a, const double *__restrict__ b,
                                const double *__restrict__ p, int ny, int nx, double d_f,
                                RcDiv K, double *__restrict__ divU, int jb, int je,
                                double rho = 0.0, double dt = 1.0,
                                const double *__restrict__ dtp = nullptr,
                                const unsigned char *__restrict__ rowmark = nullptr) {
    if (rowmark && !rowmark[jb + blockIdx.y]) return;   // only the listed rows
    if (dtp) { dt = *dtp; d_f = dt / rho; }   // the host's dt / rho
    // Grid: rows_grid (one block row per grid row, no per-cell division).
    const int j = jb + (int)blockIdx.y, i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nx || j >= je) return;
    div_rc_cell(a, b, p, ny, nx, d_f, K, divU, rho, dt, j, i);
}
// k_divergence_rc over the whole grid in 64 x 16 tiles: p staged through LDS on the tile + 2
// (rows and columns), a* and b* straight into registers (each lane owns one column and four
// consecutive rows: a*'s east / west neighbours come from the adjacent lanes, b*'s north /
// south from the lane's own column).  Each stencil value is loaded from global memory once per
// tile (the row kernel's five p rows per output row were five L2 round trips per cell), and
// every gradient / face quotient is formed once: gy and fy = (p_{j+1} - p_j) / dy at rows
// r0 - 1 .. r0 + 4 (r0 + 3) in registers, gx and fx = (p_{i+1} - p_i) / dx of the lane's
// column with its neighbours' by lane shuffles, the tile's edge columns (gx, fx at i0 - 1, gx
// at i0 + 64; a* at i0 - 1 and i0 + 64) by the first lanes in one pass: 7 quotients per cell
// instead of div_rc_cell's 14.  Every value is div_rc_cell's quotient / sum of the same
// operands in the same order, so the result is bit-identical.  152 vs 161 us per full-grid
// launch at N = 4096 (profiles/r06/ktdiv; 84 VGPRs, five blocks per CU as before: at 6 or 8
// waves per SIMD it spills, 8: 276 us).  One-dimensional grid, tiles grouped per XCD (each
// XCD's L2 sees a contiguous band of tile rows and their halos).
constexpr int DVT_X = 64, DVT_Y = 16, DVT_PX = DVT_X + 4, DVT_PY = DVT_Y + 4;
static_assert(DVT_X == 64 && DVT_Y == 16, "k_divergence_t: a wave per 4 tile rows, a lane per column");
// one 64 x 16 tile at (i0, j0), 256 threads, sp: the block's p tile (DVT_PY x DVT_PX)
__device__ __forceinline__ void div_rc_tile(const double *__restrict__ a,
                                            const double *__restrict__ b,
                                            const double *__restrict__ p, int ny, int nx,
                                            double d_f, const RcDiv &K, double *__restrict__ divU,
                                            double rho, double dt, int i0, int j0, double *sp) {
    const int tx = threadIdx.x & 63, r0 = 4 * (threadIdx.x >> 6), i = i0 + tx;
    constexpr int NP = (DVT_PY * DVT_PX + 255) / 256;
    double vp[NP], av[4], bv[6], ae = 0.0;
    // every load issued before the first LDS write (cells outside the grid: never read by an
    // interior cell's stencil, which turns one-sided at the edges)
#pragma unroll
    for (int k = 0; k < NP; ++k) {
        const int q = threadIdx.x + 256 * k, r = q / DVT_PX, s = q % DVT_PX;
        const int j = j0 - 2 + r, ii = i0 - 2 + s;
        const bool ok = q < DVT_PY * DVT_PX && j >= 0 && j < ny && ii >= 0 && ii < nx;
        vp[k] = ok ? p[(long)j * nx + ii] : 0.0;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {   // a* on rows r0 .. r0 + 3
        const int j = j0 + r0 + q;
        av[q] = (j < ny && i < nx) ? a[(long)j * nx + i] : 0.0;
    }
#pragma unroll
    for (int q = 0; q < 6; ++q) {   // b* on rows r0 - 1 .. r0 + 4
        const int j = j0 + r0 - 1 + q;
        bv[q] = (j >= 0 && j < ny && i < nx) ? b[(long)j * nx + i] : 0.0;
    }
    if (tx < 8) {   // a* at the tile's edge columns: lane 2q + 0 / 1 -> row r0 + q, i0 - 1 / i0 + 64
        const int j = j0 + r0 + (tx >> 1), ii = (tx & 1) ? i0 + DVT_X : i0 - 1;
        if (j < ny && ii >= 0 && ii < nx) ae = a[(long)j * nx + ii];
    }
#pragma unroll
    for (int k = 0; k < NP; ++k) {
        const int q = threadIdx.x + 256 * k;
        if (q < DVT_PY * DVT_PX) sp[q] = vp[k];
    }
    __syncthreads();
    const long PS = DVT_PX;
    const double *pcol = sp + 2 * DVT_PX + tx + 2;   // tile row 0, column i
    // gy at tile row rr, fy = (p_{rr+1} - p_rr) / dy (0 where no interior cell reads them)
    auto gyat = [&](int rr) {
        const int j = j0 + rr;
        return (i < nx && j >= 0 && j < ny) ? grad2k(pcol + rr * PS, PS, j, ny, K.y2) : 0.0;
    };
    auto fyat = [&](int rr) {
        const int j = j0 + rr;
        return (i < nx && j >= 0 && j + 1 < ny) ? divk(pcol[(rr + 1) * PS] - pcol[rr * PS], K.y1) : 0.0;
    };
    // a window down the column: gy at rows ty - 1, ty, ty + 1 and fy at ty - 1, ty
    double gyd = gyat(r0 - 1), gyc = gyat(r0), fys = fyat(r0 - 1);
    double ex = 0.0;
    if (tx < 12) {   // lane 3q + 0 / 1 / 2 -> row r0 + q: gx(i0 - 1), fx(i0 - 1), gx(i0 + 64)
        const int rr = r0 + tx / 3, kind = tx % 3, j = j0 + rr;
        const double *prow = sp + (rr + 2) * DVT_PX + 2;   // column i0 at [0]
        if (j < ny) {
            if (kind == 0) {
                if (i0 >= 1 && i0 - 1 < nx) ex = grad2k(prow - 1, 1, i0 - 1, nx, K.x2);
            } else if (kind == 1) {
                if (i0 >= 1 && i0 < nx) ex = divk(prow[0] - prow[-1], K.x1);
            } else if (i0 + DVT_X < nx) {
                ex = grad2k(prow + DVT_X, 1, i0 + DVT_X, nx, K.x2);
            }
        }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int ty = r0 + q, j = j0 + ty;
        const double *pc = pcol + ty * PS;
        const double gxc = (i < nx && j < ny) ? grad2k(pc, 1, i, nx, K.x2) : 0.0;
        const double fxc = (i + 1 < nx && j < ny) ? divk(pc[1] - pc[0], K.x1) : 0.0;
        double gxl = __shfl(gxc, (tx + 63) & 63), gxr = __shfl(gxc, (tx + 1) & 63);
        double fxl = __shfl(fxc, (tx + 63) & 63);
        double al = __shfl(av[q], (tx + 63) & 63), ar = __shfl(av[q], (tx + 1) & 63);
        const double e0 = __shfl(ex, 3 * q), e1 = __shfl(ex, 3 * q + 1), e2 = __shfl(ex, 3 * q + 2);
        const double a0 = __shfl(ae, 2 * q), a1 = __shfl(ae, 2 * q + 1);
        if (tx == 0) { gxl = e0; fxl = e1; al = a0; }
        if (tx == 63) { gxr = e2; ar = a1; }
        const double gyu = gyat(ty + 1), fyn = fyat(ty);
        const double gyd_ = gyd, gyc_ = gyc, fys_ = fys;
        gyd = gyc; gyc = gyu; fys = fyn;
        if (j >= ny || i >= nx) continue;
        const long c = (long)j * nx + i;
        if (j < 1 || j >= ny - 1 || i < 1 || i >= nx - 1) {
            divU[c] = rho > 0 ? (rho * 0.0) / dt : 0.0;
            continue;
        }
        // div_rc_cell's expressions, operand for operand
        double ue = 0.5 * (av[q] + ar) - d_f * (fxc - 0.5 * (gxc + gxr));
        double uw = 0.5 * (al + av[q]) - d_f * (fxl - 0.5 * (gxl + gxc));
        double vn = 0.5 * (bv[q + 1] + bv[q + 2]) - d_f * (fyn - 0.5 * (gyc_ + gyu));
        double vs = 0.5 * (bv[q] + bv[q + 1]) - d_f * (fys_ - 0.5 * (gyd_ + gyc_));
        const double d = divk(ue - uw, K.x1) + divk(vn - vs, K.y1);
        divU[c] = rho > 0 ? (rho * d) / dt : d;
    }
}
__global__ void __launch_bounds__(256) k_divergence_t(const double *__restrict__ a,
                                                      const double *__restrict__ b,
                                                      const double *__restrict__ p, int ny, int nx,
                                                      double d_f, RcDiv K,
                                                      double *__restrict__ divU, double rho,
                                                      double dt, const double *__restrict__ dtp,
                                                      int tiles_x, int ntiles) {
    __shared__ double sp[DVT_PY * DVT_PX];
    if (dtp) { dt = *dtp; d_f = dt / rho; }   // the host's dt / rho
    const int per = ntiles / 8, bk = blockIdx.x;
    const int tile = bk < 8 * per ? (bk % 8) * per + bk / 8 : bk;
    div_rc_tile(a, b, p, ny, nx, d_f, K, divU, rho, dt, (tile % tiles_x) * DVT_X,
                (tile / tiles_x) * DVT_Y, sp);
}
static int divergence_full(hipStream_t st, const double *a, const double *b, const double *p,
                           int ny, int nx, double d_f, const RcDiv &K, double *divU, double rho,
                           double dt, const double *dtp) {
    const int tx = (nx + DVT_X - 1) / DVT_X, nt = tx * ((ny + DVT_Y - 1) / DVT_Y);
    k_divergence_t<<<nt, 256, 0, st>>>(a, b, p, ny, nx, d_f, K, divU, rho, dt, dtp, tx, nt);
    RMT_LAUNCHED();
    return RMT_OK;
}
// The rhs on the listed MOM_TX x MOM_TY tiles grown by one cell (the cells whose stencil
// reads a u*, v* the momentum fix-up rewrote); one block per tile.  Overlapping grown tiles
// write the same value twice.
__global__ void __launch_bounds__(256) k_divergence_tiles(
    const double *__restrict__ a, const double *__restrict__ b, const double *__restrict__ p,
    int ny, int nx, RcDiv K, double *__restrict__ divU, double rho, double dt,
    const double *__restrict__ dtp, const int *__restrict__ tiles,
    const int *__restrict__ count, int tiles_x) {
    static_assert(MOM_TX == DVT_X && MOM_TY == DVT_Y, "k_divergence_tiles: momentum tiles are div_rc_tile's");
    __shared__ double sp[DVT_PY * DVT_PX];
    if (dtp) dt = *dtp;
    const double d_f = dt / rho;   // as the host's dt / rho
    const int cnt = *count;
    constexpr int TW = MOM_TX + 2;
    for (int bk = blockIdx.x; bk < cnt; bk += gridDim.x) {   // list_grid launch
        const int t = tiles[bk];
        const int ti0 = (t % tiles_x) * MOM_TX, tj0 = (t / tiles_x) * MOM_TY;
        // the tile itself (k_divergence_t's body), then its one-cell ring cell by cell
        div_rc_tile(a, b, p, ny, nx, d_f, K, divU, rho, dt, ti0, tj0, sp);
        for (int e = threadIdx.x; e < 2 * TW + 2 * MOM_TY; e += blockDim.x) {
            int j, i;
            if (e < 2 * TW) { j = e < TW ? tj0 - 1 : tj0 + MOM_TY; i = ti0 - 1 + e % TW; }
            else { const int f = e - 2 * TW; j = tj0 + f % MOM_TY; i = f < MOM_TY ? ti0 - 1 : ti0 + MOM_TX; }
            if (j >= 0 && j < ny && i >= 0 && i < nx)
                div_rc_cell(a, b, p, ny, nx, d_f, K, divU, rho, dt, j, i);
        }
        __syncthreads();   // sp is the next tile's
    }
}
__global__ void k_divergence_central(const double *__restrict__ a, const double *__restrict__ b,
                                     int ny, int nx, double dx, double dy,
                                     double *__restrict__ divU) {
    long c = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (c >= (long)ny * nx) return;
    int j = (int)(c / nx), i = (int)(c % nx);
    divU[c] = (j < 1 || j >= ny - 1 || i < 1 || i >= nx - 1)
                  ? 0.0
                  : (a[c + 1] - a[c - 1]) / (2 * dx) + (b[c + nx] - b[c - nx]) / (2 * dy);
}
__global__ void k_pressure_gradient(const double *__restrict__ p, int ny, int nx, double dx,
                                    double dy, double *__restrict__ gx, double *__restrict__ gy) {
    long c = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (c >= (long)ny * nx) return;
    double x, y;
    pgrad_cell(p, c, (int)(c / nx), (int)(c % nx), ny, nx, dx, dy, x, y);
    gx[c] = x; gy[c] = y;
}
// functions.py:1330-1362 after the solve: a = a* - (dt/rho) dpc/dx, BC, p = p_prev + pc,
// with pc = p_raw - mean(p_raw) (mean on device).  Writes p before its own mean removal.
// functions.py:1350-1358 after the solve: a = a* - (dt/rho) dpc/dx, BC, p = p_prev + pc.
// Writes p before its mean removal.
// pc - m is the mean-free correction (m: the solve's mean, subtracted here as pc is read)
__device__ __forceinline__ double corrected(const double *__restrict__ s,
                                            const double *__restrict__ pc, long c, int ny, int nx,
                                            const DivK &Kx2, const DivK &Ky2, double dt_rho,
                                            int comp, double m) {
    int j = (int)(c / nx), i = (int)(c % nx);
    double gx, gy;
    pgrad_cellk(pc, c, j, i, ny, nx, Kx2, Ky2, gx, gy, m);
    return s[c] - dt_rho * (comp == 0 ? gx : gy);
}
// root (nullable): the row-tree sum of pc (dct_solve's dev_root), mean = root / count
__global__ void k_project_correct(const double *__restrict__ a_s, const double *__restrict__ b_s,
                                  const double *__restrict__ pc, const double *__restrict__ p_prev,
                                  int ny, int nx, DivK Kx2, DivK Ky2, double dt_rho, int bc,
                                  double lid, double *__restrict__ a, double *__restrict__ b,
                                  double *__restrict__ p, int jb, int je,
                                  const double *__restrict__ root, double count,
                                  const double *__restrict__ dtp = nullptr, double rho = 1.0,
                                  double *__restrict__ m2part = nullptr, int defer_p = 0) {
    const int j = jb + (int)blockIdx.y, i = blockIdx.x * blockDim.x + threadIdx.x;
    double q = -INFINITY;
    if (i < nx && j < je) {
        if (dtp) dt_rho = *dtp / rho;   // the host's dt / rho
        const double m = root ? *root / count : 0.0;
        const long c = (long)j * nx + i;
        double ua, vb;
        if (j >= 1 && j < ny - 1 && i >= 1 && i < nx - 1) {
            // interior: every BC kind is the identity and grad2 is centred; the numerators are
            // differences of (pc - m) terms, certified by noting pc's four operands and m
            // (divk.hpp DivNote), else the checked division -- the same quotients either way
            const double xe = pc[c + 1], xw = pc[c - 1], yn = pc[c + nx], ys = pc[c - nx];
            DivNote nt;
            nt.note(xe); nt.note(xw); nt.note(yn); nt.note(ys); nt.note(m);
            const double nxn = (xe - m) - (xw - m), nyn = (yn - m) - (ys - m);
            double gx, gy;
            if (__builtin_expect(nt.ok() && Kx2.rspan && Ky2.rspan, 1)) {
                gx = divk_nc(nxn, Kx2); gy = divk_nc(nyn, Ky2);
            } else {
                gx = divk(nxn, Kx2); gy = divk(nyn, Ky2);
            }
            ua = a_s[c] - dt_rho * gx;
            vb = b_s[c] - dt_rho * gy;
        } else {
            BCSrc s = bc_source(bc, lid, j, i, ny, nx);
            ua = s.u_const ? s.u_val : corrected(a_s, pc, s.u_src, ny, nx, Kx2, Ky2, dt_rho, 0, m);
            vb = s.v_const ? s.v_val : corrected(b_s, pc, s.v_src, ny, nx, Kx2, Ky2, dt_rho, 1, m);
        }
        a[c] = ua; b[c] = vb;
        // defer_p: p = p_prev + (pc - m) is formed by the step's deferred mean-removal pass
        // instead (k_rowsum_upd, the same expression), off the critical path
        if (!defer_p) p[c] = p_prev ? p_prev[c] + (pc[c] - m) : (pc[c] - m);
        q = ua * ua + vb * vb;
    }
    if (m2part) {
        // max of u^2 + v^2 over the block, NaN-propagating (k_reduce_p1<3>'s rule; a max is
        // exact in any order): across each wave by shuffles, then the 4 wave results
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            const double y = __shfl_xor(q, off);
            if (y > q || y != y) q = y;
        }
        __shared__ double s[4];
        if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = q;
        __syncthreads();
        if (threadIdx.x == 0) {
            double m = s[0];
            for (int w = 1; w < 4; ++w)
                if (s[w] > m || s[w] != s[w]) m = s[w];
            m2part[(long)blockIdx.y * gridDim.x + blockIdx.x] = m;
        }
    }
}
__global__ void k_scale_copy(const double *__restrict__ x, long n, double s,
                             double *__restrict__ y) {
    long k = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (k < n) y[k] = s * x[k];
}
__global__ void k_div_scalar(const double *__restrict__ x, long n, double s,
                             double *__restrict__ y) {
    long k = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (k < n) y[k] = x[k] / s;
}
// Row-window launches for the slab-decomposed step (global cell indices, rows [jb, je))
int divergence_rc_rows(rmt_ctx *ctx, const double *a, const double *b, const double *p,
                       double d_f, double dx, double dy, double *divU, int jb, int je,
                       double rho, double dt, const double *dtp) {
    if (je > jb)
        k_divergence_rc<<<rows_grid(ctx->nx, jb, je), 256, 0, ctx->stream>>>(
            a, b, p, ctx->ny, ctx->nx, d_f, rc_div(dx, dy), divU, jb, je, rho, dt, dtp);
    RMT_LAUNCHED();
    return RMT_OK;
}
int project_correct_rows(rmt_ctx *ctx, const double *a_s, const double *b_s, const double *pc,
                         const double *p_prev, double dx, double dy, double dt_rho, int bc,
                         double lid, double *a, double *b, double *p, int jb, int je,
                         const double *dtp, double rho) {
    if (je > jb)
        k_project_correct<<<rows_grid(ctx->nx, jb, je), 256, 0, ctx->stream>>>(
            a_s, b_s, pc, p_prev, ctx->ny, ctx->nx, divk_make(2 * dx), divk_make(2 * dy), dt_rho, bc, lid, a, b, p, jb, je,
            nullptr, 1.0, dtp, rho);
    RMT_LAUNCHED();
    return RMT_OK;
}
}  // namespace rmt

using namespace rmt;

// ======================================================================== C ABI ====
extern "C" {

const char *rmt_last_error(void) { return g_err.c_str(); }
int rmt_version(void) { return 1; }

int rmt_ctx_create(int ny, int nx, int device, void *stream, rmt_ctx **out) {
    RMT_CHECK(out && ny >= 5 && nx >= 5, RMT_EINVAL, "rmt_ctx_create: need ny, nx >= 5");
    RMT_HIP(hipSetDevice(device));
    rmt_ctx *c = new rmt_ctx;
    c->ny = ny; c->nx = nx; c->device = device; c->stream = (hipStream_t)stream;
    c->opt = opts_from_env();
    RMT_HIP(hipMalloc(&c->red, (RED_BLOCKS + 64) * sizeof(double)));
    c->rsum_len = ny > 8192 ? ny : 8192;
    RMT_HIP(hipMalloc(&c->rsum, c->rsum_len * sizeof(double)));
    *out = c;
    return RMT_OK;
}
int rmt_ctx_set_option(rmt_ctx *ctx, const char *name, int value) {
    RMT_CHECK(ctx && name, RMT_EINVAL, "null argument");
    for (const auto &k : kOpts)
        if (!strcmp(k.name, name)) {
            ctx->opt.*(k.f) = value;
            ctx->bytes_gen++;   // a carried step state was prepared under the old options
            return RMT_OK;
        }
    set_error(std::string("rmt_ctx_set_option: unknown option ") + name);
    return RMT_EINVAL;
}
int rmt_ctx_get_option(rmt_ctx *ctx, const char *name, int *value) {
    RMT_CHECK(ctx && name && value, RMT_EINVAL, "null argument");
    for (const auto &k : kOpts)
        if (!strcmp(k.name, name)) { *value = ctx->opt.*(k.f); return RMT_OK; }
    set_error(std::string("rmt_ctx_get_option: unknown option ") + name);
    return RMT_EINVAL;
}
int rmt_ctx_set_stream(rmt_ctx *ctx, void *stream) {
    RMT_CHECK(ctx, RMT_EINVAL, "null ctx");
    ctx->stream = (hipStream_t)stream;
    return RMT_OK;
}
int rmt_ctx_sync(rmt_ctx *ctx) {
    RMT_HIP(hipStreamSynchronize(ctx->stream));
    return RMT_OK;
}
int rmt_ctx_set_profiling(rmt_ctx *ctx, int on) {
    RMT_CHECK(ctx, RMT_EINVAL, "null ctx");
    if (on && !ctx->ev[0])
        for (auto &e : ctx->ev) RMT_HIP(hipEventCreate(&e));
    ctx->prof = on != 0;
    return RMT_OK;
}
int rmt_ctx_kernel_ms(rmt_ctx *ctx, double *ms2) {
    RMT_CHECK(ctx && ms2 && ctx->ev[0], RMT_EINVAL, "profiling not enabled");
    RMT_HIP(hipStreamSynchronize(ctx->stream));
    for (int k = 0; k < 2; ++k) {   // an interval never recorded reads as 0
        float f = 0;
        ms2[k] = hipEventElapsedTime(&f, ctx->ev[2 * k], ctx->ev[2 * k + 1]) == hipSuccess ? f : 0.0;
    }
    (void)hipGetLastError();
    return RMT_OK;
}

int rmt_ctx_destroy(rmt_ctx *ctx) {
    if (!ctx) return RMT_OK;
    (void)hipSetDevice(ctx->device);
    if (ctx->scratch) (void)hipFree(ctx->scratch);
    if (ctx->red) (void)hipFree(ctx->red);
    if (ctx->rsum) (void)hipFree(ctx->rsum);
    if (ctx->bytes) (void)hipFree(ctx->bytes);
    if (ctx->dct) dct_destroy(ctx->dct);
    if (ctx->dct2) dct2_destroy(ctx->dct2);
    if (ctx->per) per_destroy(ctx->per);
    for (auto es : ctx->edge_sts)
        if (es) (void)hipStreamSynchronize(es);
    for (auto &e : ctx->edge)
        if (e.list) (void)hipFree(e.list);
    for (auto es : ctx->edge_sts)
        if (es) (void)hipStreamDestroy(es);
    for (auto &e : ctx->edge_ev)
        if (e) (void)hipEventDestroy(e);
    for (auto &e : ctx->ev)
        if (e) (void)hipEventDestroy(e);
    imex_destroy(ctx);
    delete ctx;
    return RMT_OK;
}

#define N_CELLS ((long)ctx->ny * ctx->nx)
#define LAUNCH1D(n) grid1d((n), 256), 256, 0, ctx->stream

int rmt_grad_x_2nd(rmt_ctx *ctx, const double *f, double h, double *out) {
    k_grad_x<<<LAUNCH1D(N_CELLS)>>>(f, ctx->ny, ctx->nx, 2 * h, out);
    RMT_LAUNCHED();
    return RMT_OK;
}
int rmt_grad_y_2nd(rmt_ctx *ctx, const double *f, double h, double *out) {
    k_grad_y<<<LAUNCH1D(N_CELLS)>>>(f, ctx->ny, ctx->nx, 2 * h, out);
    RMT_LAUNCHED();
    return RMT_OK;
}
int rmt_diff_upwind_3rd(rmt_ctx *ctx, const double *f, const double *vel, double h, int axis,
                        double *out) {
    RMT_CHECK(axis == 0 || axis == 1, RMT_EINVAL, "diff_upwind_3rd: axis must be 0 or 1");
    k_upwind<<<LAUNCH1D(N_CELLS)>>>(f, vel, ctx->ny, ctx->nx, h, axis, out);
    RMT_LAUNCHED();
    return RMT_OK;
}
int rmt_bilinear_interpolate(rmt_ctx *ctx, const double *u, const double *xq, const double *yq,
                             long nq, double dx, double dy, double *out) {
    if (nq <= 0) return RMT_OK;
    k_bilinear<<<LAUNCH1D(nq)>>>(u, xq, yq, nq, dx, dy, ctx->nx, ctx->ny, out);
    RMT_LAUNCHED();
    return RMT_OK;
}
int rmt_advect_sl_rk4(rmt_ctx *ctx, const double *q, const double *a, const double *b,
                      const double *X, const double *Y, double dt, double dx, double dy,
                      double *out) {
    k_sl_rk4<<<LAUNCH1D(N_CELLS)>>>(q, a, b, X, Y, ctx->ny, ctx->nx, dt, dx, dy, out);
    RMT_LAUNCHED();
    return RMT_OK;
}
__global__ void k_divk_selftest(const double *__restrict__ x, long n, DivK K,
                                double *__restrict__ q, double *__restrict__ qi) {
    const long k = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (k < n) { q[k] = divk(x[k], K); qi[k] = x[k] / K.d; }
}
int rmt_selftest_divk(rmt_ctx *ctx, const double *x, long n, double d, double *q,
                      double *q_ieee) {
    RMT_CHECK(ctx && (n == 0 || (x && q && q_ieee)), RMT_EINVAL, "null argument");
    RMT_CHECK(n >= 0, RMT_EINVAL, "rmt_selftest_divk: n < 0");
    if (n) k_divk_selftest<<<grid1d(n, 256), 256, 0, ctx->stream>>>(x, n, divk_make(d), q, q_ieee);
    RMT_LAUNCHED();
    return RMT_OK;
}
int rmt_all_finite2(rmt_ctx *ctx, const double *a, const double *b, int *finite) {
    RMT_TRY(ensure_bytes(ctx, 64));
    int *bad = (int *)ctx->bytes;
    RMT_HIP(hipMemsetAsync(bad, 0, sizeof(int), ctx->stream));
    k_all_finite2<<<1024, 256, 0, ctx->stream>>>(a, b, N_CELLS, bad);
    int h = 0;
    RMT_HIP(hipMemcpyAsync(&h, bad, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
    RMT_HIP(hipStreamSynchronize(ctx->stream));
    *finite = !h;
    return RMT_OK;
}
int rmt_rebuild_phi_disc(rmt_ctx *ctx, const double *X1, const double *X2, double x0, double y0,
                         double R, double *phi) {
    k_phi_disc<<<LAUNCH1D(N_CELLS)>>>(X1, X2, N_CELLS, x0, y0, R, phi);
    RMT_LAUNCHED();
    return RMT_OK;
}
int rmt_weno5_rhs(rmt_ctx *ctx, const double *q, const double *a, const double *b, double dx,
                  double dy, const double *phi, double w_cut, double *rhs) {
    k_weno5_rhs<<<LAUNCH1D(N_CELLS)>>>(q, a, b, ctx->ny, ctx->nx, dx, dy, phi, w_cut, rhs);
    RMT_LAUNCHED();
    return RMT_OK;
}
int rmt_advect_weno5_rk3(rmt_ctx *ctx, const double *q, const double *a, const double *b,
                         double dx, double dy, double dt, const double *phi, double w_cut,
                         double *out) {
    long n = N_CELLS;
    RMT_TRY(ensure_scratch(ctx, 3 * n * sizeof(double)));
    double *r = ctx->scratch, *q1 = r + n, *q2 = q1 + n;
    RMT_TRY(rmt_weno5_rhs(ctx, q, a, b, dx, dy, phi, w_cut, r));
    k_ssprk3_combine<<<LAUNCH1D(n)>>>(q, q, r, n, dt, 0, q1);
    RMT_TRY(rmt_weno5_rhs(ctx, q1, a, b, dx, dy, phi, w_cut, r));
    k_ssprk3_combine<<<LAUNCH1D(n)>>>(q, q1, r, n, dt, 1, q2);
    RMT_TRY(rmt_weno5_rhs(ctx, q2, a, b, dx, dy, phi, w_cut, r));
    k_ssprk3_combine<<<LAUNCH1D(n)>>>(q, q2, r, n, dt, 2, out);
    RMT_LAUNCHED();
    return RMT_OK;
}
int rmt_central_rhs(rmt_ctx *ctx, const double *q, const double *a, const double *b, double dx,
                    double dy, const double *phi, double w_cut, int conservative, double *rhs) {
    k_central_rhs<<<LAUNCH1D(N_CELLS)>>>(q, a, b, ctx->ny, ctx->nx, dx, dy, phi, w_cut,
                                         conservative ? 1 : 0, rhs);
    RMT_LAUNCHED();
    return RMT_OK;
}
int rmt_advect_central_rk3(rmt_ctx *ctx, const double *q, const double *a, const double *b,
                           double dx, double dy, double dt, const double *phi, double w_cut,
                           int conservative, double *out) {
    long n = N_CELLS;
    RMT_TRY(ensure_scratch(ctx, 3 * n * sizeof(double)));
    double *r = ctx->scratch, *q1 = r + n, *q2 = q1 + n;
    RMT_TRY(rmt_central_rhs(ctx, q, a, b, dx, dy, phi, w_cut, conservative, r));
    k_ssprk3_combine<<<LAUNCH1D(n)>>>(q, q, r, n, dt, 0, q1);
    RMT_TRY(rmt_central_rhs(ctx, q1, a, b, dx, dy, phi, w_cut, conservative, r));
    k_ssprk3_combine<<<LAUNCH1D(n)>>>(q, q1, r, n, dt, 1, q2);
    RMT_TRY(rmt_central_rhs(ctx, q2, a, b, dx, dy, phi, w_cut, conservative, r));
    k_ssprk3_combine<<<LAUNCH1D(n)>>>(q, q2, r, n, dt, 2, out);
    RMT_LAUNCHED();
    return RMT_OK;
}
int rmt_bicubic_interpolate(rmt_ctx *ctx, const double *u, const double *xq, const double *yq,
                            long nq, double dx, double dy, double *out) {
    if (nq <= 0) return RMT_OK;
    k_bicubic<<<LAUNCH1D(nq)>>>(u, xq, yq, nq, dx, dy, ctx->nx, ctx->ny, out);
    RMT_LAUNCHED();
    return RMT_OK;
}
int rmt_advect_sl_cubic_rk4(rmt_ctx *ctx, const double *q, const double *a, const double *b,
                            const double *X, const double *Y, double dt, double dx, double dy,
                            double *out) {
    k_sl_cubic<<<LAUNCH1D(N_CELLS)>>>(q, a, b, X, Y, ctx->ny, ctx->nx, dt, dx, dy, out);
    RMT_LAUNCHED();
    return RMT_OK;
}
int rmt_solid_cauchy_stress(rmt_ctx *ctx, const double *X1, const double *X2, double dx,
                            double dy, double mu_s, double kappa, const double *phi,
                            double w_cut, double detg_clamp, int isochoric, double *sxx,
                            double *sxy, double *syy, double *J) {
    k_solid_stress<<<LAUNCH1D(N_CELLS)>>>(X1, X2, phi, ctx->ny, ctx->nx, dx, dy, mu_s, kappa,
                                          w_cut, detg_clamp, isochoric, sxx, sxy, syy, J);
    RMT_LAUNCHED();
    return RMT_OK;
}
int rmt_smoothed_heaviside(rmt_ctx *ctx, const double *x, long n, double w_t, double *H) {
    if (n <= 0) return RMT_OK;
    k_heaviside<<<LAUNCH1D(n)>>>(x, n, w_t, H);
    RMT_LAUNCHED();
    return RMT_OK;
}
int rmt_apply_velocity_bc(rmt_ctx *ctx, int bc_kind, double lid, double *u, double *v) {
    RMT_CHECK(bc_kind >= 0 && bc_kind <= 3, RMT_EINVAL, "unknown velocity bc kind");
    k_apply_bc<<<LAUNCH1D(N_CELLS)>>>(bc_kind, lid, u, v, ctx->ny, ctx->nx);
    RMT_LAUNCHED();
    return RMT_OK;
}
int rmt_divergence_rc(rmt_ctx *ctx, const double *a, const double *b, const double *p,
                      double d_f, double dx, double dy, double *divU) {
    RMT_TRY(divergence_full(ctx->stream, a, b, p, ctx->ny, ctx->nx, d_f, rc_div(dx, dy), divU, 0.0,
                            1.0, nullptr));
    RMT_LAUNCHED();
    return RMT_OK;
}
int rmt_divergence_central(rmt_ctx *ctx, const double *a, const double *b, double dx,
                           double dy, double *divU) {
    k_divergence_central<<<LAUNCH1D(N_CELLS)>>>(a, b, ctx->ny, ctx->nx, dx, dy, divU);
    RMT_LAUNCHED();
    return RMT_OK;
}
int rmt_pressure_gradient(rmt_ctx *ctx, const double *p, double dx, double dy, double *gx,
                          double *gy) {
    k_pressure_gradient<<<LAUNCH1D(N_CELLS)>>>(p, ctx->ny, ctx->nx, dx, dy, gx, gy);
    RMT_LAUNCHED();
    return RMT_OK;
}
int rmt_solve_poisson_dct(rmt_ctx *ctx, const double *rhs, double dx, double dy, double *p) {
    return dct_solve(ctx, rhs, dx, dy, p);
}
int rmt_pressure_projection(rmt_ctx *ctx, const double *a_star, const double *b_star,
                            double dx, double dy, double dt, double rho, int bc_kind,
                            double lid, const double *p_prev, double *a, double *b, double *p) {
    RMT_CHECK(bc_kind >= 0 && bc_kind <= 3, RMT_EINVAL, "unknown velocity bc kind");
    long n = N_CELLS;
    RMT_TRY(ensure_scratch(ctx, 2 * n * sizeof(double)));
    double *rhs = ctx->scratch, *pc = rhs + n;
    // functions.py:1292-1295 + :1331: rhs = rho * divU / dt, d_f = dt / mean(rho)
    if (p_prev && rho > 0) {
        RMT_TRY(divergence_full(ctx->stream, a_star, b_star, p_prev, ctx->ny, ctx->nx, dt / rho,
                                rc_div(dx, dy), rhs, rho, dt, nullptr));
        RMT_LAUNCHED();
    } else {
        if (p_prev) RMT_TRY(rmt_divergence_rc(ctx, a_star, b_star, p_prev, dt / rho, dx, dy, rhs));
        else RMT_TRY(rmt_divergence_central(ctx, a_star, b_star, dx, dy, rhs));
        k_scale_copy<<<LAUNCH1D(n)>>>(rhs, n, rho, rhs);
        k_div_scalar<<<LAUNCH1D(n)>>>(rhs, n, dt, rhs);
    }
    // pc = the raw solve; its mean (functions.py:1119) is subtracted inside the correction
    double *root = ctx->red + RED_BLOCKS + 17;
    RMT_TRY(dct_solve(ctx, rhs, dx, dy, pc, root));
    k_project_correct<<<rows_grid(ctx->nx, 0, ctx->ny), 256, 0, ctx->stream>>>(a_star, b_star, pc, p_prev, ctx->ny, ctx->nx, divk_make(2 * dx), divk_make(2 * dy),
                                       dt / rho, bc_kind, lid, a, b, p, 0, ctx->ny, root, (double)n);
    RMT_LAUNCHED();
    RMT_TRY(sub_mean_rows(ctx, p, ctx->ny, ctx->nx));
    return RMT_OK;
}
int rmt_compute_timestep(rmt_ctx *ctx, const double *a, const double *b, double dx, double dy,
                         double CFL, double dt_min_cap, double mu_s, double rho_s, double gamma,
                         double rho_f, double mu_f, double eta_s, double kappa, double *dt) {
    (void)dy;
    RMT_TRY(reduce_maxsq2(ctx, a, b, N_CELLS, ctx->red + RED_BLOCKS));
    double m2;
    RMT_TRY(read_scalar(ctx, ctx->red + RED_BLOCKS, &m2));
    // functions.py:165-192 on the host (scalars); max(sqrt(.)) == sqrt(max(.))
    double cs = std::sqrt((kappa + mu_s * 4.0 / 3.0) / (rho_s + 1e-12));
    double d = CFL * dx / (cs + 1e-14);
    d = std::fmin(d, CFL * dx / (std::sqrt(m2) + 1e-6));
    if (gamma > 1e-12) {
        double ra = 0.5 * (rho_s + rho_f);
        d = std::fmin(d, std::sqrt((ra * std::pow(dx, 3.0)) / (2 * M_PI * gamma)) * 0.5);
    } else {
        d = std::fmin(d, 1.0);
    }
    double mu_max = std::fmax(mu_f, eta_s), rho_min = std::fmin(rho_s, rho_f);
    d = std::fmin(d, (mu_max > 1e-12 && rho_min > 1e-12) ? CFL * rho_min * std::pow(dx, 2.0) / (4.0 * mu_max)
                                                         : 1.0);
    *dt = std::fmin(d, dt_min_cap);
    return RMT_OK;
}
}  // extern "C"

namespace rmt {
// The projection in two parts around the extrapolation chain (sim.hip): the Rhie-Chow rhs and
// the row DCT-I of every row (or of the marked rows only) into scratch, then the rest.
int projection_rows(rmt_ctx *ctx, const double *a_star, const double *b_star, double dx,
                    double dy, const double *dtp, double dt, double rho, const double *p_prev,
                    const unsigned char *rowmark, const int *tiles, const int *tcount,
                    int max_tiles, const unsigned char *dct_skip) {
    RMT_CHECK(p_prev && rho > 0 && (!tiles || rowmark), RMT_EINVAL,
              "projection_rows: bad arguments");
    const long n = (long)ctx->ny * ctx->nx;
    RMT_TRY(ensure_scratch(ctx, 2 * n * sizeof(double)));
    double *rhs = ctx->scratch, *pc = rhs + n;
    if (tiles)   // the rhs of the other cells of the marked rows is still in scratch
        k_divergence_tiles<<<list_grid(max_tiles), 256, 0, ctx->stream>>>(
            a_star, b_star, p_prev, ctx->ny, ctx->nx, rc_div(dx, dy), rhs, rho, dt, dtp, tiles, tcount,
            (ctx->nx + MOM_TX - 1) / MOM_TX);
    else if (!rowmark)
        RMT_TRY(divergence_full(ctx->stream, a_star, b_star, p_prev, ctx->ny, ctx->nx, dt / rho,
                                rc_div(dx, dy), rhs, rho, dt, dtp));
    else
        k_divergence_rc<<<rows_grid(ctx->nx, 0, ctx->ny), 256, 0, ctx->stream>>>(
            a_star, b_star, p_prev, ctx->ny, ctx->nx, dt / rho, rc_div(dx, dy), rhs, 0, ctx->ny, rho, dt,
            dtp, rowmark);
    RMT_LAUNCHED();
    RMT_TRY(dct_plan(ctx, dx, dy));
    // dct_skip (the speculative full-grid call, rowmark null): the rows marked there are
    // transformed again after the fix-up -- this pass leaves them out
    if (!rowmark && dct_skip)
        return dct_pass(ctx, false, 0, rhs, pc, ctx->ny, 0, 1.0, nullptr, dct_skip, true);
    return dct_pass(ctx, false, 0, rhs, pc, ctx->ny, 0, 1.0, nullptr, rowmark);
}
int projection_finish(rmt_ctx *ctx, const double *a_star, const double *b_star, double dx,
                      double dy, const double *dtp, double dt, double rho, int bc_kind,
                      double lid, const double *p_prev, double *a, double *b, double *p,
                      double *m2part, bool sub_mean, const unsigned char *early_marks,
                      hipEvent_t done) {
    const long n = (long)ctx->ny * ctx->nx;
    double *pc = ctx->scratch + n, *root = ctx->red + RED_BLOCKS + 17;
    RMT_TRY(dct_solve_after_rows(ctx, pc, root, early_marks));
    RMT_CHECK(!done || !sub_mean, RMT_EINVAL, "projection_finish: done tracks the last kernel");
    RMT_HIP(launch_done(ctx, k_project_correct, rows_grid(ctx->nx, 0, ctx->ny), dim3(256), 0,
                        ctx->stream, done, a_star, b_star, (const double *)pc, p_prev, ctx->ny,
                        ctx->nx, divk_make(2 * dx), divk_make(2 * dy), dt / rho, bc_kind, lid, a,
                        b, p, 0, ctx->ny, (const double *)root, (double)n, dtp, rho, m2part,
                        sub_mean ? 0 : 1));
    // !sub_mean: the caller runs sub_mean_rows_upd(p, pc, root) later (the pressure update
    // and the mean removal in one deferred pass; pc and root stay untouched until then)
    return sub_mean ? sub_mean_rows(ctx, p, ctx->ny, ctx->nx) : RMT_OK;
}
int projection_dev(rmt_ctx *ctx, const double *a_star, const double *b_star, double dx,
                   double dy, const double *dtp, double rho, int bc_kind, double lid,
                   const double *p_prev, double *a, double *b, double *p, double *m2part) {
    RMT_CHECK(bc_kind >= 0 && bc_kind <= 3 && p_prev && rho > 0, RMT_EINVAL,
              "projection_dev: bad arguments");
    const long n = (long)ctx->ny * ctx->nx;
    RMT_TRY(ensure_scratch(ctx, 2 * n * sizeof(double)));
    double *rhs = ctx->scratch, *pc = rhs + n;
    RMT_TRY(divergence_full(ctx->stream, a_star, b_star, p_prev, ctx->ny, ctx->nx, 0.0,
                            rc_div(dx, dy), rhs, rho, 1.0, dtp));
    double *root = ctx->red + RED_BLOCKS + 17;
    RMT_TRY(dct_solve(ctx, rhs, dx, dy, pc, root));
    k_project_correct<<<rows_grid(ctx->nx, 0, ctx->ny), 256, 0, ctx->stream>>>(
        a_star, b_star, pc, p_prev, ctx->ny, ctx->nx, divk_make(2 * dx), divk_make(2 * dy), 0.0, bc_kind, lid, a, b, p, 0,
        ctx->ny, root, (double)n, dtp, rho, m2part);
    RMT_LAUNCHED();
    return sub_mean_rows(ctx, p, ctx->ny, ctx->nx);
}
}  // namespace rmt
