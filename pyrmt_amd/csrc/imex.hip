// imex.hip -- the MAC IMEX tier: mac.py:243-369.
//
//   _lap_u_lid_hom / _lap_v_lid_hom   mac.py:243-260  homogeneous-BC ghost-cell Laplacians
//   _cg_helmholtz / _pcg_helmholtz    mac.py:263-316  (I - coef Lap_hom) x = rhs on the interior
//                                     faces, scipy.sparse.linalg.cg (scipy 1.15's algorithm,
//                                     x0 = rhs, atol = rtol ||rhs||), optional DST-II spectral
//                                     preconditioner (I - coef Lap_Dirichlet)^-1
//   momentum_predictor_lid_imex       mac.py:319-369  explicit central advection + forces,
//                                     implicit viscosity (+ trapezoidal elastic term), PCG
//
// Interior layouts: u-faces (ny, nx - 1) (face i = m + 1 of row j), v-faces (ny - 1, nx)
// (face row j = r + 1).  The per-face arithmetic follows the reference's NumPy expressions
// operand for operand (bit-exact operators); the CG dot products are deterministic two-pass
// reductions, so iterates agree with NumPy/BLAS to rounding.  The DST-II (ortho) of a row of
// M values is the imaginary part of a rotated length-2M complex FFT of its odd extension
// (rocFFT, batched over rows; the other axis through a transpose).
#include "rmt_internal.hpp"
#include <rocfft/rocfft.h>
#include <algorithm>
#include <cmath>
#include <vector>

namespace rmt {

constexpr int IM_BLOCKS = 1024, IM_T = 256;
enum { IS_RZ = 0, IS_RZ_PREV = 1, IS_PQ = 2, IS_ALPHA = 3, IS_BETA = 4, IS_RR = 5, IS_N = 8 };

// u-kind value at (j, i) of the full (ny, nx + 1) array, FULL: the array itself; else the
// interior array (ny, nx - 1) embedded with zero walls (i = 0, nx): mac.py:350 np.pad
template <bool FULL>
__device__ __forceinline__ double uval(const double *x, int j, int i, int nx) {
    if (FULL) return x[(long)j * (nx + 1) + i];
    return (i <= 0 || i >= nx) ? 0.0 : x[(long)j * (nx - 1) + (i - 1)];
}
// v-kind value at (j, i) of the full (ny + 1, nx) array or the interior (ny - 1, nx) one
// embedded with zero walls (j = 0, ny): mac.py:365
template <bool FULL>
__device__ __forceinline__ double vval(const double *x, int j, int i, int ny, int nx) {
    if (FULL) return x[(long)j * nx + i];
    return (j <= 0 || j >= ny) ? 0.0 : x[(long)(j - 1) * nx + i];
}

// mac.py:243-250 at interior u-face (j, i), i = 1 .. nx-1: ghost rows -u[0], -u[-1]
template <bool FULL>
__device__ __forceinline__ double lap_u(const double *x, int j, int i, int ny, int nx, double dx2,
                                        double dy2) {
    const double c = uval<FULL>(x, j, i, nx);
    const double n = j + 1 < ny ? uval<FULL>(x, j + 1, i, nx) : -uval<FULL>(x, ny - 1, i, nx);
    const double s = j >= 1 ? uval<FULL>(x, j - 1, i, nx) : -uval<FULL>(x, 0, i, nx);
    return (uval<FULL>(x, j, i + 1, nx) - 2 * c + uval<FULL>(x, j, i - 1, nx)) / dx2 +
           (n - 2 * c + s) / dy2;
}
// mac.py:253-260 at interior v-face (j, i), j = 1 .. ny-1: ghost cols -v[:, 0], -v[:, -1]
template <bool FULL>
__device__ __forceinline__ double lap_v(const double *x, int j, int i, int ny, int nx, double dx2,
                                        double dy2) {
    const double c = vval<FULL>(x, j, i, ny, nx);
    const double e = i + 1 < nx ? vval<FULL>(x, j, i + 1, ny, nx) : -vval<FULL>(x, j, nx - 1, ny, nx);
    const double w = i >= 1 ? vval<FULL>(x, j, i - 1, ny, nx) : -vval<FULL>(x, j, 0, ny, nx);
    return (e - 2 * c + w) / dx2 + (vval<FULL>(x, j + 1, i, ny, nx) - 2 * c +
                                    vval<FULL>(x, j - 1, i, ny, nx)) / dy2;
}

// interior element k of kind (0: u, 1: v) -> its face (j, i)
__device__ __forceinline__ void face_of(int kind, long k, int ny, int nx, int &j, int &i) {
    if (kind == 0) { j = (int)(k / (nx - 1)); i = (int)(k % (nx - 1)) + 1; }
    else { j = (int)(k / nx) + 1; i = (int)(k % nx); }
}

__global__ void k_im_lap_full(int kind, const double *__restrict__ f, int ny, int nx, double dx2,
                              double dy2, double *__restrict__ out) {
    const long n = kind == 0 ? (long)ny * (nx - 1) : (long)(ny - 1) * nx;
    const long k = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (k >= n) return;
    int j, i;
    face_of(kind, k, ny, nx, j, i);
    out[k] = kind == 0 ? lap_u<true>(f, j, i, ny, nx, dx2, dy2) : lap_v<true>(f, j, i, ny, nx, dx2, dy2);
}

// deterministic block partial of a per-thread sum into part[blockIdx.x]
__device__ __forceinline__ void im_block_sum(double acc, double *part) {
    __shared__ double sh[IM_T];
    sh[threadIdx.x] = acc;
    __syncthreads();
    for (int w = IM_T / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w) sh[threadIdx.x] += sh[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = sh[0];
}

// q = x - coef * Lap_hom(embed(x)) (mac.py:300-302); optional partials of x.q; R: q = b - q
// (the initial residual r = b - A x0)
__global__ void __launch_bounds__(IM_T) k_im_apply(int kind, const double *__restrict__ x,
                                                   int ny, int nx, double dx2, double dy2,
                                                   double coef, const double *__restrict__ b,
                                                   double *__restrict__ q,
                                                   double *__restrict__ part) {
    const long n = kind == 0 ? (long)ny * (nx - 1) : (long)(ny - 1) * nx;
    double acc = 0.0;
    for (long k = blockIdx.x * (long)IM_T + threadIdx.x; k < n; k += (long)gridDim.x * IM_T) {
        int j, i;
        face_of(kind, k, ny, nx, j, i);
        const double L = kind == 0 ? lap_u<false>(x, j, i, ny, nx, dx2, dy2)
                                   : lap_v<false>(x, j, i, ny, nx, dx2, dy2);
        const double a = x[k] - coef * L;
        q[k] = b ? b[k] - a : a;
        acc += x[k] * a;
    }
    if (part) im_block_sum(acc, part);
}

__global__ void __launch_bounds__(IM_T) k_im_dot(const double *__restrict__ x,
                                                 const double *__restrict__ y, long n,
                                                 double *__restrict__ part) {
    double acc = 0.0;
    for (long k = blockIdx.x * (long)IM_T + threadIdx.x; k < n; k += (long)gridDim.x * IM_T)
        acc += x[k] * y[k];
    im_block_sum(acc, part);
}

// the sum of the partials into sc[slot] and the CG scalar that stage derives (scipy 1.15
// cg: beta = rho_cur / rho_prev, alpha = rho_cur / p.q, rho_prev = rho_cur)
__global__ void __launch_bounds__(IM_T) k_im_final(const double *__restrict__ part, int slot,
                                                   int it, double *__restrict__ sc) {
    double acc = 0.0;
    for (int k = threadIdx.x; k < IM_BLOCKS; k += IM_T) acc += part[k];
    __shared__ double sh[IM_T];
    sh[threadIdx.x] = acc;
    __syncthreads();
    for (int w = IM_T / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w) sh[threadIdx.x] += sh[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x) return;
    const double s = sh[0];
    sc[slot] = s;
    if (slot == IS_RZ && it > 0) sc[IS_BETA] = s / sc[IS_RZ_PREV];
    if (slot == IS_PQ) sc[IS_ALPHA] = sc[IS_RZ] / s;
    if (slot == IS_RR) sc[IS_RZ_PREV] = sc[IS_RZ];
}

// p = z (first iteration) or p *= beta; p += z
__global__ void k_im_pdir(double *__restrict__ p, const double *__restrict__ z, long n,
                          const double *__restrict__ sc, int first) {
    const long k = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (k >= n) return;
    p[k] = first ? z[k] : p[k] * sc[IS_BETA] + z[k];
}

// x += alpha p; r -= alpha q; partials of r.r
__global__ void __launch_bounds__(IM_T) k_im_xr(double *__restrict__ x, double *__restrict__ r,
                                                const double *__restrict__ p,
                                                const double *__restrict__ q, long n,
                                                const double *__restrict__ sc,
                                                double *__restrict__ part) {
    const double al = sc[IS_ALPHA];
    double acc = 0.0;
    for (long k = blockIdx.x * (long)IM_T + threadIdx.x; k < n; k += (long)gridDim.x * IM_T) {
        x[k] = x[k] + al * p[k];
        const double rv = r[k] - al * q[k];
        r[k] = rv;
        acc += rv * rv;
    }
    im_block_sum(acc, part);
}

// ---------------------------------------------------------------- DST-II (ortho) ---
// forward, row of M: y_k = f_k * 2 sum_n x_n sin(pi (k+1)(2n+1) / 2M), f_k = sqrt(1/2M)
// (sqrt(1/4M) for k = M-1) = f_k * -Im(e^{-i pi (k+1)/2M} Z_{k+1}), Z = FFT_2M of the odd
// extension z = (x_0 .. x_{M-1}, -x_{M-1} .. -x_0)
__global__ void k_dst_pack_fwd(const double *__restrict__ x, int M, long rows,
                               double2 *__restrict__ z) {
    const long k = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (k >= rows * M) return;
    const long r = k / M;
    const int n = (int)(k % M);
    const double v = x[k];
    z[r * 2 * M + n] = make_double2(v, 0.0);
    z[r * 2 * M + 2 * M - 1 - n] = make_double2(-v, 0.0);
}
__global__ void k_dst_unpack_fwd(const double2 *__restrict__ Z, int M, long rows,
                                 const double2 *__restrict__ tw, double *__restrict__ y) {
    const long k = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (k >= rows * M) return;
    const long r = k / M;
    const int m = (int)(k % M) + 1;
    const double2 a = Z[r * 2 * M + m], w = tw[m];   // w = (cos, -sin)(pi m / 2M)
    const double im = a.y * w.x + a.x * w.y;
    const double f = m == M ? sqrt(1.0 / (4.0 * M)) : sqrt(1.0 / (2.0 * M));
    y[k] = -im * f;
}
// inverse (DST-III ortho, the transpose): x_n = sum_{m=1}^{M} a_m sin(pi m (2n+1) / 2M) with
// a_m = 2 f_{m-1} y_{m-1} = Im(sum_m b_m e^{+2 pi i m n / 2M}), b_m = a_m e^{+i pi m / 2M}
__global__ void k_dst_pack_inv(const double *__restrict__ y, int M, long rows,
                               const double2 *__restrict__ tw, double2 *__restrict__ b) {
    const long k = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (k >= rows * 2 * M) return;
    const long r = k / (2 * M);
    const int m = (int)(k % (2 * M));
    double2 o = make_double2(0.0, 0.0);
    if (m >= 1 && m <= M) {
        const double f = m == M ? sqrt(1.0 / (4.0 * M)) : sqrt(1.0 / (2.0 * M));
        const double a = 2.0 * f * y[r * M + m - 1];
        const double2 w = tw[m];
        o = make_double2(a * w.x, -a * w.y);
    }
    b[k] = o;
}
__global__ void k_dst_unpack_inv(const double2 *__restrict__ B, int M, long rows,
                                 double *__restrict__ x) {
    const long k = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (k >= rows * M) return;
    const long r = k / M;
    const int n = (int)(k % M);
    x[k] = B[r * 2 * M + n].y;
}
__global__ void k_im_div(double *__restrict__ x, const double *__restrict__ d, long n) {
    const long k = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (k < n) x[k] = x[k] / d[k];
}
__global__ void __launch_bounds__(256) k_im_transpose(const double *__restrict__ in, int R, int C,
                                                      double *__restrict__ out) {
    __shared__ double t[32][33];
    const int c0 = blockIdx.x * 32, r0 = blockIdx.y * 32, tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
    for (int rr = ty; rr < 32; rr += 8)
        if (r0 + rr < R && c0 + tx < C) t[rr][tx] = in[(long)(r0 + rr) * C + c0 + tx];
    __syncthreads();
    for (int cc = ty; cc < 32; cc += 8)
        if (c0 + cc < C && r0 + tx < R) out[(long)(c0 + cc) * R + r0 + tx] = t[tx][cc];
}

// rocFFT C2C plans of length 2M over `rows` rows, forward and backward, and the rotation table
struct DstAxis {
    int M = 0;
    long rows = 0;
    rocfft_plan fwd = nullptr, inv = nullptr;
    rocfft_execution_info info = nullptr;
    void *work = nullptr;
    size_t work_bytes = 0;
    double2 *tw = nullptr;   // (cos, -sin)(pi m / 2M), m = 0 .. M
};
struct ImexPlan {
    int ny = 0, nx = 0, kind = 0;
    double dx = 0, dy = 0, coef = 0;
    DstAxis ax[2];            // [0] along rows (length of a row), [1] along columns
    double *denom = nullptr;  // 1 - coef * lambda (mac.py:297-298), (rows, cols)
    double2 *buf = nullptr;   // 2M complex per row, the larger axis
    double *T = nullptr;      // transpose scratch
    std::vector<double> denom_h;   // host copy of denom (source of its async upload)
};

static bool g_rocfft = false;
static int rfok(rocfft_status s, const char *what) {
    if (s != rocfft_status_success) {
        set_error(std::string("rocFFT ") + what + " failed");
        return RMT_EDEVICE;
    }
    return RMT_OK;
}
static void axis_destroy(DstAxis &a) {
    if (a.fwd) rocfft_plan_destroy(a.fwd);
    if (a.inv) rocfft_plan_destroy(a.inv);
    if (a.info) rocfft_execution_info_destroy(a.info);
    (void)hipFree(a.work); (void)hipFree(a.tw);
    a = DstAxis{};
}
static int axis_make(DstAxis &a, int M, long rows) {
    a.M = M; a.rows = rows;
    const size_t len = 2 * (size_t)M;
    RMT_TRY(rfok(rocfft_plan_create(&a.fwd, rocfft_placement_inplace,
                                    rocfft_transform_type_complex_forward, rocfft_precision_double,
                                    1, &len, (size_t)rows, nullptr), "plan"));
    RMT_TRY(rfok(rocfft_plan_create(&a.inv, rocfft_placement_inplace,
                                    rocfft_transform_type_complex_inverse, rocfft_precision_double,
                                    1, &len, (size_t)rows, nullptr), "plan"));
    size_t w1 = 0, w2 = 0;
    rocfft_plan_get_work_buffer_size(a.fwd, &w1);
    rocfft_plan_get_work_buffer_size(a.inv, &w2);
    a.work_bytes = std::max(w1, w2);
    RMT_TRY(rfok(rocfft_execution_info_create(&a.info), "execution_info"));
    if (a.work_bytes) {
        RMT_HIP(hipMalloc(&a.work, a.work_bytes));
        RMT_TRY(rfok(rocfft_execution_info_set_work_buffer(a.info, a.work, a.work_bytes), "work"));
    }
    const long double PI = 3.141592653589793238462643383279502884L;
    std::vector<double2> h(M + 1);
    for (int m = 0; m <= M; ++m) {
        const long double t = PI * m / (2.0L * M);
        h[m] = make_double2((double)cosl(t), (double)-sinl(t));
    }
    RMT_HIP(hipMalloc(&a.tw, (M + 1) * sizeof(double2)));
    RMT_UPLOAD(a.tw, h.data(), (M + 1) * sizeof(double2));
    return RMT_OK;
}

// the plans live on the context (ctx->imex[kind], kind 0 u, 1 v), freed with it
static void plan_destroy(ImexPlan *P) {
    if (!P) return;
    axis_destroy(P->ax[0]); axis_destroy(P->ax[1]);
    (void)hipFree(P->denom); (void)hipFree(P->buf); (void)hipFree(P->T);
    delete P;
}
void imex_destroy(rmt_ctx *ctx) {
    for (auto &p : ctx->imex) { plan_destroy((ImexPlan *)p); p = nullptr; }
}

// the plan of kind for (ny, nx, dx, dy, coef); denom as mac.py:278-298 (np.cos -> cos)
static int imex_plan(rmt_ctx *ctx, int kind, int ny, int nx, double dx, double dy, double coef,
                     ImexPlan **out) {
    ImexPlan *P = (ImexPlan *)ctx->imex[kind];
    if (P && P->ny == ny && P->nx == nx && P->dx == dx && P->dy == dy && P->coef == coef) {
        *out = P;
        return RMT_OK;
    }
    if (!g_rocfft) { RMT_TRY(rfok(rocfft_setup(), "setup")); g_rocfft = true; }
    const bool keep = P && P->ny == ny && P->nx == nx;
    if (!keep) { plan_destroy(P); P = new ImexPlan; ctx->imex[kind] = P; }
    P->ny = ny; P->nx = nx; P->kind = kind; P->dx = dx; P->dy = dy; P->coef = coef;
    const int R = kind == 0 ? ny : ny - 1, C = kind == 0 ? nx - 1 : nx;   // interior shape
    if (!keep) {
        RMT_TRY(axis_make(P->ax[0], C, R));
        RMT_TRY(axis_make(P->ax[1], R, C));
        RMT_HIP(hipMalloc(&P->buf, 2 * (size_t)R * C * sizeof(double2)));
        RMT_HIP(hipMalloc(&P->T, (size_t)R * C * sizeof(double)));
        RMT_HIP(hipMalloc(&P->denom, (size_t)R * C * sizeof(double)));
    }
    // mac.py:278-284: lambda = ly[:, None] + lx[None, :], ly/lx = -2 (1 - cos(pi (k+1)/N)) / h**2
    std::vector<double> lx(C), ly(R);
    std::vector<double> &d = P->denom_h;   // kept: the async upload reads it
    d.assign((size_t)R * C, 0.0);
    const double dx2 = std::pow(dx, 2.0), dy2 = std::pow(dy, 2.0);
    for (int k = 0; k < C; ++k) lx[k] = -2.0 * (1.0 - std::cos(M_PI * (k + 1) / C)) / dx2;
    for (int k = 0; k < R; ++k) ly[k] = -2.0 * (1.0 - std::cos(M_PI * (k + 1) / R)) / dy2;
    for (int r = 0; r < R; ++r)
        for (int c = 0; c < C; ++c) d[(size_t)r * C + c] = 1.0 - coef * (ly[r] + lx[c]);
    RMT_HIP(hipMemcpyAsync(P->denom, d.data(), d.size() * sizeof(double), hipMemcpyHostToDevice,
                           ctx->stream));
    *out = P;
    return RMT_OK;
}

// in-place DST-II (inv = false) or its inverse along the rows of x (rows x M), ortho
static int dst_rows(hipStream_t st, DstAxis &a, double2 *buf, double *x, bool inv) {
    const long n = a.rows * a.M;
    RMT_TRY(rfok(rocfft_execution_info_set_stream(a.info, st), "stream"));
    void *bp[1] = {buf};
    if (!inv) {
        k_dst_pack_fwd<<<grid1d(n, 256), 256, 0, st>>>(x, a.M, a.rows, buf);
        RMT_TRY(rfok(rocfft_execute(a.fwd, bp, nullptr, a.info), "execute"));
        k_dst_unpack_fwd<<<grid1d(n, 256), 256, 0, st>>>(buf, a.M, a.rows, a.tw, x);
    } else {
        k_dst_pack_inv<<<grid1d(2 * n, 256), 256, 0, st>>>(x, a.M, a.rows, a.tw, buf);
        RMT_TRY(rfok(rocfft_execute(a.inv, bp, nullptr, a.info), "execute"));
        k_dst_unpack_inv<<<grid1d(n, 256), 256, 0, st>>>(buf, a.M, a.rows, x);
    }
    RMT_LAUNCHED();
    return RMT_OK;
}
static void im_transpose(hipStream_t st, const double *in, int R, int C, double *out) {
    k_im_transpose<<<dim3((C + 31) / 32, (R + 31) / 32), 256, 0, st>>>(in, R, C, out);
}

// z = idstn(dstn(r, 2, ortho) / denom, 2, ortho) (mac.py:304-306), R x C
static int dst_precond(hipStream_t st, ImexPlan *P, const double *r, double *z) {
    const int R = P->ax[1].M, C = P->ax[0].M;
    const long n = (long)R * C;
    RMT_HIP(hipMemcpyAsync(z, r, n * sizeof(double), hipMemcpyDeviceToDevice, st));
    RMT_TRY(dst_rows(st, P->ax[0], P->buf, z, false));            // along x (rows of C)
    im_transpose(st, z, R, C, P->T);
    RMT_TRY(dst_rows(st, P->ax[1], P->buf, P->T, false));         // along y
    im_transpose(st, P->T, C, R, z);
    k_im_div<<<grid1d(n, 256), 256, 0, st>>>(z, P->denom, n);
    im_transpose(st, z, R, C, P->T);
    RMT_TRY(dst_rows(st, P->ax[1], P->buf, P->T, true));
    im_transpose(st, P->T, C, R, z);
    RMT_TRY(dst_rows(st, P->ax[0], P->buf, z, true));
    RMT_LAUNCHED();
    return RMT_OK;
}

// scipy.sparse.linalg.cg (scipy 1.15) for (I - coef Lap_hom) x = b, x0 = b, atol = rtol ||b||,
// optional M = the DST preconditioner; iters = the loop iterations run (callback count)
static int helmholtz(rmt_ctx *ctx, int kind, const double *b, double coef, double dx, double dy,
                     double rtol, int maxiter, int precond, double *x, int *iters) {
    const int ny = ctx->ny, nx = ctx->nx;
    const long n = kind == 0 ? (long)ny * (nx - 1) : (long)(ny - 1) * nx;
    hipStream_t st = ctx->stream;
    ImexPlan *P = nullptr;
    if (precond) RMT_TRY(imex_plan(ctx, kind, ny, nx, dx, dy, coef, &P));
    const double dx2 = std::pow(dx, 2.0), dy2 = std::pow(dy, 2.0);
    double *w = nullptr;
    RMT_HIP(hipMallocAsync((void **)&w, (4 * n + IM_BLOCKS + IS_N) * sizeof(double), st));
    double *r = w, *z = w + n, *d = w + 2 * n, *q = w + 3 * n, *part = w + 4 * n;
    double *sc = part + IM_BLOCKS;
    int status = RMT_OK, it = 0;
    do {
        RMT_HIP(hipMemcpyAsync(x, b, n * sizeof(double), hipMemcpyDeviceToDevice, st));
        RMT_HIP(hipMemsetAsync(part, 0, IM_BLOCKS * sizeof(double), st));
        k_im_dot<<<IM_BLOCKS, IM_T, 0, st>>>(b, b, n, part);
        k_im_final<<<1, IM_T, 0, st>>>(part, IS_RR, 0, sc);
        double rr = 0.0;
        RMT_HIP(hipMemcpyAsync(&rr, sc + IS_RR, sizeof(double), hipMemcpyDeviceToHost, st));
        RMT_HIP(hipStreamSynchronize(st));
        const double bnrm = std::sqrt(rr), atol = rtol * bnrm;
        if (bnrm == 0.0) break;   // scipy returns b (x = b already)
        // r = b - A x0 (x0 = b is non-zero here), and r.r for the first stopping test
        k_im_apply<<<IM_BLOCKS, IM_T, 0, st>>>(kind, x, ny, nx, dx2, dy2, coef, b, r, nullptr);
        k_im_dot<<<IM_BLOCKS, IM_T, 0, st>>>(r, r, n, part);
        k_im_final<<<1, IM_T, 0, st>>>(part, IS_RR, 0, sc);
        RMT_HIP(hipMemcpyAsync(&rr, sc + IS_RR, sizeof(double), hipMemcpyDeviceToHost, st));
        RMT_HIP(hipStreamSynchronize(st));
        for (it = 0; it < maxiter; ++it) {
            if (std::sqrt(rr) < atol) break;
            if (precond) { if ((status = dst_precond(st, P, r, z))) break; }
            const double *zz = precond ? z : r;                          // z = M r
            k_im_dot<<<IM_BLOCKS, IM_T, 0, st>>>(r, zz, n, part);
            k_im_final<<<1, IM_T, 0, st>>>(part, IS_RZ, it, sc);
            k_im_pdir<<<grid1d(n, 256), 256, 0, st>>>(d, zz, n, sc, it == 0);
            k_im_apply<<<IM_BLOCKS, IM_T, 0, st>>>(kind, d, ny, nx, dx2, dy2, coef, nullptr, q,
                                                   part);
            k_im_final<<<1, IM_T, 0, st>>>(part, IS_PQ, it, sc);
            k_im_xr<<<IM_BLOCKS, IM_T, 0, st>>>(x, r, d, q, n, sc, part);
            k_im_final<<<1, IM_T, 0, st>>>(part, IS_RR, it, sc);
            RMT_LAUNCHED();
            RMT_HIP(hipMemcpyAsync(&rr, sc + IS_RR, sizeof(double), hipMemcpyDeviceToHost, st));
            RMT_HIP(hipStreamSynchronize(st));
        }
    } while (false);
    (void)hipFreeAsync(w, st);
    if (iters) *iters = it;
    if (!status) RMT_HIP(hipStreamSynchronize(st));
    return status;
}

// mac.py:339-349 (u) / 355-364 (v): the right-hand side on the interior faces
__global__ void k_im_rhs(int kind, const double *__restrict__ u, const double *__restrict__ v,
                         int ny, int nx, double dx, double dy, double dt, double U_lid,
                         const double *__restrict__ f, double rho, double c_el, double dx2,
                         double dy2, double lid_term, double *__restrict__ rhs) {
    const long n = kind == 0 ? (long)ny * (nx - 1) : (long)(ny - 1) * nx;
    const long k = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (k >= n) return;
    int j, i;
    face_of(kind, k, ny, nx, j, i);
    const long U = nx + 1;   // u row length
    double r;
    if (kind == 0) {
        const double uc = u[j * U + i];
        const double dudx = (u[j * U + i + 1] - u[j * U + i - 1]) / (2 * dx);
        // _u_ghost_y: bottom ghost -u[0], top ghost 2 U_lid - u[-1]
        const double un = j + 1 < ny ? u[(j + 1) * U + i] : 2.0 * U_lid - u[(ny - 1) * U + i];
        const double us = j >= 1 ? u[(j - 1) * U + i] : -u[i];
        const double dudy = (un - us) / (2 * dy);
        // _v_at_u: 0.25 (v[j, i-1] + v[j, i] + v[j+1, i-1] + v[j+1, i])
        const double vu = 0.25 * (v[(long)j * nx + i - 1] + v[(long)j * nx + i] +
                                  v[(long)(j + 1) * nx + i - 1] + v[(long)(j + 1) * nx + i]);
        r = uc + dt * (-(uc * dudx + vu * dudy));
        if (f) r = r + dt * f[j * U + i] / rho;
        if (c_el > 0.0) r = r + c_el * lap_u<true>(u, j, i, ny, nx, dx2, dy2);
        if (j == ny - 1) r += lid_term;
    } else {
        const double vc = v[(long)j * nx + i];
        const double dvdy = (v[(long)(j + 1) * nx + i] - v[(long)(j - 1) * nx + i]) / (2 * dy);
        // _v_ghost_x: ghost cols -v[:, 0], -v[:, -1]
        const double ve = i + 1 < nx ? v[(long)j * nx + i + 1] : -v[(long)j * nx + nx - 1];
        const double vw = i >= 1 ? v[(long)j * nx + i - 1] : -v[(long)j * nx];
        const double dvdx = (ve - vw) / (2 * dx);
        // _u_at_v: 0.25 (u[j-1, i] + u[j-1, i+1] + u[j, i] + u[j, i+1])
        const double uv = 0.25 * (u[(j - 1) * U + i] + u[(j - 1) * U + i + 1] + u[j * U + i] +
                                  u[j * U + i + 1]);
        r = vc + dt * (-(uv * dvdx + vc * dvdy));
        if (f) r = r + dt * f[(long)j * nx + i] / rho;
        if (c_el > 0.0) r = r + c_el * lap_v<true>(v, j, i, ny, nx, dx2, dy2);
    }
    rhs[k] = r;
}

// ustar = u with the interior faces from the solve and the wall faces zero (mac.py:353, 368)
__global__ void k_im_scatter(int kind, const double *__restrict__ sol, int ny, int nx,
                             double *__restrict__ out) {
    const long n = kind == 0 ? (long)ny * (nx + 1) : (long)(ny + 1) * nx;
    const long k = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (k >= n) return;
    if (kind == 0) {
        const int j = (int)(k / (nx + 1)), i = (int)(k % (nx + 1));
        out[k] = (i == 0 || i == nx) ? 0.0 : sol[(long)j * (nx - 1) + i - 1];
    } else {
        const int j = (int)(k / nx), i = (int)(k % nx);
        out[k] = (j == 0 || j == ny) ? 0.0 : sol[(long)(j - 1) * nx + i];
    }
}


// ------------------------------------------------- semi-Lagrangian branch (mac.py:381-442) --
// scipy.ndimage.map_coordinates(f, [jq, iq], order=3, mode='nearest') (mac.py:374-378) as
// scipy 1.15 computes it: f edge-padded by 12 (_prepad_for_spline_filter), the cubic
// B-spline prefilter along axis 0 then axis 1 (gain 6, pole sqrt(3) - 2, the 'reflect'
// causal / anticausal initialisation scipy uses for 'nearest'), then the 4 x 4 tap spline
// sum at (jq + 12, iq + 12) with the taps clamped to the padded array.
constexpr int SPL_PAD = 12;

__global__ void k_spl_pad(const double *__restrict__ f, int R, int C, double *__restrict__ o) {
    const int P = R + 2 * SPL_PAD, Q = C + 2 * SPL_PAD;
    const long k = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (k >= (long)P * Q) return;
    const int a = (int)(k / Q), b = (int)(k % Q);
    const int j = min(max(a - SPL_PAD, 0), R - 1), i = min(max(b - SPL_PAD, 0), C - 1);
    o[k] = f[(long)j * C + i];
}
// in-place cubic B-spline prefilter of the line c[0], c[s], ..., c[(n-1) s]
__device__ void spl_line(double *c, int n, long s) {
    const double z = sqrt(3.0) - 2.0;
    for (int k = 0; k < n; ++k) c[k * s] *= 6.0;
    // causal init ('reflect')
    double zi = z;
    const double zn = pow(z, (double)n), c0 = c[0];
    double a = c[0] + zn * c[(n - 1) * s];
    for (int k = 1; k < n; ++k) {
        a += zi * (c[k * s] + zn * c[(n - 1 - k) * s]);
        zi *= z;
    }
    a *= z / (1.0 - zn * zn);
    c[0] = a + c0;
    for (int k = 1; k < n; ++k) c[k * s] += z * c[(k - 1) * s];
    c[(n - 1) * s] *= z / (z - 1.0);
    for (int k = n - 2; k >= 0; --k) c[k * s] = z * (c[(k + 1) * s] - c[k * s]);
}
__global__ void k_spl_cols(double *__restrict__ c, int P, int Q) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < Q) spl_line(c + i, P, Q);
}
__global__ void k_spl_rows(double *__restrict__ c, int P, int Q) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < P) spl_line(c + (long)j * Q, Q, 1);
}
// the spline value at index coordinates (jq, iq) of the unpadded field (R x C)
__device__ double spl_eval(const double *__restrict__ c, int R, int C, double jq, double iq) {
    const int P = R + 2 * SPL_PAD, Q = C + 2 * SPL_PAD;
    const double tj = jq + SPL_PAD, ti = iq + SPL_PAD;
    const double fj = floor(tj), fi = floor(ti);
    double wj[4], wi[4];
    {
        const double y = tj - fj, z = 1.0 - y;
        wj[0] = z * z * z / 6.0; wj[1] = (y * y * (y - 2.0) * 3.0 + 4.0) / 6.0;
        wj[2] = (z * z * (z - 2.0) * 3.0 + 4.0) / 6.0; wj[3] = y * y * y / 6.0;
    }
    {
        const double y = ti - fi, z = 1.0 - y;
        wi[0] = z * z * z / 6.0; wi[1] = (y * y * (y - 2.0) * 3.0 + 4.0) / 6.0;
        wi[2] = (z * z * (z - 2.0) * 3.0 + 4.0) / 6.0; wi[3] = y * y * y / 6.0;
    }
    // a NaN / huge coordinate: clamp the base index (the weights carry the NaN)
    const double bj = fmin(fmax(fj, -4.0), (double)P), bi = fmin(fmax(fi, -4.0), (double)Q);
    const int j0 = (int)bj - 1, i0 = (int)bi - 1;
    double s = 0.0;
    for (int a = 0; a < 4; ++a) {
        const long row = (long)min(max(j0 + a, 0), P - 1) * Q;
        double r = 0.0;
        for (int b = 0; b < 4; ++b) r += wi[b] * c[row + min(max(i0 + b, 0), Q - 1)];
        s += wj[a] * r;
    }
    return s;
}
struct SplFields {           // prefiltered coefficients (padded) of the four grids
    const double *u, *v, *up, *vp;
};
// mac.py:395-405 (u faces) / 407-417 (v faces): midpoint backtrace and the departure value,
// written as the interior array (the implicit solve's rhs before forces)
__global__ void k_sl_faces(int kind, const double *__restrict__ u, const double *__restrict__ v,
                           SplFields S, int ny, int nx, double dx, double dy, double dt,
                           double *__restrict__ out) {
    const long n = kind == 0 ? (long)ny * (nx - 1) : (long)(ny - 1) * nx;
    const long k = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (k >= n) return;
    int j, i;
    face_of(kind, k, ny, nx, j, i);
    const long U = nx + 1;
    if (kind == 0) {
        const double xf = i * dx, yf = (j + 0.5) * dy;
        const double velx = u[j * U + i];
        const double vely = 0.25 * (v[(long)j * nx + i - 1] + v[(long)j * nx + i] +
                                    v[(long)(j + 1) * nx + i - 1] + v[(long)(j + 1) * nx + i]);
        const double xm = xf - 0.5 * dt * velx, ym = yf - 0.5 * dt * vely;
        const double vxm = spl_eval(S.u, ny, nx + 1, ym / dy, xm / dx);
        const double vym = spl_eval(S.vp, ny + 1, nx + 2, ym / dy - 0.0, xm / dx + 0.5);
        const double xd = xf - dt * vxm, yd = yf - dt * vym;
        out[k] = spl_eval(S.up, ny + 2, nx + 1, yd / dy + 0.5, xd / dx);
    } else {
        const double xf = (i + 0.5) * dx, yf = j * dy;
        const double velx = 0.25 * (u[(j - 1) * U + i] + u[(j - 1) * U + i + 1] + u[j * U + i] +
                                    u[j * U + i + 1]);
        const double vely = v[(long)j * nx + i];
        const double xm = xf - 0.5 * dt * velx, ym = yf - 0.5 * dt * vely;
        const double vxm = spl_eval(S.up, ny + 2, nx + 1, ym / dy + 0.5, xm / dx);
        const double vym = spl_eval(S.v, ny + 1, nx, ym / dy, xm / dx - 0.5);
        const double xd = xf - dt * vxm, yd = yf - dt * vym;
        out[k] = spl_eval(S.vp, ny + 1, nx + 2, yd / dy, xd / dx + 0.5);
    }
}
// mac.py:420-440: rhs = advected interior (+ dt f / rho) (+ c_el Lap_hom(u^n)) (+ lid term)
__global__ void k_sl_rhs(int kind, const double *f0, const double *__restrict__ full,
                         const double *__restrict__ f, int ny, int nx, double dt, double rho,
                         double c_el, double dx2, double dy2, double lid_term, double *rhs) {
    const long n = kind == 0 ? (long)ny * (nx - 1) : (long)(ny - 1) * nx;
    const long k = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (k >= n) return;
    int j, i;
    face_of(kind, k, ny, nx, j, i);
    double r = f0[k];
    if (kind == 0) {
        if (f) r = r + dt * f[(long)j * (nx + 1) + i] / rho;
        if (c_el > 0.0) r = r + c_el * lap_u<true>(full, j, i, ny, nx, dx2, dy2);
        if (j == ny - 1) r += lid_term;
    } else {
        if (f) r = r + dt * f[(long)j * nx + i] / rho;
        if (c_el > 0.0) r = r + c_el * lap_v<true>(full, j, i, ny, nx, dx2, dy2);
    }
    rhs[k] = r;
}
// _u_ghost_y / _v_ghost_x (mac.py:147-165)
__global__ void k_ghosts(const double *__restrict__ u, const double *__restrict__ v, int ny,
                         int nx, double U_lid, double *__restrict__ up, double *__restrict__ vp) {
    const long nu = (long)(ny + 2) * (nx + 1), nvp = (long)(ny + 1) * (nx + 2);
    const long k = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (k < nu) {
        const int r = (int)(k / (nx + 1)), i = (int)(k % (nx + 1));
        up[k] = r == 0 ? -u[i] : r == ny + 1 ? 2.0 * U_lid - u[(long)(ny - 1) * (nx + 1) + i]
                                             : u[(long)(r - 1) * (nx + 1) + i];
    }
    if (k < nvp) {
        const int j = (int)(k / (nx + 2)), c = (int)(k % (nx + 2));
        vp[k] = c == 0 ? -v[(long)j * nx] : c == nx + 1 ? -v[(long)j * nx + nx - 1]
                                                        : v[(long)j * nx + c - 1];
    }
}

}  // namespace rmt

using namespace rmt;

extern "C" {

int rmt_mac_lap_lid_hom(rmt_ctx *ctx, int kind, const double *f, double dx, double dy,
                        double *out) {
    RMT_CHECK(ctx && f && out && (kind == 0 || kind == 1) && ctx->ny >= 2 && ctx->nx >= 2,
              RMT_EINVAL, "bad argument");
    const int ny = ctx->ny, nx = ctx->nx;
    const long n = kind == 0 ? (long)ny * (nx - 1) : (long)(ny - 1) * nx;
    k_im_lap_full<<<grid1d(n, 256), 256, 0, ctx->stream>>>(kind, f, ny, nx, std::pow(dx, 2.0),
                                                           std::pow(dy, 2.0), out);
    RMT_LAUNCHED();
    return RMT_OK;
}

int rmt_mac_helmholtz(rmt_ctx *ctx, int kind, const double *rhs, double coef, double dx,
                      double dy, double rtol, int maxiter, int precond, double *x, int *iters) {
    RMT_CHECK(ctx && rhs && x && (kind == 0 || kind == 1) && ctx->ny >= 2 && ctx->nx >= 2,
              RMT_EINVAL, "bad argument");
    RMT_CHECK(maxiter >= 0 && coef >= 0.0, RMT_EINVAL, "maxiter < 0 or coef < 0");
    return helmholtz(ctx, kind, rhs, coef, dx, dy, rtol, maxiter, precond, x, iters);
}

int rmt_mac_momentum_predictor_lid_imex(rmt_ctx *ctx, const double *u, const double *v,
                                        double nu, double dx, double dy, double dt,
                                        double U_lid, const double *fu, const double *fv,
                                        double rho, double rtol, double cs2, double *ustar,
                                        double *vstar, int *iters) {
    RMT_CHECK(ctx && u && v && ustar && vstar && ctx->ny >= 2 && ctx->nx >= 2, RMT_EINVAL,
              "bad argument");
    const int ny = ctx->ny, nx = ctx->nx;
    const long nu_i = (long)ny * (nx - 1), nv_i = (long)(ny - 1) * nx;
    hipStream_t st = ctx->stream;
    // mac.py:336-337 (Python float arithmetic, as scalars)
    const double c_el = 0.25 * dt * dt * cs2, coef = dt * nu + c_el;
    const double dx2 = std::pow(dx, 2.0), dy2 = std::pow(dy, 2.0);
    const double lid_term = coef * (2.0 * U_lid / dy2);
    double *w = nullptr;
    RMT_HIP(hipMallocAsync((void **)&w, 2 * (nu_i + nv_i) * sizeof(double), st));
    double *ru = w, *rv = w + nu_i, *xu = w + nu_i + nv_i, *xv = xu + nu_i;
    int status = RMT_OK, it[2] = {0, 0};
    do {
        k_im_rhs<<<grid1d(nu_i, 256), 256, 0, st>>>(0, u, v, ny, nx, dx, dy, dt, U_lid, fu, rho,
                                                    c_el, dx2, dy2, lid_term, ru);
        k_im_rhs<<<grid1d(nv_i, 256), 256, 0, st>>>(1, u, v, ny, nx, dx, dy, dt, U_lid, fv, rho,
                                                    c_el, dx2, dy2, 0.0, rv);
        RMT_LAUNCHED();
        if ((status = helmholtz(ctx, 0, ru, coef, dx, dy, rtol, 500, 1, xu, &it[0]))) break;
        if ((status = helmholtz(ctx, 1, rv, coef, dx, dy, rtol, 500, 1, xv, &it[1]))) break;
        k_im_scatter<<<grid1d((long)ny * (nx + 1), 256), 256, 0, st>>>(0, xu, ny, nx, ustar);
        k_im_scatter<<<grid1d((long)(ny + 1) * nx, 256), 256, 0, st>>>(1, xv, ny, nx, vstar);
        RMT_LAUNCHED();
    } while (false);
    (void)hipFreeAsync(w, st);
    if (iters) { iters[0] = it[0]; iters[1] = it[1]; }
    if (!status) RMT_HIP(hipStreamSynchronize(st));
    return status;
}

// mac.py:381-442 semi-Lagrangian branch (the caller took it: CFL > cfl_switch)
int rmt_mac_momentum_predictor_lid_semilag(rmt_ctx *ctx, const double *u, const double *v,
                                           double nu, double dx, double dy, double dt,
                                           double U_lid, const double *fu, const double *fv,
                                           double rho, double cs2, double rtol, double *ustar,
                                           double *vstar, int *iters) {
    RMT_CHECK(ctx && u && v && ustar && vstar && ctx->ny >= 2 && ctx->nx >= 2, RMT_EINVAL,
              "bad argument");
    const int ny = ctx->ny, nx = ctx->nx;
    const long nu_i = (long)ny * (nx - 1), nv_i = (long)(ny - 1) * nx;
    hipStream_t st = ctx->stream;
    const double c_el = 0.25 * dt * dt * cs2, coef = dt * nu + c_el;
    const double dx2 = std::pow(dx, 2.0), dy2 = std::pow(dy, 2.0);
    const double lid_term = coef * (2.0 * U_lid / dy2);
    const int R[4] = {ny, ny + 1, ny + 2, ny + 1}, C[4] = {nx + 1, nx, nx + 1, nx + 2};
    long off[5] = {0};
    for (int q = 0; q < 4; ++q) off[q + 1] = off[q] + (long)(R[q] + 2 * SPL_PAD) * (C[q] + 2 * SPL_PAD);
    const long ng = (long)(ny + 2) * (nx + 1) + (long)(ny + 1) * (nx + 2);
    double *w = nullptr;
    RMT_HIP(hipMallocAsync((void **)&w, (off[4] + ng + 2 * (nu_i + nv_i)) * sizeof(double), st));
    double *up = w + off[4], *vp = up + (long)(ny + 2) * (nx + 1);
    double *au = w + off[4] + ng, *av = au + nu_i, *xu = av + nv_i, *xv = xu + nu_i;
    int status = RMT_OK, it[2] = {0, 0};
    do {
        k_ghosts<<<grid1d(std::max((long)(ny + 2) * (nx + 1), (long)(ny + 1) * (nx + 2)), 256), 256, 0,
                   st>>>(u, v, ny, nx, U_lid, up, vp);
        const double *src[4] = {u, v, up, vp};
        for (int q = 0; q < 4; ++q) {
            const int P = R[q] + 2 * SPL_PAD, Q = C[q] + 2 * SPL_PAD;
            k_spl_pad<<<grid1d((long)P * Q, 256), 256, 0, st>>>(src[q], R[q], C[q], w + off[q]);
            k_spl_cols<<<grid1d(Q, 64), 64, 0, st>>>(w + off[q], P, Q);
            k_spl_rows<<<grid1d(P, 64), 64, 0, st>>>(w + off[q], P, Q);
        }
        const SplFields S{w + off[0], w + off[1], w + off[2], w + off[3]};
        k_sl_faces<<<grid1d(nu_i, 256), 256, 0, st>>>(0, u, v, S, ny, nx, dx, dy, dt, au);
        k_sl_faces<<<grid1d(nv_i, 256), 256, 0, st>>>(1, u, v, S, ny, nx, dx, dy, dt, av);
        k_sl_rhs<<<grid1d(nu_i, 256), 256, 0, st>>>(0, au, u, fu, ny, nx, dt, rho, c_el, dx2, dy2,
                                                   lid_term, au);
        k_sl_rhs<<<grid1d(nv_i, 256), 256, 0, st>>>(1, av, v, fv, ny, nx, dt, rho, c_el, dx2, dy2,
                                                   0.0, av);
        RMT_LAUNCHED();
        if ((status = helmholtz(ctx, 0, au, coef, dx, dy, rtol, 500, 1, xu, &it[0]))) break;
        if ((status = helmholtz(ctx, 1, av, coef, dx, dy, rtol, 500, 1, xv, &it[1]))) break;
        k_im_scatter<<<grid1d((long)ny * (nx + 1), 256), 256, 0, st>>>(0, xu, ny, nx, ustar);
        k_im_scatter<<<grid1d((long)(ny + 1) * nx, 256), 256, 0, st>>>(1, xv, ny, nx, vstar);
        RMT_LAUNCHED();
    } while (false);
    (void)hipFreeAsync(w, st);
    if (iters) { iters[0] = it[0]; iters[1] = it[1]; }
    if (!status) RMT_HIP(hipStreamSynchronize(st));
    return status;
}

}  // extern "C"
