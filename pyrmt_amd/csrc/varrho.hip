// varrho.hip -- the variable-density branch of pressure_projection_amg:
// functions.py:1296-1328 with the matrix-free operator of :1122-1168, preconditioned
// conjugate gradients with the DCT-I solve (poisson.hip) as the preconditioner.
//
//   rhs = divU_rc(rho) / dt - mean          functions.py:1016-1070 (per-face d_f), :1302-1303
//   CG (x0 = 0, ||r|| < rtol ||b||, maxiter) scipy.sparse.linalg.cg (scipy 1.15 algorithm)
//   p_c -= mean; a = a* - (dt / rho) dp_c/dx; BC; p = p_prev + p_c; p -= mean   :1326-1364
//
// The CG scalars (rho_k = r.z, p.q, alpha, beta) stay on the device; the host reads r.r once
// per iteration for the stopping test.  Dot products are deterministic two-pass reductions
// (fixed block partials, then one block), so a run is reproducible bit for bit; against
// NumPy / BLAS they agree to rounding, which is the parity bar of this branch.
#include "rmt_internal.hpp"
#include <algorithm>
#include <cmath>

namespace rmt {

constexpr int VR_BLOCKS = 1024, VR_T = 256;
enum { VS_RZ = 0, VS_RZ_PREV = 1, VS_PQ = 2, VS_ALPHA = 3, VS_BETA = 4, VS_RR = 5, VS_N = 8 };

// 1.0 / rho (functions.py:1305)
__global__ void k_vr_inv(const double *__restrict__ rho, long n, double *__restrict__ ir) {
    const long k = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (k < n) ir[k] = 1.0 / rho[k];
}

// functions.py:1016-1070 with variable rho: d_f per face = dt * 0.5 * (1/rho_l + 1/rho_r);
// writes divU, or divU / dt (over_dt: the projection's rhs, functions.py:1302)
__global__ void k_vr_div_rc(const double *__restrict__ a, const double *__restrict__ b,
                            const double *__restrict__ p, const double *__restrict__ ir, int ny,
                            int nx, double dt, double dx, double dy, int over_dt,
                            double *__restrict__ out) {
    const long c = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (c >= (long)ny * nx) return;
    const int j = (int)(c / nx), i = (int)(c % nx);
    if (j < 1 || j >= ny - 1 || i < 1 || i >= nx - 1) {
        out[c] = over_dt ? 0.0 / dt : 0.0;
        return;
    }
    const double h2x = 2.0 * dx, h2y = 2.0 * dy;
    const double gxl = grad2(p + c - 1, 1, i - 1, nx, h2x), gxc = grad2(p + c, 1, i, nx, h2x),
                 gxr = grad2(p + c + 1, 1, i + 1, nx, h2x);
    const double gyd = grad2(p + c - nx, nx, j - 1, ny, h2y), gyc = grad2(p + c, nx, j, ny, h2y),
                 gyu = grad2(p + c + nx, nx, j + 1, ny, h2y);
    const double hdt = dt * 0.5;
    const double fe = hdt * (ir[c] + ir[c + 1]), fw = hdt * (ir[c - 1] + ir[c]);
    const double fn = hdt * (ir[c] + ir[c + nx]), fs = hdt * (ir[c - nx] + ir[c]);
    const double ue = 0.5 * (a[c] + a[c + 1]) - fe * ((p[c + 1] - p[c]) / dx - 0.5 * (gxc + gxr));
    const double uw = 0.5 * (a[c - 1] + a[c]) - fw * ((p[c] - p[c - 1]) / dx - 0.5 * (gxl + gxc));
    const double vn = 0.5 * (b[c] + b[c + nx]) - fn * ((p[c + nx] - p[c]) / dy - 0.5 * (gyc + gyu));
    const double vs = 0.5 * (b[c - nx] + b[c]) - fs * ((p[c] - p[c - nx]) / dy - 0.5 * (gyd + gyc));
    const double d = (ue - uw) / dx + (vn - vs) / dy;
    out[c] = over_dt ? d / dt : d;
}

__global__ void k_vr_over(double *__restrict__ x, long n, double s) {
    const long k = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (k < n) x[k] = x[k] / s;
}

// functions.py:1122-1168 at one cell: div((1/rho) grad p) with face-averaged 1/rho and mirror
// ghosts (p[-1] = p[1], p[N] = p[N-2]; the same for 1/rho); result = (0 + x-part) + y-part
__device__ __forceinline__ double vr_apply(const double *__restrict__ p,
                                           const double *__restrict__ ir, long c, int j, int i,
                                           int ny, int nx, double cx, double cy) {
    const double pc = p[c], rc = ir[c];
    const long e = i + 1 < nx ? c + 1 : c - 1, w = i > 0 ? c - 1 : c + 1;
    const long nn = j + 1 < ny ? c + nx : c - nx, s = j > 0 ? c - nx : c + nx;
    const double be = 0.5 * (rc + ir[e]), bw = 0.5 * (ir[w] + rc);
    const double bn = 0.5 * (rc + ir[nn]), bs = 0.5 * (ir[s] + rc);
    double res = 0.0;
    res = res + cx * (be * (p[e] - pc) - bw * (pc - p[w]));
    res = res + cy * (bn * (p[nn] - pc) - bs * (pc - p[s]));
    return res;
}

// block partial of sum x*y (fixed grid: deterministic)
__device__ __forceinline__ void vr_block_sum(double v, double *part) {
    __shared__ double sh[VR_T];
    sh[threadIdx.x] = v;
    __syncthreads();
    for (int w = VR_T / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w) sh[threadIdx.x] += sh[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = sh[0];
}

// out = A p (the operator only, rmt_apply_variable_poisson) or q = A p and partials of p.q
__global__ void __launch_bounds__(VR_T) k_vr_apply(const double *__restrict__ p,
                                                   const double *__restrict__ ir, int ny, int nx,
                                                   double cx, double cy, double *__restrict__ q,
                                                   double *__restrict__ part) {
    double acc = 0.0;
    const long n = (long)ny * nx;
    for (long c = blockIdx.x * (long)VR_T + threadIdx.x; c < n; c += (long)gridDim.x * VR_T) {
        const double v = vr_apply(p, ir, c, (int)(c / nx), (int)(c % nx), ny, nx, cx, cy);
        q[c] = v;
        acc += p[c] * v;
    }
    if (part) vr_block_sum(acc, part);
}

__global__ void __launch_bounds__(VR_T) k_vr_dot(const double *__restrict__ x,
                                                 const double *__restrict__ y, long n,
                                                 double *__restrict__ part) {
    double acc = 0.0;
    for (long c = blockIdx.x * (long)VR_T + threadIdx.x; c < n; c += (long)gridDim.x * VR_T)
        acc += x[c] * y[c];
    vr_block_sum(acc, part);
}

// the final sum of the partials into sc[slot], then the derived scalar of that stage:
// slot VS_RZ: beta = rz / rz_prev (iteration > 0); VS_PQ: alpha = rz / pq;
// VS_RR: rz_prev = rz
__global__ void __launch_bounds__(VR_T) k_vr_final(const double *__restrict__ part, int slot,
                                                   int it, double *__restrict__ sc) {
    double acc = 0.0;
    for (int k = threadIdx.x; k < VR_BLOCKS; k += VR_T) acc += part[k];
    __shared__ double sh[VR_T];
    sh[threadIdx.x] = acc;
    __syncthreads();
    for (int w = VR_T / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w) sh[threadIdx.x] += sh[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x) return;
    const double s = sh[0];
    sc[slot] = s;
    if (slot == VS_RZ && it > 0) sc[VS_BETA] = s / sc[VS_RZ_PREV];
    if (slot == VS_PQ) sc[VS_ALPHA] = sc[VS_RZ] / s;
    if (slot == VS_RR) sc[VS_RZ_PREV] = sc[VS_RZ];
}

// p = z (first iteration) or p = p * beta + z  (p *= beta; p += z)
__global__ void k_vr_pdir(double *__restrict__ p, const double *__restrict__ z, long n,
                          const double *__restrict__ sc, int first) {
    const long k = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (k >= n) return;
    p[k] = first ? z[k] : p[k] * sc[VS_BETA] + z[k];
}

// x += alpha p; r -= alpha q; partials of r.r
__global__ void __launch_bounds__(VR_T) k_vr_xr(double *__restrict__ x, double *__restrict__ r,
                                                const double *__restrict__ p,
                                                const double *__restrict__ q, long n,
                                                const double *__restrict__ sc,
                                                double *__restrict__ part) {
    const double al = sc[VS_ALPHA];
    double acc = 0.0;
    for (long c = blockIdx.x * (long)VR_T + threadIdx.x; c < n; c += (long)gridDim.x * VR_T) {
        x[c] = x[c] + al * p[c];
        const double rv = r[c] - al * q[c];
        r[c] = rv;
        acc += rv * rv;
    }
    vr_block_sum(acc, part);
}

// a = a* - (dt / rho) dpc/dx at the BC source cell (functions.py:1350-1356), p = p_prev + pc
__global__ void k_vr_correct(const double *__restrict__ a_s, const double *__restrict__ b_s,
                             const double *__restrict__ pc, const double *__restrict__ p_prev,
                             const double *__restrict__ rho, int ny, int nx, double dx,
                             double dy, double dt, int bc, double lid, double *__restrict__ a,
                             double *__restrict__ b, double *__restrict__ p) {
    const long c = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (c >= (long)ny * nx) return;
    const int j = (int)(c / nx), i = (int)(c % nx);
    const BCSrc s = bc_source(bc, lid, j, i, ny, nx);
    double gx, gy;
    if (s.u_const) {
        a[c] = s.u_val;
    } else {
        const long q = s.u_src;
        pgrad_cell(pc, q, (int)(q / nx), (int)(q % nx), ny, nx, dx, dy, gx, gy);
        a[c] = a_s[q] - (dt / rho[q]) * gx;
    }
    if (s.v_const) {
        b[c] = s.v_val;
    } else {
        const long q = s.v_src;
        pgrad_cell(pc, q, (int)(q / nx), (int)(q % nx), ny, nx, dx, dy, gx, gy);
        b[c] = b_s[q] - (dt / rho[q]) * gy;
    }
    p[c] = p_prev ? p_prev[c] + pc[c] : pc[c];
}

}  // namespace rmt

using namespace rmt;

extern "C" {

int rmt_apply_variable_poisson(rmt_ctx *ctx, const double *p, double dx, double dy,
                               const double *inv_rho, double *out) {
    RMT_CHECK(ctx && p && inv_rho && out && ctx->ny >= 2 && ctx->nx >= 2, RMT_EINVAL,
              "bad argument");
    const int ny = ctx->ny, nx = ctx->nx;
    k_vr_apply<<<std::min<long>(VR_BLOCKS, grid1d((long)ny * nx, VR_T)), VR_T, 0, ctx->stream>>>(
        p, inv_rho, ny, nx, 1.0 / std::pow(dx, 2.0), 1.0 / std::pow(dy, 2.0), out, nullptr);
    RMT_LAUNCHED();
    return RMT_OK;
}

int rmt_divergence_rc_variable(rmt_ctx *ctx, const double *a, const double *b, const double *p,
                               double dt, const double *rho, double dx, double dy,
                               double *divU) {
    RMT_CHECK(ctx && a && b && p && rho && divU, RMT_EINVAL, "bad argument");
    const long n = (long)ctx->ny * ctx->nx;
    RMT_TRY(ensure_scratch(ctx, n * sizeof(double)));
    k_vr_inv<<<grid1d(n, 256), 256, 0, ctx->stream>>>(rho, n, ctx->scratch);
    k_vr_div_rc<<<grid1d(n, 256), 256, 0, ctx->stream>>>(a, b, p, ctx->scratch, ctx->ny, ctx->nx,
                                                         dt, dx, dy, 0, divU);
    RMT_LAUNCHED();
    return RMT_OK;
}

int rmt_pressure_projection_variable(rmt_ctx *ctx, const double *a_star, const double *b_star,
                                     double dx, double dy, double dt, const double *rho,
                                     int bc_kind, double lid, const double *p_prev, double rtol,
                                     int maxiter, double *a, double *b, double *p, int *iters) {
    RMT_CHECK(ctx && a_star && b_star && rho && a && b && p, RMT_EINVAL, "null argument");
    RMT_CHECK(bc_kind >= 0 && bc_kind <= 2, RMT_EINVAL, "unknown velocity bc kind");
    RMT_CHECK(maxiter >= 0, RMT_EINVAL, "maxiter < 0");
    const int ny = ctx->ny, nx = ctx->nx;
    const long n = (long)ny * nx;
    hipStream_t st = ctx->stream;
    // workspace: ir, rhs/r, x, z, dir, q, partials + scalars
    double *w = nullptr;
    RMT_HIP(hipMallocAsync((void **)&w, (6 * n + VR_BLOCKS + VS_N) * sizeof(double), st));
    double *ir = w, *r = w + n, *x = w + 2 * n, *z = w + 3 * n, *d = w + 4 * n, *q = w + 5 * n;
    double *part = w + 6 * n, *sc = part + VR_BLOCKS;
    const unsigned g = grid1d(n, 256), gr = VR_BLOCKS;   // reductions: every partial written
    int status = RMT_OK, it = 0;
    do {
        k_vr_inv<<<g, 256, 0, st>>>(rho, n, ir);
        if (p_prev) {
            k_vr_div_rc<<<g, 256, 0, st>>>(a_star, b_star, p_prev, ir, ny, nx, dt, dx, dy, 1, r);
        } else {
            if ((status = rmt_divergence_central(ctx, a_star, b_star, dx, dy, r))) break;
            k_vr_over<<<g, 256, 0, st>>>(r, n, dt);
        }
        if ((status = sub_mean_rows(ctx, r, ny, nx))) break;   // rhs -= mean(rhs)
        RMT_HIP(hipMemsetAsync(x, 0, n * sizeof(double), st));
        RMT_HIP(hipMemsetAsync(part, 0, VR_BLOCKS * sizeof(double), st));
        // ||b||: scipy's atol = rtol * ||b|| (x0 = 0, r = b)
        k_vr_dot<<<VR_BLOCKS, VR_T, 0, st>>>(r, r, n, part);
        k_vr_final<<<1, VR_T, 0, st>>>(part, VS_RR, 0, sc);
        double rr = 0.0;
        RMT_HIP(hipMemcpyAsync(&rr, sc + VS_RR, sizeof(double), hipMemcpyDeviceToHost, st));
        RMT_HIP(hipStreamSynchronize(st));
        const double bnrm = std::sqrt(rr), atol = rtol * bnrm;
        const double cx = 1.0 / std::pow(dx, 2.0), cy = 1.0 / std::pow(dy, 2.0);
        if (bnrm != 0.0) {
            for (it = 0; it < maxiter; ++it) {
                if (std::sqrt(rr) < atol) break;
                if ((status = dct_solve(ctx, r, dx, dy, z))) break;          // z = M r
                k_vr_dot<<<VR_BLOCKS, VR_T, 0, st>>>(r, z, n, part);
                k_vr_final<<<1, VR_T, 0, st>>>(part, VS_RZ, it, sc);
                k_vr_pdir<<<g, 256, 0, st>>>(d, z, n, sc, it == 0);
                k_vr_apply<<<gr, VR_T, 0, st>>>(d, ir, ny, nx, cx, cy, q, part);
                k_vr_final<<<1, VR_T, 0, st>>>(part, VS_PQ, it, sc);
                k_vr_xr<<<gr, VR_T, 0, st>>>(x, r, d, q, n, sc, part);
                k_vr_final<<<1, VR_T, 0, st>>>(part, VS_RR, it, sc);
                RMT_LAUNCHED();
                RMT_HIP(hipMemcpyAsync(&rr, sc + VS_RR, sizeof(double), hipMemcpyDeviceToHost,
                                       st));
                RMT_HIP(hipStreamSynchronize(st));
            }
            if (status) break;
        }
        // bnrm == 0: scipy returns b (all zeros) -- x is zero already
        if ((status = sub_mean_rows(ctx, x, ny, nx))) break;               // p_c -= mean
        k_vr_correct<<<g, 256, 0, st>>>(a_star, b_star, x, p_prev, rho, ny, nx, dx, dy, dt,
                                        bc_kind, lid, a, b, p);
        RMT_LAUNCHED();
        status = sub_mean_rows(ctx, p, ny, nx);
    } while (false);
    (void)hipFreeAsync(w, st);
    if (iters) *iters = it;
    if (!status) RMT_HIP(hipStreamSynchronize(st));
    return status;
}

}  // extern "C"
