// diag.hip -- standalone drop-ins for the reference's per-step diagnostics and the blended
// momentum RHS (pyRMT/__init__.py:16, :28-31 exports):
//   compute_kinetic_energy        output.py:6-39
//   compute_strain_energy         output.py:41-134
//   compute_viscous_dissipation   output.py:136-193
//   velocity_rhs_blended_optimized functions.py:897-944
// The fused step computes the same energies inside k_diag_p1 (sim.hip) with a block-tree
// reduction; these entry points reproduce np.sum's own summation order instead (numpy's
// pairwise sum over 8192-element chunks, chunk sums added left to right: the order the
// oracle's rmto_pairwise_sum restates), so a density that is bit-exact gives a bit-exact
// energy.
#include "rmt_internal.hpp"
#include <vector>

namespace rmt {

constexpr int NP_CHUNK = 8192, NP_BLOCK = 128;

// numpy pairwise_sum (loops_utils.h.src) of a[0, n), n < NP_CHUNK: the recursion with an
// explicit stack (one thread)
__device__ double np_pairwise_serial(const double *a, long n) {
    struct Fr { long o, n; double left; int state; };
    Fr st[16];
    int sp = 0;
    st[0] = {0, n, 0.0, 0};
    double ret = 0.0;
    for (;;) {
        Fr &f = st[sp];
        if (f.state == 0) {
            if (f.n < 8) {
                double res = -0.0;
                for (long i = 0; i < f.n; ++i) res += a[f.o + i];
                ret = res;
            } else if (f.n <= NP_BLOCK) {
                double r[8];
                for (int k = 0; k < 8; ++k) r[k] = a[f.o + k];
                long i;
                for (i = 8; i < f.n - (f.n % 8); i += 8)
                    for (int k = 0; k < 8; ++k) r[k] += a[f.o + i + k];
                double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
                for (; i < f.n; ++i) res += a[f.o + i];
                ret = res;
            } else {
                long n2 = f.n / 2;
                n2 -= n2 % 8;
                f.state = 1;
                st[sp + 1] = {f.o, n2, 0.0, 0};
                ++sp;
                continue;
            }
        } else if (f.state == 1) {
            // left half returned in ret; now the right half
            long n2 = f.n / 2;
            n2 -= n2 % 8;
            f.left = ret;
            f.state = 2;
            st[sp + 1] = {f.o + n2, f.n - n2, 0.0, 0};
            ++sp;
            continue;
        } else {
            ret = f.left + ret;
        }
        if (sp == 0) return ret;
        --sp;
    }
}

// one wave per NP_CHUNK chunk: a full chunk is a perfect binary tree over 64 leaves of 128
// (8 running partials each), combined left + right level by level; a partial chunk (the
// last one) runs the general recursion on lane 0
__global__ void __launch_bounds__(64) k_np_pairwise(const double *__restrict__ x, long n,
                                                    double *__restrict__ part) {
    const long o = (long)blockIdx.x * NP_CHUNK;
    const long m = min((long)NP_CHUNK, n - o);
    const int lane = threadIdx.x;
    if (m < NP_CHUNK) {
        if (lane == 0) part[blockIdx.x] = np_pairwise_serial(x + o, m);
        return;
    }
    const double2 *a = (const double2 *)(x + o + (long)lane * NP_BLOCK);
    double r[8];
#pragma unroll
    for (int k = 0; k < 4; ++k) { const double2 t = a[k]; r[2 * k] = t.x; r[2 * k + 1] = t.y; }
#pragma unroll 4
    for (int i = 1; i < NP_BLOCK / 8; ++i)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const double2 t = a[4 * i + k];
            r[2 * k] += t.x; r[2 * k + 1] += t.y;
        }
    double v = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const double w = __shfl_down(v, d);
        if ((lane & (2 * d - 1)) == 0) v = v + w;
    }
    if (lane == 0) part[blockIdx.x] = v;
}

// np.sum(x) for n cells: chunk partials on the device, then `s += chunk` on the host
static int np_sum_host(rmt_ctx *ctx, const double *x, long n, double *out) {
    const long nch = (n + NP_CHUNK - 1) / NP_CHUNK;
    RMT_CHECK(n > 0, RMT_EINVAL, "np_sum: empty array");
    double *part = ctx->scratch + n;   // the density plane sits at ctx->scratch[0, n)
    k_np_pairwise<<<nch, 64, 0, ctx->stream>>>(x, n, part);
    RMT_LAUNCHED();
    std::vector<double> h(nch);
    RMT_HIP(hipMemcpyAsync(h.data(), part, nch * sizeof(double), hipMemcpyDeviceToHost,
                           ctx->stream));
    RMT_HIP(hipStreamSynchronize(ctx->stream));
    double s = 0.0;
    for (long k = 0; k < nch; ++k) s += h[k];
    *out = s;
    return RMT_OK;
}

// output.py:30-34: 0.5 * rho_local * (a**2 + b**2)
__global__ void k_ke_density(const double *__restrict__ a, const double *__restrict__ b,
                             const double *__restrict__ phi, long n, double rho_f, double rho_s,
                             double w_t, double *__restrict__ d) {
    const long c = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (c >= n) return;
    const double H = heaviside(phi[c], w_t);
    const double rho = (1 - H) * rho_s + H * rho_f;
    const double ac = a[c], bc = b[c];
    d[c] = 0.5 * rho * (ac * ac + bc * bc);
}

// output.py:66-129: edge-padded central gradients, W on phi <= 0 cells with |det G| > 1e-10
__global__ void k_se_density(const double *__restrict__ X1, const double *__restrict__ X2,
                             const double *__restrict__ phi, int ny, int nx, double dx, double dy,
                             double mu_s, double kappa, double *__restrict__ d) {
    const long c = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (c >= (long)ny * nx) return;
    const int j = (int)(c / nx), i = (int)(c % nx);
    d[c] = phi[c] <= 0.0 ? se_density(X1, X2, c, j, i, ny, nx, dx, dy, mu_s, kappa) : 0.0;
}

// output.py:168-188: 2 mu_local (D_xx^2 + D_yy^2 + 2 D_xy^2), one-sided grads at the edges
__global__ void k_diss_density(const double *__restrict__ a, const double *__restrict__ b,
                               const double *__restrict__ phi, int ny, int nx, double dx,
                               double dy, double mu_f, double eta_s, double w_t,
                               double *__restrict__ d) {
    const long c = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (c >= (long)ny * nx) return;
    const int j = (int)(c / nx), i = (int)(c % nx);
    const double h2x = 2 * dx, h2y = 2 * dy;
    const double dudx = grad2(a + c, 1, i, nx, h2x), dvdy = grad2(b + c, nx, j, ny, h2y);
    const double dxy = 0.5 * (grad2(a + c, nx, j, ny, h2y) + grad2(b + c, 1, i, nx, h2x));
    const double H = heaviside(phi[c], w_t);
    const double mu = H * mu_f + (1 - H) * eta_s;
    d[c] = 2.0 * mu * (dudx * dudx + dvdy * dvdy + 2.0 * (dxy * dxy));
}

// functions.py:906-921: the blended stress (no Kelvin-Voigt term: momentum_step_rk4 adds that
// to the elastic stress before calling, functions.py:717-735)
__global__ void k_vrhs_sigma(const double *__restrict__ u, const double *__restrict__ v,
                             const double *__restrict__ sxx, const double *__restrict__ sxy,
                             const double *__restrict__ syy, const double *__restrict__ H,
                             double mu_f, double dx, double dy, int ny, int nx,
                             double *__restrict__ gxx, double *__restrict__ gxy,
                             double *__restrict__ gyy) {
    const long c = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (c >= (long)ny * nx) return;
    const int j = (int)(c / nx), i = (int)(c % nx);
    const double h2x = 2 * dx, h2y = 2 * dy;
    const double dudx = grad2(u + c, 1, i, nx, h2x), dvdy = grad2(v + c, nx, j, ny, h2y);
    const double dudy = grad2(u + c, nx, j, ny, h2y), dvdx = grad2(v + c, 1, i, nx, h2x);
    const double h = H[c], omh = 1 - h;
    gxx[c] = h * (2 * mu_f * dudx) + omh * sxx[c];
    gyy[c] = h * (2 * mu_f * dvdy) + omh * syy[c];
    gxy[c] = h * (mu_f * (dudy + dvdx)) + omh * sxy[c];
}

// functions.py:923-944: divergence of the blended stress, upwind-3 advection, grad p; the
// surface-tension force is an array or (fx == nullptr) the scalar 0.0 of the gamma = 0 path
__global__ void k_vrhs(const double *__restrict__ u, const double *__restrict__ v,
                       const double *__restrict__ p, const double *__restrict__ gxx,
                       const double *__restrict__ gxy, const double *__restrict__ gyy,
                       const double *__restrict__ rho, const double *__restrict__ fx,
                       const double *__restrict__ fy, double dx, double dy, int ny, int nx,
                       double *__restrict__ ru, double *__restrict__ rv) {
    const long c = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (c >= (long)ny * nx) return;
    const int j = (int)(c / nx), i = (int)(c % nx);
    const double h2x = 2 * dx, h2y = 2 * dy;
    const double divx = grad2(gxx + c, 1, i, nx, h2x) + grad2(gxy + c, nx, j, ny, h2y);
    const double divy = grad2(gxy + c, 1, i, nx, h2x) + grad2(gyy + c, nx, j, ny, h2y);
    const double uc = u[c], vc = v[c];
    const double uadv = -uc * upwind3(u + c, 1, i, nx, uc, dx) - vc * upwind3(u + c, nx, j, ny, vc, dy);
    const double vadv = -uc * upwind3(v + c, 1, i, nx, uc, dx) - vc * upwind3(v + c, nx, j, ny, vc, dy);
    const double dpx = grad2(p + c, 1, i, nx, h2x), dpy = grad2(p + c, nx, j, ny, h2y);
    const double den = rho[c] + 1e-12;
    const double sx = fx ? fx[c] : 0.0, sy = fy ? fy[c] : 0.0;
    ru[c] = uadv + (divx + sx - dpx) / den;
    rv[c] = vadv + (divy + sy - dpy) / den;
}

}  // namespace rmt

using namespace rmt;

// output.py:195-211 divergence_2d_interior: central differences on [pad, N - pad)^2,
// (u[j, i+1] - u[j, i-1]) / (2dx) + (v[j+1, i] - v[j-1, i]) / (2dy); 0 elsewhere
__global__ void k_div_interior(const double *__restrict__ u, const double *__restrict__ v,
                               int ny, int nx, DivK Kx2, DivK Ky2, int pad,
                               double *__restrict__ out) {
    const long c = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (c >= (long)ny * nx) return;
    const int j = (int)(c / nx), i = (int)(c % nx);
    double d = 0.0;
    if (j >= pad && j < ny - pad && i >= pad && i < nx - pad)
        d = divk(u[c + 1] - u[c - 1], Kx2) + divk(v[c + nx] - v[c - nx], Ky2);
    out[c] = d;
}

extern "C" {

int rmt_divergence_2d_interior(rmt_ctx *ctx, const double *u, const double *v, double dx,
                               double dy, int pad, double *div) {
    RMT_CHECK(ctx && u && v && div, RMT_EINVAL, "null argument");
    RMT_CHECK(pad >= 1, RMT_EINVAL, "divergence_2d_interior: pad >= 1");
    const long n = (long)ctx->ny * ctx->nx;
    k_div_interior<<<grid1d(n, 256), 256, 0, ctx->stream>>>(u, v, ctx->ny, ctx->nx,
                                                              divk_make(2 * dx), divk_make(2 * dy),
                                                              pad, div);
    RMT_LAUNCHED();
    return RMT_OK;
}

int rmt_compute_kinetic_energy(rmt_ctx *ctx, const double *a, const double *b, double rho_f,
                               double rho_s, const double *phi, double w_t, double dx, double dy,
                               double *ke) {
    RMT_CHECK(ctx && a && b && phi && ke, RMT_EINVAL, "null argument");
    const long n = (long)ctx->ny * ctx->nx;
    RMT_TRY(ensure_scratch(ctx, (n + n / NP_CHUNK + 8) * sizeof(double)));
    k_ke_density<<<grid1d(n, 256), 256, 0, ctx->stream>>>(a, b, phi, n, rho_f, rho_s, w_t,
                                                          ctx->scratch);
    RMT_LAUNCHED();
    double s;
    RMT_TRY(np_sum_host(ctx, ctx->scratch, n, &s));
    *ke = s * dx * dy;
    return RMT_OK;
}

int rmt_compute_strain_energy(rmt_ctx *ctx, const double *X1, const double *X2, const double *phi,
                              double mu_s, double dx, double dy, double kappa, double *se) {
    RMT_CHECK(ctx && X1 && X2 && phi && se, RMT_EINVAL, "null argument");
    const long n = (long)ctx->ny * ctx->nx;
    RMT_TRY(ensure_scratch(ctx, (n + n / NP_CHUNK + 8) * sizeof(double)));
    k_se_density<<<grid1d(n, 256), 256, 0, ctx->stream>>>(X1, X2, phi, ctx->ny, ctx->nx, dx, dy,
                                                          mu_s, kappa, ctx->scratch);
    RMT_LAUNCHED();
    double s;
    RMT_TRY(np_sum_host(ctx, ctx->scratch, n, &s));
    *se = s * dx * dy;
    return RMT_OK;
}

int rmt_compute_viscous_dissipation(rmt_ctx *ctx, const double *a, const double *b, double mu_f,
                                    const double *phi, double w_t, double dx, double dy,
                                    double eta_s, double *diss) {
    RMT_CHECK(ctx && a && b && phi && diss, RMT_EINVAL, "null argument");
    RMT_CHECK(ctx->ny >= 3 && ctx->nx >= 3, RMT_EINVAL, "grid too small for the gradients");
    const long n = (long)ctx->ny * ctx->nx;
    RMT_TRY(ensure_scratch(ctx, (n + n / NP_CHUNK + 8) * sizeof(double)));
    k_diss_density<<<grid1d(n, 256), 256, 0, ctx->stream>>>(a, b, phi, ctx->ny, ctx->nx, dx, dy,
                                                            mu_f, eta_s, w_t, ctx->scratch);
    RMT_LAUNCHED();
    double s;
    RMT_TRY(np_sum_host(ctx, ctx->scratch, n, &s));
    *diss = s * dx * dy;
    return RMT_OK;
}

int rmt_velocity_rhs_blended(rmt_ctx *ctx, const double *u, const double *v, const double *p,
                             const double *sxx, const double *sxy, const double *syy, double dx,
                             double dy, double mu_f, const double *H, const double *rho,
                             const double *fx, const double *fy, double *rhs_u, double *rhs_v) {
    RMT_CHECK(ctx && u && v && p && sxx && sxy && syy && H && rho && rhs_u && rhs_v, RMT_EINVAL,
              "null argument");
    RMT_CHECK(!fx == !fy, RMT_EINVAL, "surface-tension force: both arrays or neither");
    RMT_CHECK(ctx->ny >= 5 && ctx->nx >= 5, RMT_EINVAL, "grid too small for the stencils");
    const int ny = ctx->ny, nx = ctx->nx;
    const long n = (long)ny * nx;
    RMT_TRY(ensure_scratch(ctx, 3 * n * sizeof(double)));
    double *g = ctx->scratch;
    k_vrhs_sigma<<<grid1d(n, 256), 256, 0, ctx->stream>>>(u, v, sxx, sxy, syy, H, mu_f, dx, dy,
                                                          ny, nx, g, g + n, g + 2 * n);
    k_vrhs<<<grid1d(n, 256), 256, 0, ctx->stream>>>(u, v, p, g, g + n, g + 2 * n, rho, fx, fy, dx,
                                                    dy, ny, nx, rhs_u, rhs_v);
    RMT_LAUNCHED();
    return RMT_OK;
}

}  // extern "C"
