// mac.hip -- the staggered (MAC) path of config 5 on MI355X: pyRMT/mac.py operators and the
// loop body of benchmarks/mac_multi_disc_lid.py:36-98 (K discs, contact stress).
//
// Layout (mac.py:1-14) for an N x N cell grid: p, per-disc X1/X2/phi (N, N) cell centres;
// u (N, N+1) x-faces; v (N+1, N) y-faces; all row-major fp64.  Per step:
//   k_mac_centres   face -> centre velocity (u_c, v_c), finiteness flag
//   per disc        SL-RK4 of the map on (u_c, v_c) with the index-grid coordinates and the
//                   pre-advection mask (sim.hip k_sim_sl), exact extrapolation (extrap*.hip),
//                   phi rebuilt                                    mac_multi_disc_lid.py:70-77
//   k_mac_stress    sum_k (1 - H_k) sigma_k + pair contact stresses, J range  :79-89
//   k_mac_predict   explicit MAC predictor with the face force 1/2 (div S_l + div S_r)
//                   computed in place from S (fu / fv never stored)        :91-94
//   k_mac_rhs       rhs = (rho/dt) div u*; row-tree mean removed; DCT-II solve (poisson.hip)
//   k_mac_correct   u = u* - (dt/rho) grad phi on the interior faces            mac.py:126-139
//   k_mac_diag      per-disc centroids over phi <= 0, max|u|
// Every formula keeps the reference's NumPy operation order; only sin (H), the DCT and the
// reductions' summation order differ from the reference in the last bits.
#include "rmt_internal.hpp"
#include <algorithm>
#include <cmath>
#include <vector>

namespace rmt {

constexpr int MAC_MAXD = 8;
struct DiscSet {
    const double *X1[MAC_MAXD], *X2[MAC_MAXD], *phi[MAC_MAXD];
    int K;
};

__global__ void k_mac_centres(const double *__restrict__ u, const double *__restrict__ v, int N,
                              double *__restrict__ uc, double *__restrict__ vc, int *bad) {
    const long c = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (c >= (long)N * N) return;
    const int j = (int)(c / N), i = (int)(c % N);
    const double a = 0.5 * (u[(long)j * (N + 1) + i] + u[(long)j * (N + 1) + i + 1]);
    const double b = 0.5 * (v[c] + v[c + N]);
    uc[c] = a; vc[c] = b;
    if (!(isfinite(a) && isfinite(b))) atomicOr(bad, 1);
}

__global__ void k_mac_phi(const double *__restrict__ X1n, const double *__restrict__ X2n, long n,
                          double x0, double y0, double R, double *__restrict__ X1,
                          double *__restrict__ X2, double *__restrict__ phi) {
    const long c = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (c >= n) return;
    const double a = X1n[c], b = X2n[c];
    X1[c] = a; X2[c] = b;
    phi[c] = disc_phi(a, b, x0, y0, R);
}

// mac.py:729-749 at one cell: f(phi) = 1/2 (1 - phi/eps) below eps; d = phi_a - phi_b with
// central gradients inside and 0 on the boundary rows / columns
__device__ __forceinline__ void contact_cell(const double *__restrict__ pa,
                                             const double *__restrict__ pb, long c, int j, int i,
                                             int N, double eta, double Gsum, double eps,
                                             double dx, double dy, double &txx, double &txy,
                                             double &tyy) {
    const double a = pa[c], b = pb[c];
    const double fa = a < eps ? 0.5 * (1.0 - a / eps) : 0.0;
    const double fb = b < eps ? 0.5 * (1.0 - b / eps) : 0.0;
    const double fc = fb < fa ? fb : fa;
    double gx = 0.0, gy = 0.0;
    if (i >= 1 && i < N - 1) gx = ((pa[c + 1] - pb[c + 1]) - (pa[c - 1] - pb[c - 1])) / (2 * dx);
    if (j >= 1 && j < N - 1) gy = ((pa[c + N] - pb[c + N]) - (pa[c - N] - pb[c - N])) / (2 * dy);
    const double mag = sqrt(gx * gx + gy * gy) + 1e-12;
    const double nx = gx / mag, ny = gy / mag;
    const double s = -eta * fc * Gsum;
    txx = s * (nx * nx - 0.5);
    txy = s * (nx * ny);
    tyy = s * (ny * ny - 0.5);
}

__global__ void k_contact(const double *__restrict__ pa, const double *__restrict__ pb, int N,
                          double eta, double Gsum, double eps, double dx, double dy,
                          double *__restrict__ txx, double *__restrict__ txy,
                          double *__restrict__ tyy) {
    const long c = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (c >= (long)N * N) return;
    double a, b, d;
    contact_cell(pa, pb, c, (int)(c / N), (int)(c % N), N, eta, Gsum, eps, dx, dy, a, b, d);
    txx[c] = a; txy[c] = b; tyy[c] = d;
}

constexpr int MS_BLOCKS = 1024, MS_TPB = 256;
// S = sum_k (1 - H_k) sigma_k (+ contacts); J range partials per block
__global__ void __launch_bounds__(MS_TPB) k_mac_stress(DiscSet D, int N, double dx, double dy,
                                                       double mu_s, double w_t, double eta,
                                                       double eps, double *__restrict__ Sxx,
                                                       double *__restrict__ Sxy,
                                                       double *__restrict__ Syy,
                                                       double *__restrict__ part) {
    __shared__ double smin[MS_TPB], smax[MS_TPB];
    double jmin = 1.0, jmax = 1.0;
    const long n = (long)N * N;
    for (long c = blockIdx.x * (long)MS_TPB + threadIdx.x; c < n; c += (long)MS_BLOCKS * MS_TPB) {
        const int j = (int)(c / N), i = (int)(c % N);
        double axx = 0.0, axy = 0.0, ayy = 0.0;
        for (int k = 0; k < D.K; ++k) {
            Stress s{0.0, 0.0, 0.0, 1.0};
            if (j >= 1 && j < N - 1 && i >= 1 && i < N - 1)
                solid_stress_cell(D.X1[k], D.X2[k], D.phi[k], c, N, dx, dy, mu_s, 0.0, 0.0, 0.0,
                                  false, s);
            const double omh = 1 - heaviside(D.phi[k][c], w_t);
            axx = axx + omh * s.sxx; axy = axy + omh * s.sxy; ayy = ayy + omh * s.syy;
            jmin = fmin(jmin, s.J); jmax = fmax(jmax, s.J);
        }
        if (eta > 0)
            for (int a = 0; a < D.K; ++a)
                for (int b = a + 1; b < D.K; ++b) {
                    double txx, txy, tyy;
                    contact_cell(D.phi[a], D.phi[b], c, j, i, N, eta, 2 * mu_s, eps, dx, dy, txx,
                                 txy, tyy);
                    axx = axx + txx; axy = axy + txy; ayy = ayy + tyy;
                }
        Sxx[c] = axx; Sxy[c] = axy; Syy[c] = ayy;
    }
    smin[threadIdx.x] = jmin; smax[threadIdx.x] = jmax;
    __syncthreads();
    for (int w = MS_TPB / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w) {
            smin[threadIdx.x] = fmin(smin[threadIdx.x], smin[threadIdx.x + w]);
            smax[threadIdx.x] = fmax(smax[threadIdx.x], smax[threadIdx.x + w]);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) { part[2 * blockIdx.x] = smin[0]; part[2 * blockIdx.x + 1] = smax[0]; }
}

// utils.py grad_central at cell (j, i) of an N x N plane (one-sided at the edges)
__device__ __forceinline__ double divx_at(const double *Sxx, const double *Sxy, int j, int i, int N,
                                          double dx, double dy) {
    const long c = (long)j * N + i;
    return grad2(Sxx + c, 1, i, N, 2 * dx) + grad2(Sxy + c, N, j, N, 2 * dy);
}
__device__ __forceinline__ double divy_at(const double *Sxy, const double *Syy, int j, int i, int N,
                                          double dx, double dy) {
    const long c = (long)j * N + i;
    return grad2(Sxy + c, 1, i, N, 2 * dx) + grad2(Syy + c, N, j, N, 2 * dy);
}

// mac.py:196-232 with fu / fv of mac_multi_disc_lid.py:91-94 (S == nullptr: no force).
// Threads [0, N(N+1)) take u faces, [N(N+1), 2N(N+1)) v faces.
__global__ void k_mac_predict(const double *__restrict__ u, const double *__restrict__ v,
                              const double *__restrict__ Sxx, const double *__restrict__ Sxy,
                              const double *__restrict__ Syy, const double *__restrict__ fu,
                              const double *__restrict__ fv, int N, double nu, double dx,
                              double dy, double dx2, double dy2, double dt, double U, double rho,
                              double *__restrict__ us, double *__restrict__ vs) {
    // dx2, dy2: the reference's dx**2 on a Python float (libm pow), computed on the host
    const long q = blockIdx.x * (long)blockDim.x + threadIdx.x;
    const long nf = (long)N * (N + 1);
    const int W = N + 1;
    if (q < nf) {   // u face (j, i), row stride N + 1
        const int j = (int)(q / W), i = (int)(q % W);
        if (i == 0 || i == N) { us[q] = 0.0; return; }
        const double uc = u[q], ul = u[q - 1], ur = u[q + 1];
        const double dn = j > 0 ? u[q - W] : -u[q];                 // ghost: -u[0]
        const double up = j < N - 1 ? u[q + W] : 2.0 * U - u[q];    // ghost: 2U - u[-1]
        const double dudx = (ur - ul) / (2 * dx);
        const double dudy = (up - dn) / (2 * dy);
        const double lap = (ur - 2 * uc + ul) / dx2 + (up - 2 * uc + dn) / dy2;
        const long cv = (long)j * N + i;   // v[j][i]
        const double vu = 0.25 * (((v[cv - 1] + v[cv]) + v[cv + N - 1]) + v[cv + N]);
        double r = -(uc * dudx + vu * dudy) + nu * lap;
        if (Sxx) r = r + 0.5 * (divx_at(Sxx, Sxy, j, i, N, dx, dy) + divx_at(Sxx, Sxy, j, i - 1, N, dx, dy)) / rho;
        else if (fu) r = r + fu[q] / rho;
        us[q] = uc + dt * r;
    } else if (q < 2 * nf) {   // v face (j, i), row stride N
        const long p = q - nf;
        const int j = (int)(p / N), i = (int)(p % N);
        if (j == 0 || j == N) { vs[p] = 0.0; return; }
        const double vc = v[p], vd = v[p - N], vup = v[p + N];
        const double vl = i > 0 ? v[p - 1] : -v[p];
        const double vr = i < N - 1 ? v[p + 1] : -v[p];
        const double dvdx = (vr - vl) / (2 * dx);
        const double dvdy = (vup - vd) / (2 * dy);
        const double lap = (vr - 2 * vc + vl) / dx2 + (vup - 2 * vc + vd) / dy2;
        const long cu = (long)(j - 1) * W + i;   // u[j-1][i]
        const double uv = 0.25 * (((u[cu] + u[cu + 1]) + u[cu + W]) + u[cu + W + 1]);
        double r = -(uv * dvdx + vc * dvdy) + nu * lap;
        if (Sxx) r = r + 0.5 * (divy_at(Sxy, Syy, j, i, N, dx, dy) + divy_at(Sxy, Syy, j - 1, i, N, dx, dy)) / rho;
        else if (fv) r = r + fv[p] / rho;
        vs[p] = vc + dt * r;
    }
}

// rhs = (rho / dt) * div(u*, v*)  (mac.py:81-84, 133-134)
__global__ void k_mac_rhs(const double *__restrict__ u, const double *__restrict__ v, int N,
                          double dx, double dy, double coef, double *__restrict__ rhs) {
    const long c = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (c >= (long)N * N) return;
    const int j = (int)(c / N), i = (int)(c % N);
    const long cu = (long)j * (N + 1) + i;
    const double d = (u[cu + 1] - u[cu]) / dx + (v[c + N] - v[c]) / dy;
    rhs[c] = coef * d;
}

// u = u* - (dt/rho) grad_p_u(phi), v likewise (mac.py:87-101, 137-138)
__global__ void k_mac_correct(const double *__restrict__ us, const double *__restrict__ vs,
                              const double *__restrict__ phi, int N, double dx, double dy,
                              double c0, double *__restrict__ u, double *__restrict__ v) {
    const long q = blockIdx.x * (long)blockDim.x + threadIdx.x;
    const long nf = (long)N * (N + 1);
    if (q < nf) {
        const int j = (int)(q / (N + 1)), i = (int)(q % (N + 1));
        const double g = (i == 0 || i == N) ? 0.0 : (phi[(long)j * N + i] - phi[(long)j * N + i - 1]) / dx;
        u[q] = us[q] - c0 * g;
    } else if (q < 2 * nf) {
        const long p = q - nf;
        const int j = (int)(p / N), i = (int)(p % N);
        const double g = (j == 0 || j == N) ? 0.0 : (phi[p] - phi[p - N]) / dy;
        v[p] = vs[p] - c0 * g;
    }
}

// per-disc centroid sums over phi <= 0 (x, y, count) and max|u| partials
constexpr int MD_VALS = 3 * MAC_MAXD + 1;
__global__ void __launch_bounds__(MS_TPB) k_mac_diag(DiscSet D, const double *__restrict__ u,
                                                     int N, double dx, double *__restrict__ part) {
    __shared__ double s[MS_TPB];
    double acc[MD_VALS];
    for (int k = 0; k < MD_VALS; ++k) acc[k] = 0.0;
    const long n = (long)N * N, nf = (long)N * (N + 1);
    for (long c = blockIdx.x * (long)MS_TPB + threadIdx.x; c < nf; c += (long)MS_BLOCKS * MS_TPB) {
        acc[3 * MAC_MAXD] = fmax(acc[3 * MAC_MAXD], fabs(u[c]));
        if (c < n) {
            const int j = (int)(c / N), i = (int)(c % N);
            const double xc = (i + 0.5) * dx, yc = (j + 0.5) * dx;
            for (int k = 0; k < D.K; ++k)
                if (D.phi[k][c] <= 0.0) { acc[3 * k] += xc; acc[3 * k + 1] += yc; acc[3 * k + 2] += 1.0; }
        }
    }
    for (int k = 0; k < MD_VALS; ++k) {
        s[threadIdx.x] = acc[k];
        __syncthreads();
        for (int w = MS_TPB / 2; w > 0; w >>= 1) {
            if (threadIdx.x < w)
                s[threadIdx.x] = k == 3 * MAC_MAXD ? fmax(s[threadIdx.x], s[threadIdx.x + w])
                                                   : s[threadIdx.x] + s[threadIdx.x + w];
            __syncthreads();
        }
        if (threadIdx.x == 0) part[(long)blockIdx.x * MD_VALS + k] = s[0];
        __syncthreads();
    }
}

static int mac_project_impl(rmt_ctx *ctx, const double *us, const double *vs, double dx,
                            double dy, double dt, double rho, double *u, double *v, double *phi,
                            double *rhs, bool plan = true) {
    const int N = ctx->nx;
    const long n = (long)N * N, nf = (long)N * (N + 1);
    if (plan) RMT_TRY(dct2_plan(ctx, N, N, dx, dy));
    k_mac_rhs<<<grid1d(n, 256), 256, 0, ctx->stream>>>(us, vs, N, dx, dy, rho / dt, rhs);
    RMT_LAUNCHED();
    RMT_TRY(sub_mean_rows(ctx, rhs, N, N));     // rhs - rhs.mean() (mac.py:135)
    RMT_TRY(dct2_solve(ctx, rhs, phi));
    k_mac_correct<<<grid1d(2 * nf, 256), 256, 0, ctx->stream>>>(us, vs, phi, N, dx, dy, dt / rho,
                                                                u, v);
    RMT_LAUNCHED();
    return RMT_OK;
}

}  // namespace rmt

// ------------------------------------------------------------------ fused MAC sim --
struct rmt_mac_sim {
    rmt_ctx *ctx = nullptr;
    rmt_mac_params P{};
    void *block = nullptr;
    double *u, *v, *p, *us, *vs, *uc, *vc, *X1n, *X2n, *phi_pre, *Sxx, *Sxy, *Syy;
    double *X1[RMT_MAC_MAXD], *X2[RMT_MAC_MAXD], *phi[RMT_MAC_MAXD];
    double *xs, *ys, *part, *out;
    int *flags;
    double t = 0;
    std::vector<rmt_mac_diag> diag;
};

using namespace rmt;

extern "C" {

int rmt_mac_divergence(rmt_ctx *ctx, const double *u, const double *v, double dx, double dy,
                       double *out) {
    RMT_CHECK(ctx && u && v && out && ctx->nx == ctx->ny, RMT_EINVAL, "bad argument");
    const long n = (long)ctx->nx * ctx->nx;
    k_mac_rhs<<<grid1d(n, 256), 256, 0, ctx->stream>>>(u, v, ctx->nx, dx, dy, 1.0, out);
    RMT_LAUNCHED();
    return RMT_OK;
}

int rmt_mac_gradient_p(rmt_ctx *ctx, const double *p, double dx, double dy, double *gu,
                       double *gv) {
    RMT_CHECK(ctx && p && gu && gv && ctx->nx == ctx->ny, RMT_EINVAL, "bad argument");
    const int N = ctx->nx;
    const long nf = (long)N * (N + 1);
    // u - c*g with u = 0 and c = -1 gives g exactly (0 - (-1)*g = g)
    RMT_TRY(ensure_scratch(ctx, nf * sizeof(double)));
    RMT_HIP(hipMemsetAsync(ctx->scratch, 0, nf * sizeof(double), ctx->stream));
    k_mac_correct<<<grid1d(2 * nf, 256), 256, 0, ctx->stream>>>(ctx->scratch, ctx->scratch, p, N,
                                                                dx, dy, -1.0, gu, gv);
    RMT_LAUNCHED();
    return RMT_OK;
}

int rmt_mac_solve_poisson_neumann(rmt_ctx *ctx, const double *rhs, double dx, double dy,
                                  const double *lamx, const double *lamy, double *out) {
    RMT_CHECK(ctx && rhs && out && !lamx == !lamy, RMT_EINVAL, "bad argument");
    RMT_TRY(dct2_plan(ctx, ctx->ny, ctx->nx, dx, dy));
    if (lamx) RMT_TRY(dct2_set_lambda(ctx, lamx, lamy));
    return dct2_solve(ctx, rhs, out);
}

int rmt_mac_project(rmt_ctx *ctx, const double *us, const double *vs, double dx, double dy,
                    double dt, double rho, const double *lamx, const double *lamy, double *u,
                    double *v, double *phi) {
    RMT_CHECK(ctx && us && vs && u && v && phi && ctx->nx == ctx->ny && !lamx == !lamy,
              RMT_EINVAL, "bad argument");
    const long n = (long)ctx->nx * ctx->nx;
    RMT_TRY(ensure_scratch(ctx, n * sizeof(double)));
    RMT_TRY(dct2_plan(ctx, ctx->ny, ctx->nx, dx, dy));
    if (lamx) RMT_TRY(dct2_set_lambda(ctx, lamx, lamy));
    return mac_project_impl(ctx, us, vs, dx, dy, dt, rho, u, v, phi, ctx->scratch, !lamx);
}

int rmt_mac_momentum_predictor(rmt_ctx *ctx, const double *u, const double *v, double nu,
                               double dx, double dy, double dt, double U_lid, const double *fu,
                               const double *fv, double rho, double *us, double *vs) {
    RMT_CHECK(ctx && u && v && us && vs && ctx->nx == ctx->ny, RMT_EINVAL, "bad argument");
    RMT_CHECK(!fu == !fv, RMT_EINVAL, "give both face forces or neither");
    const int N = ctx->nx;
    const long nf = (long)N * (N + 1);
    k_mac_predict<<<grid1d(2 * nf, 256), 256, 0, ctx->stream>>>(
        u, v, nullptr, nullptr, nullptr, fu, fv, N, nu, dx, dy, std::pow(dx, 2.0),
        std::pow(dy, 2.0), dt, U_lid, rho, us, vs);
    RMT_LAUNCHED();
    return RMT_OK;
}

int rmt_mac_contact_stress(rmt_ctx *ctx, const double *phi_a, const double *phi_b, double eta,
                           double Gsum, double eps, double dx, double dy, double *txx,
                           double *txy, double *tyy);

int rmt_mac_sim_create(rmt_ctx *ctx, const rmt_mac_params *prm, rmt_mac_sim **out) {
    RMT_CHECK(ctx && prm && out, RMT_EINVAL, "null argument");
    RMT_CHECK(prm->n_discs >= 1 && prm->n_discs <= RMT_MAC_MAXD, RMT_EINVAL, "1..8 discs");
    RMT_CHECK(ctx->nx == prm->N && ctx->ny == prm->N, RMT_EINVAL, "ctx grid != N x N");
    const int N = prm->N;
    RMT_TRY(dct2_plan(ctx, N, N, prm->dx, prm->dx));
    rmt_mac_sim *S = new rmt_mac_sim;
    S->ctx = ctx; S->P = *prm;
    const long n = (long)N * N, nf = (long)N * (N + 1);
    const int K = prm->n_discs;
    const size_t dbl = 5 * nf + (9 + 3 * K) * n + 2 * N + (2 + MD_VALS) * MS_BLOCKS + 64;
    RMT_HIP(hipMalloc(&S->block, dbl * 8 + 64));
    RMT_HIP(hipMemsetAsync(S->block, 0, dbl * 8 + 64, ctx->stream));
    double *q = (double *)S->block;
    double **faces[] = {&S->u, &S->v, &S->us, &S->vs};
    for (auto pp : faces) { *pp = q; q += nf; }
    q += nf;   // spare
    double **cells[] = {&S->p, &S->uc, &S->vc, &S->X1n, &S->X2n, &S->phi_pre, &S->Sxx, &S->Sxy,
                        &S->Syy};
    for (auto pp : cells) { *pp = q; q += n; }
    for (int k = 0; k < K; ++k) {
        S->X1[k] = q; q += n; S->X2[k] = q; q += n; S->phi[k] = q; q += n;
    }
    S->xs = q; q += N;
    S->ys = q; q += N;
    S->part = q; q += (2 + MD_VALS) * MS_BLOCKS;   // J range, then centroid partials
    S->out = q; q += 32;
    S->flags = (int *)q;
    // index-grid coordinates (mac_multi_disc_lid.py:41): Xg = arange(N) * dx
    std::vector<double> g(N);
    for (int i = 0; i < N; ++i) g[i] = i * prm->dx;
    RMT_HIP(hipMemcpyAsync(S->xs, g.data(), N * 8, hipMemcpyHostToDevice, ctx->stream));
    RMT_HIP(hipMemcpyAsync(S->ys, g.data(), N * 8, hipMemcpyHostToDevice, ctx->stream));
    RMT_TRY(ensure_bytes(ctx, extrap_workspace(N, N, prm->layers)));
    RMT_HIP(hipStreamSynchronize(ctx->stream));
    *out = S;
    return RMT_OK;
}

int rmt_mac_sim_destroy(rmt_mac_sim *S) {
    if (!S) return RMT_OK;
    hipFree(S->block);
    delete S;
    return RMT_OK;
}

int rmt_mac_sim_field(rmt_mac_sim *S, int field, int disc, double **ptr) {
    RMT_CHECK(S && ptr, RMT_EINVAL, "null argument");
    if (field <= 2) {
        double *f[] = {S->u, S->v, S->p};
        *ptr = f[field];
        return RMT_OK;
    }
    RMT_CHECK(field <= 5 && disc >= 0 && disc < S->P.n_discs, RMT_EINVAL, "unknown field/disc");
    *ptr = field == 3 ? S->X1[disc] : field == 4 ? S->X2[disc] : S->phi[disc];
    return RMT_OK;
}

int rmt_mac_sim_step(rmt_mac_sim *S, int nsteps, double t_end) {
    RMT_CHECK(S, RMT_EINVAL, "null sim");
    rmt_ctx *ctx = S->ctx;
    const rmt_mac_params &P = S->P;
    const int N = P.N, K = P.n_discs;
    const long n = (long)N * N, nf = (long)N * (N + 1);
    hipStream_t st = ctx->stream;
    DiscSet D{};
    D.K = K;
    for (int k = 0; k < K; ++k) { D.X1[k] = S->X1[k]; D.X2[k] = S->X2[k]; D.phi[k] = S->phi[k]; }
    const double dx = P.dx, w_t = 2.0 * dx, eps = 3.0 * dx, nu = P.mu_f / P.rho;
    const double dx2 = std::pow(dx, 2.0);
    for (int it = 0; it < nsteps; ++it) {
        if (!(S->t < t_end)) break;
        double dt = P.dt;
        if (S->t + dt > t_end) dt = t_end - S->t;
        RMT_HIP(hipMemsetAsync(S->flags, 0, 4 * sizeof(int), st));
        k_mac_centres<<<grid1d(n, 256), 256, 0, st>>>(S->u, S->v, N, S->uc, S->vc, S->flags);
        RMT_LAUNCHED();
        for (int k = 0; k < K; ++k) {
            // phi from the current map (already S->phi[k]), advect with the pre-advection mask
            RMT_TRY(sl_disc_map(ctx, S->X1[k], S->X2[k], S->uc, S->vc, S->xs, S->ys, dt, dx, dx,
                                P.cx[k], P.cy[k], P.R[k], S->X1n, S->X2n, S->phi_pre,
                                S->flags + 1));
            RMT_TRY(extrapolate(ctx, S->X1n, S->X2n, S->phi_pre, dx, dx, P.layers, S->X1n, S->X2n,
                                S->flags + 2));
            k_mac_phi<<<grid1d(n, 256), 256, 0, st>>>(S->X1n, S->X2n, n, P.cx[k], P.cy[k], P.R[k],
                                                      S->X1[k], S->X2[k], S->phi[k]);
            RMT_LAUNCHED();
        }
        k_mac_stress<<<MS_BLOCKS, MS_TPB, 0, st>>>(D, N, dx, dx, P.mu_s, w_t, P.eta, eps, S->Sxx,
                                                    S->Sxy, S->Syy, S->part);
        RMT_LAUNCHED();
        double jr[2 * MS_BLOCKS];
        RMT_HIP(hipMemcpyAsync(jr, S->part, sizeof(jr), hipMemcpyDeviceToHost, st));
        k_mac_predict<<<grid1d(2 * nf, 256), 256, 0, st>>>(S->u, S->v, S->Sxx, S->Sxy, S->Syy,
                                                            nullptr, nullptr, N, nu, dx, dx, dx2,
                                                            dx2, dt, P.U_lid, P.rho, S->us, S->vs);
        RMT_LAUNCHED();
        RMT_TRY(mac_project_impl(ctx, S->us, S->vs, dx, dx, dt, P.rho, S->u, S->v, S->p,
                                 S->X1n));
        k_mac_diag<<<MS_BLOCKS, MS_TPB, 0, st>>>(D, S->u, N, dx, S->part + 2 * MS_BLOCKS);
        RMT_LAUNCHED();
        std::vector<double> dp((size_t)MS_BLOCKS * MD_VALS);
        RMT_HIP(hipMemcpyAsync(dp.data(), S->part + 2 * MS_BLOCKS, dp.size() * 8,
                               hipMemcpyDeviceToHost, st));
        int fl[4];
        RMT_HIP(hipMemcpyAsync(fl, S->flags, sizeof(fl), hipMemcpyDeviceToHost, st));
        RMT_HIP(hipStreamSynchronize(st));
        RMT_CHECK(!fl[0] && !fl[1], RMT_ENONFINITE,
                  "advect_reference_map: non-finite velocity (the simulation diverged)");
        S->t += dt;
        rmt_mac_diag r{};
        r.t = S->t; r.dt = dt; r.n_discs = K;
        r.minJ = 1.0; r.maxJ = 1.0;
        for (int b = 0; b < MS_BLOCKS; ++b) {
            r.minJ = std::fmin(r.minJ, jr[2 * b]); r.maxJ = std::fmax(r.maxJ, jr[2 * b + 1]);
        }
        double acc[MD_VALS] = {0};
        for (int b = 0; b < MS_BLOCKS; ++b)
            for (int k = 0; k < MD_VALS; ++k) {
                const double x = dp[(size_t)b * MD_VALS + k];
                acc[k] = k == 3 * MAC_MAXD ? std::fmax(acc[k], x) : acc[k] + x;
            }
        for (int k = 0; k < K; ++k) {
            r.cx[k] = acc[3 * k + 2] > 0 ? acc[3 * k] / acc[3 * k + 2] : NAN;
            r.cy[k] = acc[3 * k + 2] > 0 ? acc[3 * k + 1] / acc[3 * k + 2] : NAN;
        }
        r.umax = acc[3 * MAC_MAXD];
        S->diag.push_back(r);
    }
    return RMT_OK;
}

int rmt_mac_sim_diagnostics(rmt_mac_sim *S, rmt_mac_diag *out, int max_records, int *n_records) {
    RMT_CHECK(S && n_records, RMT_EINVAL, "null argument");
    const int m = (int)std::min<size_t>(S->diag.size(), (size_t)std::max(0, max_records));
    for (int k = 0; k < m; ++k) out[k] = S->diag[S->diag.size() - m + k];
    *n_records = (int)S->diag.size();
    return RMT_OK;
}

int rmt_mac_contact_stress(rmt_ctx *ctx, const double *phi_a, const double *phi_b, double eta,
                           double Gsum, double eps, double dx, double dy, double *txx,
                           double *txy, double *tyy) {
    RMT_CHECK(ctx && phi_a && phi_b && txx && txy && tyy && ctx->nx == ctx->ny, RMT_EINVAL,
              "bad argument");
    const int N = ctx->nx;
    const long n = (long)N * N;
    k_contact<<<grid1d(n, 256), 256, 0, ctx->stream>>>(phi_a, phi_b, N, eta, Gsum, eps, dx, dy,
                                                       txx, txy, tyy);
    RMT_LAUNCHED();
    return RMT_OK;
}

}  // extern "C"
