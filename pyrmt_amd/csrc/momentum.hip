// momentum.hip -- functions.py:673-762 momentum_step_rk4 (gamma = 0) on MI355X.
//
// Structure: one prep pass (elastic stress, smoothed Heaviside H, rho, solid mask) and
// four LDS-tiled RK4 stage passes.  A stage pass owns a TY x TX output tile; it stages
// the BC'd stage velocity on the tile + 3 halo and the blended stress on the tile + 2
// halo in LDS (the domain-edge one-sided stencils reach 2 cells inward for the stress
// divergence and 3 for the velocity gradients feeding it), then evaluates
// velocity_rhs_blended_optimized (functions.py:897-944) per output cell.
// Stage outputs: s0 -> k1; s1 -> k2, acc = k1 + 2 k2; s2 -> k3, acc += 2 k3;
// s3 -> u* = u + dt/6 (acc + k4) (pre-BC; the final BC pass follows), i.e. exactly the
// reference's left-to-right (((k1 + 2 k2) + 2 k3) + k4).
#include "rmt_internal.hpp"

namespace rmt {

// Debug builds (-DRMT_CHECKED): every global index is range-checked against the plane
// size, reported once per wave with printf and clamped, so a bad index is located
// without faulting the GPU.
#ifdef RMT_CHECKED
__device__ __forceinline__ long ck(long idx, long n, int line) {
    if (idx < 0 || idx >= n) {
        printf("RMT_CHECKED momentum.hip:%d idx %ld n %ld block (%d,%d) thread %d\n", line, idx,
               n, (int)blockIdx.x, (int)blockIdx.y, (int)threadIdx.x);
        return idx < 0 ? 0 : n - 1;
    }
    return idx;
}
#define CK(idx) ::rmt::ck((idx), (long)ny * nx, __LINE__)
#else
#define CK(idx) (idx)
#endif

constexpr int MTX = 64, MTY = 8, MT = MTX * MTY;      // output tile, 512 threads
constexpr int VH = 3, SH = 2;                          // velocity / stress halos
constexpr int VW = MTX + 2 * VH, VHh = MTY + 2 * VH;   // velocity region 70 x 14
constexpr int SW = MTX + 2 * SH, SHh = MTY + 2 * SH;   // stress region 68 x 12

struct MomArgs {
    const double *u, *v, *kpu, *kpv, *p, *sxx, *sxy, *syy, *H, *rho;
    const unsigned char *solid;
    double *ku, *kv, *accu, *accv;   // stage outputs
    double *outu, *outv;             // final stage: u*, v*
    int ny, nx, stage, bc, visc;
    double coef, lid, dx, dy, mu_f, eta_s, dt6;
};

__global__ void k_mom_prep(const double *__restrict__ X1, const double *__restrict__ X2,
                           const double *__restrict__ phi, int ny, int nx, double dx, double dy,
                           double mu_s, double kappa, double w_cut, double clamp, double w_t,
                           double rho_s, double rho_f, double *__restrict__ sxx,
                           double *__restrict__ sxy, double *__restrict__ syy,
                           double *__restrict__ J, double *__restrict__ H,
                           double *__restrict__ rho, unsigned char *__restrict__ solid,
                           int *any_solid) {
    long c = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (c >= (long)ny * nx) return;
    int j = (int)(c / nx), i = (int)(c % nx);
    Stress s{0.0, 0.0, 0.0, 1.0};
    if (j >= 1 && j < ny - 1 && i >= 1 && i < nx - 1)
        solid_stress_cell(X1, X2, phi, c, nx, dx, dy, mu_s, kappa, w_cut, clamp, false, s);
    sxx[c] = s.sxx; sxy[c] = s.sxy; syy[c] = s.syy; J[c] = s.J;
    double pc = phi[c], h = heaviside(pc, w_t);
    H[c] = h;
    rho[c] = (1 - h) * rho_s + h * rho_f;
    bool sd = pc <= 0.0;
    solid[c] = sd;
    if (__any(sd) && (threadIdx.x & 63) == 0) atomicOr(any_solid, 1);
}

__global__ void __launch_bounds__(MT) k_mom_stage(MomArgs A) {
    __shared__ double su[VHh * VW], sv[VHh * VW];
    __shared__ double gxx[SHh * SW], gxy[SHh * SW], gyy[SHh * SW];
    const int ny = A.ny, nx = A.nx;
    const int i0 = blockIdx.x * MTX, j0 = blockIdx.y * MTY;
    const int t = threadIdx.x;
    const double h2x = 2 * A.dx, h2y = 2 * A.dy;

    // raw (pre-BC) stage velocity from global
    auto rawu = [&](int j, int i) {
        long c = (long)j * nx + i;
        return A.stage == 0 ? A.u[CK(c)] : A.u[CK(c)] + A.coef * A.kpu[CK(c)];
    };
    auto rawv = [&](int j, int i) {
        long c = (long)j * nx + i;
        return A.stage == 0 ? A.v[CK(c)] : A.v[CK(c)] + A.coef * A.kpv[CK(c)];
    };
    // 1. BC'd stage velocity on the tile + VH halo (cells outside the domain unused)
    for (int q = t; q < VHh * VW; q += MT) {
        int j = j0 - VH + q / VW, i = i0 - VH + q % VW;
        if (j < 0 || j >= ny || i < 0 || i >= nx) continue;
        double uu, vv;
        bc_value(A.bc, A.lid, j, i, ny, nx, rawu, rawv, uu, vv);
        su[q] = uu; sv[q] = vv;
    }
    __syncthreads();
    // 2. blended stress on the tile + SH halo: H sigma_f + (1-H) (sigma_el + eta_s visc)
    const double m2 = 2 * A.mu_f, es_h = A.eta_s * 0.5;
    for (int q = t; q < SHh * SW; q += MT) {
        int j = j0 - SH + q / SW, i = i0 - SH + q % SW;
        if (j < 0 || j >= ny || i < 0 || i >= nx) continue;
        int vq = (q / SW + (VH - SH)) * VW + (q % SW + (VH - SH));
        double dudx = grad2(su + vq, 1, i, nx, h2x), dvdy = grad2(sv + vq, VW, j, ny, h2y);
        double dudy = grad2(su + vq, VW, j, ny, h2y), dvdx = grad2(sv + vq, 1, i, nx, h2x);
        long c = (long)j * nx + i;
        double ex = A.sxx[CK(c)], ey = A.syy[CK(c)], exy = A.sxy[CK(c)];
        if (A.visc && A.solid[CK(c)]) {
            ex = ex + A.eta_s * dudx;
            ey = ey + A.eta_s * dvdy;
            exy = exy + es_h * (dudy + dvdx);
        }
        double h = A.H[CK(c)], omh = 1 - h;
        gxx[q] = h * (m2 * dudx) + omh * ex;
        gyy[q] = h * (m2 * dvdy) + omh * ey;
        gxy[q] = h * (A.mu_f * (dudy + dvdx)) + omh * exy;
    }
    __syncthreads();
    // 3. per output cell: div sigma, upwind advection, -grad p, / (rho + 1e-12)
    const int tj = t / MTX, ti = t % MTX;
    const int j = j0 + tj, i = i0 + ti;
    if (j >= ny || i >= nx) return;
    const long c = (long)j * nx + i;
    const int sq = (tj + SH) * SW + (ti + SH), vq = (tj + VH) * VW + (ti + VH);
    double divx = grad2(gxx + sq, 1, i, nx, h2x) + grad2(gxy + sq, SW, j, ny, h2y);
    double divy = grad2(gxy + sq, 1, i, nx, h2x) + grad2(gyy + sq, SW, j, ny, h2y);
    double us = su[vq], vs = sv[vq];
    double uadv = -us * upwind3(su + vq, 1, i, nx, us, A.dx) - vs * upwind3(su + vq, VW, j, ny, vs, A.dy);
    double vadv = -us * upwind3(sv + vq, 1, i, nx, us, A.dx) - vs * upwind3(sv + vq, VW, j, ny, vs, A.dy);
    double dpx = grad2(A.p + c, 1, i, nx, h2x), dpy = grad2(A.p + c, nx, j, ny, h2y);
    double den = A.rho[CK(c)] + 1e-12;
    double ku = uadv + (divx + 0.0 - dpx) / den;
    double kv = vadv + (divy + 0.0 - dpy) / den;
    switch (A.stage) {
    case 0: A.ku[c] = ku; A.kv[c] = kv; break;
    case 1: A.accu[c] = A.kpu[c] + 2 * ku; A.accv[c] = A.kpv[c] + 2 * kv;
            A.ku[c] = ku; A.kv[c] = kv; break;
    case 2: A.accu[c] = A.accu[c] + 2 * ku; A.accv[c] = A.accv[c] + 2 * kv;
            A.ku[c] = ku; A.kv[c] = kv; break;
    default: A.outu[c] = A.u[c] + A.dt6 * (A.accu[c] + ku);
             A.outv[c] = A.v[c] + A.dt6 * (A.accv[c] + kv); break;
    }
}

// Final BC (functions.py:760) on the boundary cells only: 2(nx + ny) threads.
__global__ void k_bc_edges(int kind, double lid, double *u, double *v, int ny, int nx) {
    int q = blockIdx.x * blockDim.x + threadIdx.x;
    int j, i;
    if (q < nx) { j = 0; i = q; }
    else if (q < 2 * nx) { j = ny - 1; i = q - nx; }
    else if (q < 2 * nx + ny - 2) { j = q - 2 * nx + 1; i = 0; }
    else if (q < 2 * nx + 2 * (ny - 2)) { j = q - 2 * nx - (ny - 2) + 1; i = nx - 1; }
    else return;
    auto ru = [&](int jj, int ii) { return u[(long)jj * nx + ii]; };
    auto rv = [&](int jj, int ii) { return v[(long)jj * nx + ii]; };
    double uu, vv;
    bc_value(kind, lid, j, i, ny, nx, ru, rv, uu, vv);   // reads interior cells only
    u[(long)j * nx + i] = uu; v[(long)j * nx + i] = vv;
}

int momentum_rk4(rmt_ctx *ctx, const rmt_momentum_params *P, const double *u, const double *v,
                 const double *p, const double *X1, const double *X2, const double *phi,
                 double *u_new, double *v_new, double *sxx, double *sxy, double *syy, double *J,
                 const MomWork &W) {
    const int ny = ctx->ny, nx = ctx->nx;
    const long n = (long)ny * nx;
    RMT_CHECK(P->bc_kind >= 0 && P->bc_kind <= 2, RMT_EINVAL, "unknown velocity bc kind");
    double w_cut = P->stress_band ? P->w_t : 0.0, clamp = P->stress_band ? P->detg_clamp : 0.0;
    RMT_HIP(hipMemsetAsync(W.any_solid, 0, sizeof(int), ctx->stream));
    k_mom_prep<<<grid1d(n, 256), 256, 0, ctx->stream>>>(
        X1, X2, phi, ny, nx, P->dx, P->dy, P->mu_s, P->kappa, w_cut, clamp, P->w_t, P->rho_s,
        P->rho_f, sxx, sxy, syy, J, W.H, W.rho, W.solid, W.any_solid);
    RMT_LAUNCHED();
    // visc = eta_s > 0 and any(solid): evaluated on device; pass eta_s and let the
    // kernel read the flag through the solid mask (no solid cell -> no viscous add).
    MomArgs A{};
    A.u = u; A.v = v; A.p = p; A.sxx = sxx; A.sxy = sxy; A.syy = syy; A.H = W.H; A.rho = W.rho;
    A.solid = W.solid; A.ny = ny; A.nx = nx; A.bc = P->bc_kind; A.lid = P->lid;
    A.dx = P->dx; A.dy = P->dy; A.mu_f = P->mu_f; A.eta_s = P->eta_s; A.dt6 = P->dt / 6.0;
    A.visc = P->eta_s > 0.0;
    A.accu = W.accu; A.accv = W.accv; A.outu = u_new; A.outv = v_new;
    dim3 grid((nx + MTX - 1) / MTX, (ny + MTY - 1) / MTY);
    const double coef[4] = {0.0, 0.5 * P->dt, 0.5 * P->dt, P->dt};
    double *kbu[2] = {W.k1u, W.k2u}, *kbv[2] = {W.k1v, W.k2v};
    if (ctx->prof) RMT_HIP(hipEventRecord(ctx->ev[0], ctx->stream));
    for (int s = 0; s < 4; ++s) {
        A.stage = s; A.coef = coef[s];
        // stage 0 reads only u, v; kp* still point at valid planes so that no load the
        // compiler may speculate from the stage select can touch address 0
        A.kpu = s ? kbu[(s - 1) & 1] : u; A.kpv = s ? kbv[(s - 1) & 1] : v;
        A.ku = kbu[s & 1]; A.kv = kbv[s & 1];
        k_mom_stage<<<grid, MT, 0, ctx->stream>>>(A);
        RMT_LAUNCHED();
    }
    if (ctx->prof) RMT_HIP(hipEventRecord(ctx->ev[1], ctx->stream));
    k_bc_edges<<<grid1d(2 * (nx + ny), 256), 256, 0, ctx->stream>>>(P->bc_kind, P->lid, u_new,
                                                                     v_new, ny, nx);
    RMT_LAUNCHED();
    return RMT_OK;
}

}  // namespace rmt

using namespace rmt;

extern "C" int rmt_momentum_step_rk4(rmt_ctx *ctx, const rmt_momentum_params *P, const double *u,
                                     const double *v, const double *p, const double *X1,
                                     const double *X2, const double *phi, double *u_new,
                                     double *v_new, double *sxx, double *sxy, double *syy,
                                     double *J) {
    RMT_CHECK(ctx && P, RMT_EINVAL, "null argument");
    const long n = (long)ctx->ny * ctx->nx;
    RMT_TRY(ensure_scratch(ctx, 8 * n * sizeof(double)));
    RMT_TRY(ensure_bytes(ctx, n + 64));
    double *w = ctx->scratch;
    MomWork W{w, w + n, w + 2 * n, w + 3 * n, w + 4 * n, w + 5 * n, w + 6 * n, w + 7 * n,
              ctx->bytes + 64, (int *)ctx->bytes};
    return momentum_rk4(ctx, P, u, v, p, X1, X2, phi, u_new, v_new, sxx, sxy, syy, J, W);
}
