// periodic.hip -- functions.py:1177-1290, the doubly-periodic projection branch (A25).
//
// The collocated grid carries an overlap row / column (x[-1] == x[0] physically); the
// periodic field lives on the reduced (N-1) x (N-1) sub-grid.  Operators: wide central
// divergence / gradient with wrap-around on the reduced grid, tiled back onto the overlap
// grid (_tile_overlap :1205-1213); the Poisson solve is a 2D real FFT of the reduced rhs
// (rocFFT D2Z / Z2D, the reference uses numpy.fft), divided by the separable symbol
// -sin^2(2 pi k / m) / h^2 per axis with the null modes (|eig| < 1e-12: constant and
// Nyquist) zeroed; means by the row-tree reduction.
#include "rmt_internal.hpp"
#include <algorithm>
#include <vector>

namespace rmt {

struct PerPlan {
    int m = 0;
    rocfft_plan fwd = nullptr, inv = nullptr;
    rocfft_execution_info info = nullptr;
    void *work = nullptr;
    size_t work_bytes = 0;
    double *red = nullptr, *C = nullptr, *lamx = nullptr, *lamy = nullptr, *g = nullptr;
};

static int rfc(rocfft_status s, const char *what) {
    if (s != rocfft_status_success) {
        set_error(std::string("rocFFT (periodic): ") + what + " failed");
        return RMT_EDEVICE;
    }
    return RMT_OK;
}

void per_destroy(PerPlan *P) {
    if (!P) return;
    if (P->fwd) rocfft_plan_destroy(P->fwd);
    if (P->inv) rocfft_plan_destroy(P->inv);
    if (P->info) rocfft_execution_info_destroy(P->info);
    (void)hipFree(P->work); (void)hipFree(P->red); (void)hipFree(P->C); (void)hipFree(P->lamx); (void)hipFree(P->lamy);
    (void)hipFree(P->g);
    delete P;
}

static int per_plan(rmt_ctx *ctx, const double *lamx, const double *lamy) {
    const int N = ctx->nx, m = N - 1;
    RMT_CHECK(ctx->nx == ctx->ny && m >= 2, RMT_EINVAL, "periodic solve: square grid, N >= 3");
    PerPlan *P = ctx->per;
    if (!P || P->m != m) {
        if (P) per_destroy(P);
        P = ctx->per = new PerPlan;
        P->m = m;
        static bool setup = false;
        if (!setup) { RMT_TRY(rfc(rocfft_setup(), "setup")); setup = true; }
        const size_t len[2] = {(size_t)m, (size_t)m};
        RMT_TRY(rfc(rocfft_plan_create(&P->fwd, rocfft_placement_notinplace,
                                       rocfft_transform_type_real_forward,
                                       rocfft_precision_double, 2, len, 1, nullptr), "plan fwd"));
        RMT_TRY(rfc(rocfft_plan_create(&P->inv, rocfft_placement_notinplace,
                                       rocfft_transform_type_real_inverse,
                                       rocfft_precision_double, 2, len, 1, nullptr), "plan inv"));
        size_t w1 = 0, w2 = 0;
        rocfft_plan_get_work_buffer_size(P->fwd, &w1);
        rocfft_plan_get_work_buffer_size(P->inv, &w2);
        P->work_bytes = std::max(w1, w2);
        if (P->work_bytes) RMT_HIP(hipMalloc(&P->work, P->work_bytes));
        RMT_TRY(rfc(rocfft_execution_info_create(&P->info), "execution_info_create"));
        if (P->work_bytes)
            RMT_TRY(rfc(rocfft_execution_info_set_work_buffer(P->info, P->work, P->work_bytes),
                        "set_work_buffer"));
        RMT_HIP(hipMalloc(&P->red, (size_t)m * m * sizeof(double)));
        RMT_HIP(hipMalloc(&P->C, (size_t)m * (m / 2 + 1) * 2 * sizeof(double)));
        RMT_HIP(hipMalloc(&P->lamx, m * sizeof(double)));
        RMT_HIP(hipMalloc(&P->lamy, m * sizeof(double)));
        RMT_HIP(hipMalloc(&P->g, 2 * (size_t)N * N * sizeof(double)));
    }
    RMT_HIP(hipMemcpyAsync(P->lamx, lamx, m * 8, hipMemcpyHostToDevice, ctx->stream));
    RMT_HIP(hipMemcpyAsync(P->lamy, lamy, m * 8, hipMemcpyHostToDevice, ctx->stream));
    RMT_HIP(hipStreamSynchronize(ctx->stream));
    return RMT_OK;
}

// functions.py:1236-1252: (roll(f, -1) - roll(f, 1)) / 2h on the reduced grid, tiled
__global__ void k_per_grad(const double *__restrict__ a, const double *__restrict__ b, int N,
                           double dx, double dy, int mode, double *__restrict__ o1,
                           double *__restrict__ o2) {
    const long c = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (c >= (long)N * N) return;
    const int m = N - 1;
    const int j = (int)(c / N) % m, i = (int)(c % N) % m;   // tile overlap
    const int ip = (i + 1) % m, im = (i + m - 1) % m, jp = (j + 1) % m, jm = (j + m - 1) % m;
    const double ddx = (a[(long)j * N + ip] - a[(long)j * N + im]) / (2.0 * dx);
    const double *f = mode ? a : b;   // mode 0: divergence of (a, b); 1: gradient of a
    const double ddy = (f[(long)jp * N + i] - f[(long)jm * N + i]) / (2.0 * dy);
    if (mode == 0) o1[c] = ddx + ddy;
    else { o1[c] = ddx; o2[c] = ddy; }
}

__global__ void k_per_extract(const double *__restrict__ full, int N, double s, double dt,
                              double *__restrict__ red) {
    const int m = N - 1;
    const long q = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (q >= (long)m * m) return;
    const int j = (int)(q / m), i = (int)(q % m);
    // rhs_2d = rho_bar * divU / dt (functions.py:1282), then r = rhs[:-1, :-1]
    red[q] = dt > 0 ? (s * full[(long)j * N + i]) / dt : full[(long)j * N + i];
}

// phat = rhat / eig, null modes (|eig| < 1e-12) -> 0 (functions.py:1196-1201, 1228-1229)
__global__ void k_per_divide(double2 *__restrict__ C, int m, const double *__restrict__ lamx,
                             const double *__restrict__ lamy) {
    const int h = m / 2 + 1;
    const long q = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (q >= (long)m * h) return;
    const int ky = (int)(q / h), kx = (int)(q % h);
    const double e = lamx[kx] + lamy[ky];
    const double2 z = C[q];
    C[q] = fabs(e) < 1e-12 ? make_double2(0.0, 0.0) : make_double2(z.x / e, z.y / e);
}

__global__ void k_per_tile(const double *__restrict__ red, int N, double scale,
                           double *__restrict__ out) {
    const long c = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (c >= (long)N * N) return;
    const int m = N - 1;
    out[c] = red[(long)((int)(c / N) % m) * m + (int)(c % N) % m] * scale;
}

// correction with the local or scalar density, BC by source cell, p accumulation
__global__ void k_per_correct(const double *__restrict__ as, const double *__restrict__ bs,
                              const double *__restrict__ gx, const double *__restrict__ gy,
                              const double *__restrict__ rho, double rho_s, double dt, int N,
                              int bc, double lid, const double *__restrict__ pc,
                              const double *__restrict__ p_prev, double *__restrict__ a,
                              double *__restrict__ b, double *__restrict__ p) {
    const long c = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (c >= (long)N * N) return;
    const BCSrc s = bc_source(bc, lid, (int)(c / N), (int)(c % N), N, N);
    auto cu = [&](long k) { return as[k] - (dt / (rho ? rho[k] : rho_s)) * gx[k]; };
    auto cv = [&](long k) { return bs[k] - (dt / (rho ? rho[k] : rho_s)) * gy[k]; };
    a[c] = s.u_const ? s.u_val : cu(s.u_src);
    b[c] = s.v_const ? s.v_val : cv(s.v_src);
    p[c] = p_prev ? p_prev[c] + pc[c] : pc[c];
}

// functions.py:1216-1233 on device buffers: rhs_full (N x N) -> p (N x N); rhs scaled by
// s / dt first when dt > 0
static int per_solve(rmt_ctx *ctx, const double *rhs, double s, double dt, double *p) {
    PerPlan *P = ctx->per;
    const int N = ctx->nx, m = P->m;
    const long nr = (long)m * m, nn = (long)N * N;
    hipStream_t st = ctx->stream;
    k_per_extract<<<grid1d(nr, 256), 256, 0, st>>>(rhs, N, s, dt, P->red);
    RMT_LAUNCHED();
    RMT_TRY(sub_mean_rows(ctx, P->red, m, m));                       // r -= mean(r)
    RMT_TRY(rfc(rocfft_execution_info_set_stream(P->info, st), "set_stream"));
    void *in[1] = {P->red}, *out[1] = {P->C};
    RMT_TRY(rfc(rocfft_execute(P->fwd, in, out, P->info), "execute fwd"));
    k_per_divide<<<grid1d((long)m * (m / 2 + 1), 256), 256, 0, st>>>((double2 *)P->C, m, P->lamx,
                                                                       P->lamy);
    RMT_LAUNCHED();
    void *in2[1] = {P->C}, *out2[1] = {P->red};
    RMT_TRY(rfc(rocfft_execute(P->inv, in2, out2, P->info), "execute inv"));
    k_per_tile<<<grid1d(nn, 256), 256, 0, st>>>(P->red, N, 1.0 / ((double)m * m), p);
    RMT_LAUNCHED();
    return sub_mean_rows(ctx, p, N, N);                              // p -= mean(p)
}

}  // namespace rmt

using namespace rmt;

extern "C" {

int rmt_divergence_periodic(rmt_ctx *ctx, const double *a, const double *b, double dx, double dy,
                            double *divU) {
    RMT_CHECK(ctx && a && b && divU && ctx->nx == ctx->ny && ctx->nx >= 3, RMT_EINVAL,
              "bad argument");
    const long n = (long)ctx->nx * ctx->nx;
    k_per_grad<<<grid1d(n, 256), 256, 0, ctx->stream>>>(a, b, ctx->nx, dx, dy, 0, divU, nullptr);
    RMT_LAUNCHED();
    return RMT_OK;
}

int rmt_pressure_gradient_periodic(rmt_ctx *ctx, const double *p, double dx, double dy,
                                   double *gx, double *gy) {
    RMT_CHECK(ctx && p && gx && gy && ctx->nx == ctx->ny && ctx->nx >= 3, RMT_EINVAL,
              "bad argument");
    const long n = (long)ctx->nx * ctx->nx;
    k_per_grad<<<grid1d(n, 256), 256, 0, ctx->stream>>>(p, p, ctx->nx, dx, dy, 1, gx, gy);
    RMT_LAUNCHED();
    return RMT_OK;
}

int rmt_solve_poisson_fft(rmt_ctx *ctx, const double *rhs, const double *lamx, const double *lamy,
                          double *p) {
    RMT_CHECK(ctx && rhs && lamx && lamy && p, RMT_EINVAL, "bad argument");
    RMT_TRY(per_plan(ctx, lamx, lamy));
    return per_solve(ctx, rhs, 1.0, 0.0, p);
}

int rmt_pressure_projection_periodic(rmt_ctx *ctx, const double *a_star, const double *b_star,
                                     double dx, double dy, double dt, double rho_bar,
                                     const double *rho_cells, int bc_kind, double lid,
                                     const double *lamx, const double *lamy,
                                     const double *p_prev, double *a, double *b, double *p) {
    RMT_CHECK(ctx && a_star && b_star && lamx && lamy && a && b && p, RMT_EINVAL, "bad argument");
    RMT_CHECK(bc_kind >= 0 && bc_kind <= 3, RMT_EINVAL, "unknown velocity bc kind");
    RMT_TRY(per_plan(ctx, lamx, lamy));
    PerPlan *P = ctx->per;
    const int N = ctx->nx;
    const long n = (long)N * N;
    RMT_TRY(ensure_scratch(ctx, n * sizeof(double)));
    double *div = P->g, *pc = ctx->scratch, *gx = P->g, *gy = P->g + n;
    k_per_grad<<<grid1d(n, 256), 256, 0, ctx->stream>>>(a_star, b_star, N, dx, dy, 0, div,
                                                        nullptr);
    RMT_LAUNCHED();
    RMT_TRY(per_solve(ctx, div, rho_bar, dt, pc));
    k_per_grad<<<grid1d(n, 256), 256, 0, ctx->stream>>>(pc, pc, N, dx, dy, 1, gx, gy);
    k_per_correct<<<grid1d(n, 256), 256, 0, ctx->stream>>>(a_star, b_star, gx, gy, rho_cells,
                                                           rho_bar, dt, N, bc_kind, lid, pc,
                                                           p_prev, a, b, p);
    RMT_LAUNCHED();
    return sub_mean_rows(ctx, p, N, N);
}

}  // extern "C"
