// poisson.hip -- functions.py:1091-1119 DCT-I Neumann Poisson solve on MI355X.
//
// p = idctn(dctn(rhs, type=1) / eig, type=1) - mean(p).  An unnormalised DCT-I of length
// n is the real part of the length-M = 2(n-1) real DFT of the even extension
// [x0 .. x_{n-1}, x_{n-2} .. x1] (the same construction pocketfft uses inside scipy).
// Each 2D transform = two rounds of {even-extend rows -> rocFFT batched R2C -> take the
// real part transposed through LDS}, so both rounds transform contiguous rows.  scipy's
// inverse DCT-I is the forward one scaled by 1/(2(n-1)) per axis.
#include "rmt_internal.hpp"
#include <vector>

namespace rmt {

struct DctPlan {
    int ny = 0, nx = 0;
    rocfft_plan px = nullptr, py = nullptr;
    rocfft_execution_info info = nullptr;
    void *work = nullptr;
    size_t work_bytes = 0;
    double *E = nullptr;      // even-extended rows (real)
    double *C = nullptr;      // R2C output (complex, interleaved)
    double *T = nullptr;      // transposed real plane
    double *lamx = nullptr, *lamy = nullptr;
    double dx = 0, dy = 0;
};

static bool g_rocfft_ready = false;

static int rf(rocfft_status s, const char *what) {
    if (s != rocfft_status_success) {
        set_error(std::string("rocFFT: ") + what + " failed (" + std::to_string((int)s) + ")");
        return RMT_EDEVICE;
    }
    return RMT_OK;
}

static int make_r2c(rocfft_plan *plan, size_t M, size_t batch) {
    rocfft_plan_description d = nullptr;
    RMT_TRY(rf(rocfft_plan_description_create(&d), "description_create"));
    size_t istr = 1, ostr = 1, idist = M, odist = M / 2 + 1;
    RMT_TRY(rf(rocfft_plan_description_set_data_layout(d, rocfft_array_type_real,
                                                       rocfft_array_type_hermitian_interleaved,
                                                       nullptr, nullptr, 1, &istr, idist, 1, &ostr,
                                                       odist), "set_data_layout"));
    int s = rf(rocfft_plan_create(plan, rocfft_placement_notinplace,
                                  rocfft_transform_type_real_forward, rocfft_precision_double, 1,
                                  &M, batch, d), "plan_create");
    rocfft_plan_description_destroy(d);
    return s;
}

void dct_destroy(DctPlan *P) {
    if (!P) return;
    if (P->px) rocfft_plan_destroy(P->px);
    if (P->py) rocfft_plan_destroy(P->py);
    if (P->info) rocfft_execution_info_destroy(P->info);
    hipFree(P->work); hipFree(P->E); hipFree(P->C); hipFree(P->T);
    hipFree(P->lamx); hipFree(P->lamy);
    delete P;
}

// functions.py:1091-1104: lam = -2 (1 - cos(pi k / (n-1))) / h**2, eig = lam_x + lam_y,
// eig[0,0] = 1.  (h**2 of a numpy float64 scalar is libm pow.)
static void host_lambda(int n, double h, std::vector<double> &lam) {
    lam.resize(n);
    double h2 = std::pow(h, 2.0);
    for (int k = 0; k < n; ++k) lam[k] = -2.0 * (1.0 - std::cos(M_PI * k / (n - 1))) / h2;
}

static int dct_plan(rmt_ctx *ctx, double dx, double dy) {
    DctPlan *P = ctx->dct;
    if (P && P->dx == dx && P->dy == dy) return RMT_OK;
    if (!g_rocfft_ready) { RMT_TRY(rf(rocfft_setup(), "setup")); g_rocfft_ready = true; }
    if (!P) {
        P = ctx->dct = new DctPlan;
        P->ny = ctx->ny; P->nx = ctx->nx;
        size_t Mx = 2 * (size_t)(P->nx - 1), My = 2 * (size_t)(P->ny - 1);
        RMT_TRY(make_r2c(&P->px, Mx, P->ny));
        if (P->ny == P->nx) P->py = nullptr;
        else RMT_TRY(make_r2c(&P->py, My, P->nx));
        size_t w1 = 0, w2 = 0;
        rocfft_plan_get_work_buffer_size(P->px, &w1);
        if (P->py) rocfft_plan_get_work_buffer_size(P->py, &w2);
        P->work_bytes = std::max(w1, w2);
        if (P->work_bytes) RMT_HIP(hipMalloc(&P->work, P->work_bytes));
        RMT_TRY(rf(rocfft_execution_info_create(&P->info), "execution_info_create"));
        if (P->work_bytes)
            RMT_TRY(rf(rocfft_execution_info_set_work_buffer(P->info, P->work, P->work_bytes),
                       "set_work_buffer"));
        size_t ne = std::max((size_t)P->ny * Mx, (size_t)P->nx * My);
        size_t n = (size_t)P->ny * P->nx;
        RMT_HIP(hipMalloc(&P->E, ne * sizeof(double)));
        RMT_HIP(hipMalloc(&P->C, 2 * n * sizeof(double)));
        RMT_HIP(hipMalloc(&P->T, n * sizeof(double)));
        RMT_HIP(hipMalloc(&P->lamx, P->nx * sizeof(double)));
        RMT_HIP(hipMalloc(&P->lamy, P->ny * sizeof(double)));
    }
    std::vector<double> lx, ly;
    host_lambda(P->nx, dx, lx);
    host_lambda(P->ny, dy, ly);
    RMT_HIP(hipMemcpy(P->lamx, lx.data(), lx.size() * 8, hipMemcpyHostToDevice));
    RMT_HIP(hipMemcpy(P->lamy, ly.data(), ly.size() * 8, hipMemcpyHostToDevice));
    P->dx = dx; P->dy = dy;
    return RMT_OK;
}

// E[r][k] = src[r][k] (k < n), src[r][M-k] (n <= k < M): even extension of each row.
__global__ void k_even_ext(const double *__restrict__ src, int rows, int n,
                           double *__restrict__ E) {
    const long M = 2L * (n - 1);
    long q = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (q >= (long)rows * M) return;
    long r = q / M, k = q % M;
    E[q] = src[r * n + (k < n ? k : M - k)];
}

// out[k][r] = scale * Re(C[r][k]) (/ (lamx[k] + lamy[r]) when lam given: the reference's
// eig[kj][ki] = lam_x[ki] + lam_y[kj], with (0,0) -> 1), LDS-tiled transpose.
constexpr int TT = 32;
__global__ void __launch_bounds__(TT * 8) k_real_T(const double *__restrict__ C, int rows, int n,
                                                   double scale, const double *__restrict__ lamr,
                                                   const double *__restrict__ lamk,
                                                   double *__restrict__ out) {
    __shared__ double tile[TT][TT + 1];
    int k0 = blockIdx.x * TT, r0 = blockIdx.y * TT;
    for (int rr = threadIdx.y; rr < TT; rr += 8) {
        int r = r0 + rr, k = k0 + threadIdx.x;
        if (r < rows && k < n) tile[rr][threadIdx.x] = C[2 * ((long)r * n + k)];
    }
    __syncthreads();
    for (int kk = threadIdx.y; kk < TT; kk += 8) {
        int k = k0 + kk, r = r0 + threadIdx.x;
        if (r < rows && k < n) {
            double v = tile[threadIdx.x][kk] * scale;
            if (lamr) {
                // orientation of this round: rows r = x-frequency ki, k = y-frequency kj
                double e = (k == 0 && r == 0) ? 1.0 : lamr[r] + lamk[k];
                v = v / e;
            }
            out[(long)k * rows + r] = v;
        }
    }
}

// One round along the rows of src (rows x n) -> out (n x rows).
static int round_rows(rmt_ctx *ctx, DctPlan *P, rocfft_plan plan, const double *src, int rows,
                      int n, double scale, const double *lamr, const double *lamk, double *out) {
    const long M = 2L * (n - 1);
    k_even_ext<<<grid1d((long)rows * M, 256), 256, 0, ctx->stream>>>(src, rows, n, P->E);
    RMT_LAUNCHED();
    RMT_TRY(rf(rocfft_execution_info_set_stream(P->info, ctx->stream), "set_stream"));
    void *in[1] = {P->E}, *o[1] = {P->C};
    RMT_TRY(rf(rocfft_execute(plan, in, o, P->info), "execute"));
    dim3 g((n + TT - 1) / TT, (rows + TT - 1) / TT);
    k_real_T<<<g, dim3(TT, 8), 0, ctx->stream>>>(P->C, rows, n, scale, lamr, lamk, out);
    RMT_LAUNCHED();
    return RMT_OK;
}

__global__ void k_sub_mean(double *__restrict__ x, long n, const double *__restrict__ s) {
    long k = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (k < n) x[k] = x[k] - *s;
}

int dct_solve(rmt_ctx *ctx, const double *rhs, double dx, double dy, double *p,
              const double *dev_mean_sub) {
    (void)dev_mean_sub;
    RMT_TRY(dct_plan(ctx, dx, dy));
    DctPlan *P = ctx->dct;
    const int ny = P->ny, nx = P->nx;
    rocfft_plan px = P->px, py = P->py ? P->py : P->px;
    // forward: along x (rows of rhs) -> T[ki][j]; along y -> p[kj][ki] / eig
    RMT_TRY(round_rows(ctx, P, px, rhs, ny, nx, 1.0, nullptr, nullptr, P->T));
    RMT_TRY(round_rows(ctx, P, py, P->T, nx, ny, 1.0, P->lamx, P->lamy, p));
    // inverse: same transform, scaled by 1/(2(n-1)) per axis
    RMT_TRY(round_rows(ctx, P, px, p, ny, nx, 1.0 / (2.0 * (nx - 1)), nullptr, nullptr, P->T));
    RMT_TRY(round_rows(ctx, P, py, P->T, nx, ny, 1.0 / (2.0 * (ny - 1)), nullptr, nullptr, p));
    const long n = (long)ny * nx;
    double *mean = ctx->red + RED_BLOCKS + 8;
    RMT_TRY(reduce_mean(ctx, p, n, mean));
    k_sub_mean<<<grid1d(n, 256), 256, 0, ctx->stream>>>(p, n, mean);
    RMT_LAUNCHED();
    return RMT_OK;
}

}  // namespace rmt
