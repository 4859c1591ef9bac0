// poisson.hip -- functions.py:1091-1119 DCT-I Neumann Poisson solve on MI355X.
//
// p = idctn(dctn(rhs, type=1) / eig, type=1) - mean(p).  An unnormalised DCT-I of length
// n is the length-M = 2(n-1) DFT of the even extension [x0 .. x_{n-1}, x_{n-2} .. x1]
// (the construction pocketfft uses inside scipy); that DFT is real, so TWO rows packed as
// the real and imaginary parts of one complex sequence come back separated in Re and Im.
// scipy's inverse DCT-I is the forward one scaled by 1/(2(n-1)) per axis.
//
// Main path (M <= 8192 and M = product of radices 2..31): k_dct1 -- one workgroup per row
// pair, the whole length-M complex sequence resident in LDS (<= 128 KB), a mixed-radix
// Stockham FFT with register-staged passes (read every butterfly input -> barrier ->
// twiddle + small DFT -> write -> barrier).  A 2D solve is five launches:
//   rows (x)  ->  transpose  ->  columns: DCT, / eig, inverse DCT, fused  ->  transpose
//   ->  rows (x, inverse).
// HBM traffic: 10 planes per solve.  Other sizes: rocFFT R2C rounds (the previous path).
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
    // LDS FFT path
    bool lds = false;
    int big = 0;                            // a radix above 13 present
    double2 *Wx = nullptr, *Wy = nullptr;   // e^{-2 pi i t / M} tables
    int radx[16] = {0}, rady[16] = {0}, npx = 0, npy = 0;
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
    hipFree(P->Wx); hipFree(P->Wy);
    delete P;
}

// functions.py:1091-1104: lam = -2 (1 - cos(pi k / (n-1))) / h**2, eig = lam_x + lam_y,
// eig[0,0] = 1.  (h**2 of a numpy float64 scalar is libm pow.)
static void host_lambda(int n, double h, std::vector<double> &lam) {
    lam.resize(n);
    double h2 = std::pow(h, 2.0);
    for (int k = 0; k < n; ++k) lam[k] = -2.0 * (1.0 - std::cos(M_PI * k / (n - 1))) / h2;
}

constexpr int DCT_T = 512;        // threads per row pair
constexpr int DCT_MAXM = 8192;    // complex LDS entries (128 KB)
constexpr int DCT_RCS = 98;       // 3 + 5 + 7 + 11 + 13 + 17 + 19 + 23 radix constants

// radices of M for the LDS FFT (4 for pairs of 2); false if a prime factor > 31 remains
static bool factor(int M, int *rad, int *np) {
    int n = 0, m = M;
    while (m % 4 == 0) { rad[n++] = 4; m /= 4; }
    for (int r : {2, 3, 5, 7, 11, 13, 17, 19, 23})
        while (m % r == 0) { if (n >= 16) return false; rad[n++] = r; m /= r; }
    *np = n;
    return m == 1 && M >= 2 && M <= DCT_MAXM;
}

// radix constants e^{-2 pi i t/R} for every supported odd radix, at these offsets
static const int kRcR[8] = {3, 5, 7, 11, 13, 17, 19, 23};
static int rc_offset(int R) {
    int o = 0;
    for (int r : kRcR) { if (r == R) return o; o += r; }
    return 0;
}

static int twiddles(int M, double2 **W) {
    const long double PI = 3.141592653589793238462643383279502884L;
    std::vector<double2> h(M + DCT_RCS);
    for (int t = 0; t < M; ++t) {
        long double a = 2.0L * PI * t / M;
        h[t] = make_double2((double)cosl(a), (double)-sinl(a));
    }
    int o = M;
    for (int R : kRcR)
        for (int t = 0; t < R; ++t, ++o) {
            long double a = 2.0L * PI * t / R;
            h[o] = make_double2((double)cosl(a), (double)-sinl(a));
        }
    RMT_HIP(hipMalloc(W, h.size() * sizeof(double2)));
    RMT_HIP(hipMemcpy(*W, h.data(), h.size() * sizeof(double2), hipMemcpyHostToDevice));
    return RMT_OK;
}

int dct_plan(rmt_ctx *ctx, double dx, double dy) {
    DctPlan *P = ctx->dct;
    if (P && P->dx == dx && P->dy == dy) return RMT_OK;
    if (!P) {
        P = ctx->dct = new DctPlan;
        P->ny = ctx->ny; P->nx = ctx->nx;
        const int Mx = 2 * (P->nx - 1), My = 2 * (P->ny - 1);
        static const bool force_rocfft = getenv("RMT_DCT_ROCFFT") && atoi(getenv("RMT_DCT_ROCFFT"));
        P->lds = !force_rocfft && factor(Mx, P->radx, &P->npx) && factor(My, P->rady, &P->npy);
        for (int k = 0; k < P->npx; ++k) P->big |= P->radx[k] > 13;
        for (int k = 0; k < P->npy; ++k) P->big |= P->rady[k] > 13;
    }
    if (!P->lds && !g_rocfft_ready) { RMT_TRY(rf(rocfft_setup(), "setup")); g_rocfft_ready = true; }
    if (P->lds && !P->Wx) {
        const size_t n = (size_t)P->ny * P->nx;
        RMT_TRY(twiddles(2 * (P->nx - 1), &P->Wx));
        RMT_TRY(twiddles(2 * (P->ny - 1), &P->Wy));
        RMT_HIP(hipMalloc(&P->T, n * sizeof(double)));
        RMT_HIP(hipMalloc(&P->lamx, P->nx * sizeof(double)));
        RMT_HIP(hipMalloc(&P->lamy, P->ny * sizeof(double)));
    }
    if (!P->lds && !P->px) {
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

// ---------------------------------------------------------------- LDS FFT path --
__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
    return make_double2(__builtin_fma(a.x, b.x, -a.y * b.y), __builtin_fma(a.x, b.y, a.y * b.x));
}
__device__ __forceinline__ double2 cadd(double2 a, double2 b) { return make_double2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ double2 csub(double2 a, double2 b) { return make_double2(a.x - b.x, a.y - b.y); }

// in-register DFT of length R (forward, e^{-2 pi i jm/R}); constants from the W table
template <int R>
__device__ __forceinline__ void small_dft(double2 (&v)[R], const double2 *rc) {
    if constexpr (R == 2) {
        const double2 a = v[0], b = v[1];
        v[0] = cadd(a, b); v[1] = csub(a, b);
    } else if constexpr (R == 4) {
        const double2 t0 = cadd(v[0], v[2]), t1 = csub(v[0], v[2]);
        const double2 t2 = cadd(v[1], v[3]), t3 = csub(v[1], v[3]);
        v[0] = cadd(t0, t2); v[2] = csub(t0, t2);
        v[1] = make_double2(t1.x + t3.y, t1.y - t3.x);   // t1 - i t3
        v[3] = make_double2(t1.x - t3.y, t1.y + t3.x);   // t1 + i t3
    } else {
        constexpr int K = (R - 1) / 2;
        double2 a[K], b[K];
        double2 x0 = v[0];
#pragma unroll
        for (int j = 1; j <= K; ++j) {
            a[j - 1] = cadd(v[j], v[R - j]);
            b[j - 1] = csub(v[j], v[R - j]);
            x0 = cadd(x0, a[j - 1]);
        }
#pragma unroll
        for (int m = 1; m <= K; ++m) {
            double2 A = v[0], S = make_double2(0.0, 0.0);
#pragma unroll
            for (int j = 1; j <= K; ++j) {
                const double2 w = rc[(j * m) % R];   // (cos, -sin) of 2 pi jm / R
                A.x = __builtin_fma(a[j - 1].x, w.x, A.x);
                A.y = __builtin_fma(a[j - 1].y, w.x, A.y);
                S.x = __builtin_fma(b[j - 1].x, -w.y, S.x);
                S.y = __builtin_fma(b[j - 1].y, -w.y, S.y);
            }
            v[m] = make_double2(A.x + S.y, A.y - S.x);        // A - i S
            v[R - m] = make_double2(A.x - S.y, A.y + S.x);    // A + i S
        }
        v[0] = x0;
    }
}

// Twiddles e^{-2 pi i t/M} as Wh[t >> 7] * Wl[t & 127] (both tables in LDS, <= 2 ulp)
struct Tw { const double2 *hi, *lo; };
__device__ __forceinline__ double2 tw(const Tw &T, int t) { return cmul(T.hi[t >> 7], T.lo[t & 127]); }

// Per pass: radix, Ns (product of the earlier radices), and 1/Ns for divide-free index math
struct Pass { int R, Ns; float inv; int rc; };   // rc: offset of this radix's constants
struct Radices { Pass p[16]; int n; };

// one Stockham pass of radix R over z[0..M)
template <int R>
__device__ __forceinline__ void fft_pass(double2 *z, int M, const Pass &ps, const Tw &T,
                                         const double2 *rcs) {
    constexpr int BPT = (DCT_MAXM / DCT_T + R - 1) / R;   // butterflies per thread (max)
    const int nb = M / R, tid = threadIdx.x, Ns = ps.Ns;
    const double2 *rc = rcs + ps.rc;
    double2 v[BPT][R];
#pragma unroll
    for (int b = 0; b < BPT; ++b) {
        const int j = tid + b * DCT_T;
        if (j < nb)
#pragma unroll
            for (int r = 0; r < R; ++r) v[b][r] = z[j + r * nb];
    }
    __syncthreads();
    const int tstep = M / (Ns * R);
#pragma unroll
    for (int b = 0; b < BPT; ++b) {
        const int j = tid + b * DCT_T;
        if (j < nb) {
            int g = (int)((float)j * ps.inv), k = j - g * Ns;   // j = g Ns + k
            if (k < 0) { --g; k += Ns; } else if (k >= Ns) { ++g; k -= Ns; }
            if (Ns > 1)
#pragma unroll
                for (int r = 1; r < R; ++r) v[b][r] = cmul(v[b][r], tw(T, k * r * tstep));
            small_dft<R>(v[b], rc);
            const int o = g * Ns * R + k;
#pragma unroll
            for (int r = 0; r < R; ++r) z[o + r * Ns] = v[b][r];
        }
    }
    __syncthreads();
}

// BIG = 0: radices 2..13; BIG = 1: up to 23 (one kernel holding every radix up to 31 spills,
// so 29 and 31 go to rocFFT)
template <int BIG>
__device__ void fft_lds(double2 *z, int M, const Radices &rd, const Tw &T, const double2 *rcs) {
    for (int q = 0; q < rd.n; ++q) {
        const Pass &ps = rd.p[q];
        switch (ps.R) {
            case 2: fft_pass<2>(z, M, ps, T, rcs); break;
            case 3: fft_pass<3>(z, M, ps, T, rcs); break;
            case 4: fft_pass<4>(z, M, ps, T, rcs); break;
            case 5: fft_pass<5>(z, M, ps, T, rcs); break;
            case 7: fft_pass<7>(z, M, ps, T, rcs); break;
            case 11: fft_pass<11>(z, M, ps, T, rcs); break;
            case 13: fft_pass<13>(z, M, ps, T, rcs); break;
            default:
                if constexpr (BIG) {
                    switch (ps.R) {
                        case 17: fft_pass<17>(z, M, ps, T, rcs); break;
                        case 19: fft_pass<19>(z, M, ps, T, rcs); break;
                        case 23: fft_pass<23>(z, M, ps, T, rcs); break;
                    }
                }
        }
    }
}

// even extension of the row pair (a, b) into z: z[j] = z[M - j] = (a_j, b_j)
__device__ __forceinline__ void put_even(double2 *z, int n, int M, int j, double a, double b) {
    z[j] = make_double2(a, b);
    if (j >= 1 && j <= n - 2) z[M - j] = make_double2(a, b);
}

// DCT-I along the rows of src (rows x n) -> dst, row pairs per workgroup.  SOLVE: rows are
// x-frequencies kx (transposed plane), and the column transform is forward DCT, / eig,
// inverse DCT (the eig of functions.py:1091-1104: lam_x[kx] + lam_y[ky], (0,0) -> 1).
template <bool SOLVE, int BIG>
__global__ void __launch_bounds__(DCT_T) k_dct1(const double *__restrict__ src,
                                                double *__restrict__ dst, int rows, int n,
                                                const double2 *__restrict__ W, Radices rd,
                                                double scale, const double *__restrict__ lamr,
                                                const double *__restrict__ lamk, int row0) {
    extern __shared__ double2 z[];
    __shared__ double2 twh[DCT_MAXM / 128], twl[128], rcs[DCT_RCS];
    const int M = 2 * (n - 1), rA = 2 * blockIdx.x, rB = rA + 1, tid = threadIdx.x;
    // tables: W has M + 192 entries: [0, M) e^{-2 pi i t/M}, then at M the small-radix constants
    if (tid < DCT_MAXM / 128) twh[tid] = (tid << 7) < M ? W[tid << 7] : make_double2(1.0, 0.0);
    if (tid < 128) twl[tid] = tid < M ? W[tid] : make_double2(1.0, 0.0);
    if (tid < DCT_RCS) rcs[tid] = W[M + tid];
    const Tw T{twh, twl};
    const bool hasB = rB < rows;
    const double *sa = src + (long)rA * n, *sb = src + (long)rB * n;
    for (int j = tid; j < n; j += DCT_T) put_even(z, n, M, j, sa[j], hasB ? sb[j] : 0.0);
    __syncthreads();
    fft_lds<BIG>(z, M, rd, T, rcs);
    if constexpr (SOLVE) {
        constexpr int PER = (4096 + DCT_T) / DCT_T;
        double2 q[PER];
#pragma unroll
        for (int t = 0; t < PER; ++t) {
            const int k = tid + t * DCT_T;
            if (k < n) {
                const double2 Z = z[k];
                // row0: global frequency of local row 0 (slab-decomposed solves)
                const double eA = (row0 + rA == 0 && k == 0) ? 1.0 : lamr[row0 + rA] + lamk[k];
                const double eB = hasB ? lamr[row0 + rB] + lamk[k] : 1.0;
                q[t] = make_double2(Z.x / eA, hasB ? Z.y / eB : 0.0);
            }
        }
        __syncthreads();
#pragma unroll
        for (int t = 0; t < PER; ++t) {
            const int k = tid + t * DCT_T;
            if (k < n) put_even(z, n, M, k, q[t].x, q[t].y);
        }
        __syncthreads();
        fft_lds<BIG>(z, M, rd, T, rcs);
    }
    double *da = dst + (long)rA * n, *db = dst + (long)rB * n;
    for (int k = tid; k < n; k += DCT_T) {
        const double2 Z = z[k];
        da[k] = Z.x * scale;
        if (hasB) db[k] = Z.y * scale;
    }
}

// out (C x R) = in (R x C) transposed, 64 x 64 tiles through LDS
__global__ void __launch_bounds__(256) k_transpose(const double *__restrict__ in, int R, int C,
                                                   double *__restrict__ out) {
    __shared__ double t[64][65];
    const int c0 = blockIdx.x * 64, r0 = blockIdx.y * 64, tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    for (int rr = ty; rr < 64; rr += 4) {
        const int r = r0 + rr, c = c0 + tx;
        if (r < R && c < C) t[rr][tx] = in[(long)r * C + c];
    }
    __syncthreads();
    for (int cc = ty; cc < 64; cc += 4) {
        const int c = c0 + cc, r = r0 + tx;
        if (r < R && c < C) out[(long)c * R + r] = t[tx][cc];
    }
}

static Radices radices(const int *rad, int np) {
    Radices rd{};
    int Ns = 1;
    for (int k = 0; k < np; ++k) {
        rd.p[k] = Pass{rad[k], Ns, (float)(1.0 / Ns), rc_offset(rad[k])};
        Ns *= rad[k];
    }
    rd.n = np;
    return rd;
}

// One LDS DCT-I pass over nrows rows of length n (axis 0: n = nx, axis 1: n = ny).  SOLVE
// (axis 1 only): forward, / eig, inverse, with rows = x-frequencies row0 .. row0 + nrows.
int dct_pass(rmt_ctx *ctx, bool solve, int axis, const double *src, double *dst, int nrows,
             int row0, double scale) {
    DctPlan *P = ctx->dct;
    RMT_CHECK(P && P->lds, RMT_ENOTSUP, "dct_pass: no LDS DCT plan for this grid");
    RMT_CHECK(!solve || axis == 1, RMT_EINVAL, "dct_pass: the solve pass runs along y");
    static bool attr = false;
    if (!attr) {
        const void *fs[4] = {(const void *)k_dct1<false, 0>, (const void *)k_dct1<true, 0>,
                             (const void *)k_dct1<false, 1>, (const void *)k_dct1<true, 1>};
        for (auto f : fs)
            RMT_HIP(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize,
                                        DCT_MAXM * 16));
        attr = true;
    }
    if (nrows <= 0) return RMT_OK;
    const int n = axis == 0 ? P->nx : P->ny;
    const Radices rd = axis == 0 ? radices(P->radx, P->npx) : radices(P->rady, P->npy);
    const double2 *W = axis == 0 ? P->Wx : P->Wy;
    const size_t lds = 2 * (size_t)(n - 1) * sizeof(double2);
    const unsigned g = (nrows + 1) / 2;
    hipStream_t st = ctx->stream;
    if (solve) {
        if (P->big) k_dct1<true, 1><<<g, DCT_T, lds, st>>>(src, dst, nrows, n, W, rd, scale, P->lamx, P->lamy, row0);
        else k_dct1<true, 0><<<g, DCT_T, lds, st>>>(src, dst, nrows, n, W, rd, scale, P->lamx, P->lamy, row0);
    } else {
        if (P->big) k_dct1<false, 1><<<g, DCT_T, lds, st>>>(src, dst, nrows, n, W, rd, scale, nullptr, nullptr, 0);
        else k_dct1<false, 0><<<g, DCT_T, lds, st>>>(src, dst, nrows, n, W, rd, scale, nullptr, nullptr, 0);
    }
    RMT_LAUNCHED();
    return RMT_OK;
}

bool dct_lds_ready(rmt_ctx *ctx) { return ctx->dct && ctx->dct->lds; }

void transpose(hipStream_t st, const double *in, int R, int C, double *out) {
    k_transpose<<<dim3((C + 63) / 64, (R + 63) / 64), 256, 0, st>>>(in, R, C, out);
}

static int dct_lds_solve(rmt_ctx *ctx, DctPlan *P, const double *rhs, double *p) {
    const int ny = P->ny, nx = P->nx;
    hipStream_t st = ctx->stream;
    // forward along x: p <- DCT_x(rhs) (p doubles as scratch), then T <- p^T (nx x ny)
    RMT_TRY(dct_pass(ctx, false, 0, rhs, p, ny, 0, 1.0));
    transpose(st, p, ny, nx, P->T);
    // columns: DCT_y, / eig, inverse DCT_y (scaled), in place on T
    RMT_TRY(dct_pass(ctx, true, 1, P->T, P->T, nx, 0, 1.0 / (2.0 * (ny - 1))));
    transpose(st, P->T, nx, ny, p);
    // inverse along x, in place
    RMT_TRY(dct_pass(ctx, false, 0, p, p, ny, 0, 1.0 / (2.0 * (nx - 1))));
    RMT_LAUNCHED();
    return RMT_OK;
}

int dct_solve(rmt_ctx *ctx, const double *rhs, double dx, double dy, double *p,
              const double *dev_mean_sub) {
    (void)dev_mean_sub;
    RMT_TRY(dct_plan(ctx, dx, dy));
    DctPlan *P = ctx->dct;
    const int ny = P->ny, nx = P->nx;
    if (P->lds) {
        RMT_TRY(dct_lds_solve(ctx, P, rhs, p));
    } else {
        rocfft_plan px = P->px, py = P->py ? P->py : P->px;
        // forward: along x (rows of rhs) -> T[ki][j]; along y -> p[kj][ki] / eig
        RMT_TRY(round_rows(ctx, P, px, rhs, ny, nx, 1.0, nullptr, nullptr, P->T));
        RMT_TRY(round_rows(ctx, P, py, P->T, nx, ny, 1.0, P->lamx, P->lamy, p));
        // inverse: same transform, scaled by 1/(2(n-1)) per axis
        RMT_TRY(round_rows(ctx, P, px, p, ny, nx, 1.0 / (2.0 * (nx - 1)), nullptr, nullptr, P->T));
        RMT_TRY(round_rows(ctx, P, py, P->T, nx, ny, 1.0 / (2.0 * (ny - 1)), nullptr, nullptr, p));
    }
    RMT_TRY(sub_mean_rows(ctx, p, ny, nx));
    return RMT_OK;
}


// ============================================================ DCT-II (MAC grid) ====
// mac.py:118-123 solves the cell-centred Neumann Poisson problem with an orthonormal
// DCT-II both ways.  The orthonormal scalings cancel between the forward and the inverse
// transform (they are diagonal per axis), so the solve runs the unnormalised pair
// y = D x (y_k = 2 sum_n x_n cos(pi k (2n+1) / 2N)) and x = D^-1 y: equal to rounding,
// like every FFT-based DCT against pocketfft's.  Makhoul's method: D x is 2 Re(w_k V_k),
// V = FFT_N of the even/odd-reordered x, w_k = e^{-i pi k/2N}; D^-1 builds
// V_k = 1/2 conj(w_k) (y_k - i y_{N-k}) and inverts the FFT.  Two rows share one complex
// FFT (their spectra separate by conjugate symmetry), the whole row resident in LDS.
//   MODE 0: forward along rows; 1: forward, / eig ((0,0) -> 0), inverse (fused column
//   solve); 2: inverse along rows.
__device__ __forceinline__ int mk_src(int m, int n) { return m < n / 2 ? 2 * m : 2 * (n - 1 - m) + 1; }

template <int MODE, int BIG>
__global__ void __launch_bounds__(DCT_T) k_dct2(const double *__restrict__ src,
                                                double *__restrict__ dst, int rows, int n,
                                                const double2 *__restrict__ W,
                                                const double2 *__restrict__ Wq, Radices rd,
                                                const double *__restrict__ lamr,
                                                const double *__restrict__ lamk, int row0,
                                                double scale) {
    extern __shared__ double2 z[];
    __shared__ double2 twh[DCT_MAXM / 128], twl[128], rcs[DCT_RCS];
    constexpr int PER = DCT_MAXM / DCT_T;
    const int rA = 2 * blockIdx.x, rB = rA + 1, tid = threadIdx.x;
    if (tid < DCT_MAXM / 128) twh[tid] = (tid << 7) < n ? W[tid << 7] : make_double2(1.0, 0.0);
    if (tid < 128) twl[tid] = tid < n ? W[tid] : make_double2(1.0, 0.0);
    if (tid < DCT_RCS) rcs[tid] = W[n + tid];
    const Tw T{twh, twl};
    const bool hasB = rB < rows;
    const double *sa = src + (long)rA * n, *sb = src + (long)rB * n;
    double *da = dst + (long)rA * n, *db = dst + (long)rB * n;
    if constexpr (MODE != 2) {
        for (int m = tid; m < n; m += DCT_T) {
            const int q = mk_src(m, n);
            z[m] = make_double2(sa[q], hasB ? sb[q] : 0.0);
        }
        __syncthreads();
        fft_lds<BIG>(z, n, rd, T, rcs);
        double2 y[PER];
#pragma unroll
        for (int t = 0; t < PER; ++t) {
            const int k = tid + t * DCT_T;
            if (k < n) {
                const double2 Zk = z[k], Zm = z[k ? n - k : 0], w = Wq[k];
                y[t].x = w.x * (Zk.x + Zm.x) - w.y * (Zk.y - Zm.y);
                y[t].y = w.x * (Zk.y + Zm.y) + w.y * (Zk.x - Zm.x);
                if constexpr (MODE == 1) {
                    y[t].x = (row0 + rA == 0 && k == 0) ? 0.0 : y[t].x / (lamr[row0 + rA] + lamk[k]);
                    y[t].y = hasB ? y[t].y / (lamr[row0 + rB] + lamk[k]) : 0.0;
                }
            }
        }
        if constexpr (MODE == 0) {
#pragma unroll
            for (int t = 0; t < PER; ++t) {
                const int k = tid + t * DCT_T;
                if (k < n) { da[k] = y[t].x * scale; if (hasB) db[k] = y[t].y * scale; }
            }
            return;
        }
        __syncthreads();
#pragma unroll
        for (int t = 0; t < PER; ++t) {
            const int k = tid + t * DCT_T;
            if (k < n) z[k] = y[t];
        }
    } else {
        for (int k = tid; k < n; k += DCT_T) z[k] = make_double2(sa[k], hasB ? sb[k] : 0.0);
    }
    __syncthreads();
    // inverse: conj(Z), Z_k = V^a_k + i V^b_k, V_k = 1/2 conj(w_k) (y_k - i y_{n-k})
    {
        double2 c[PER];
#pragma unroll
        for (int t = 0; t < PER; ++t) {
            const int k = tid + t * DCT_T;
            if (k < n) {
                const double2 Y = z[k], Ym = k ? z[n - k] : make_double2(0.0, 0.0);
                const double2 w = Wq[k];   // (cos, -sin); conj(w) = (cos, sin)
                const double cs = w.x, sn = -w.y;
                const double vax = 0.5 * (cs * Y.x + sn * Ym.x), vay = 0.5 * (sn * Y.x - cs * Ym.x);
                const double vbx = 0.5 * (cs * Y.y + sn * Ym.y), vby = 0.5 * (sn * Y.y - cs * Ym.y);
                c[t] = make_double2(vax - vby, -(vay + vbx));
            }
        }
        __syncthreads();
#pragma unroll
        for (int t = 0; t < PER; ++t) {
            const int k = tid + t * DCT_T;
            if (k < n) z[k] = c[t];
        }
    }
    __syncthreads();
    fft_lds<BIG>(z, n, rd, T, rcs);
    const double s = scale / n;
    for (int m = tid; m < n; m += DCT_T) {
        const double2 R = z[m];
        const int q = mk_src(m, n);
        da[q] = R.x * s;
        if (hasB) db[q] = -R.y * s;
    }
}

struct Dct2Plan {
    int ny = 0, nx = 0, big = 0;
    double dx = 0, dy = 0;
    int radx[16] = {0}, rady[16] = {0}, npx = 0, npy = 0;
    double2 *Wx = nullptr, *Wy = nullptr, *Qx = nullptr, *Qy = nullptr;
    double *lamx = nullptr, *lamy = nullptr, *T = nullptr;
};

void dct2_destroy(Dct2Plan *P) {
    if (!P) return;
    hipFree(P->Wx); hipFree(P->Wy); hipFree(P->Qx); hipFree(P->Qy);
    hipFree(P->lamx); hipFree(P->lamy); hipFree(P->T);
    delete P;
}

static int quarter_twiddles(int n, double2 **Q) {
    const long double PI = 3.141592653589793238462643383279502884L;
    std::vector<double2> h(n);
    for (int k = 0; k < n; ++k) {
        long double a = PI * k / (2.0L * n);
        h[k] = make_double2((double)cosl(a), (double)-sinl(a));
    }
    RMT_HIP(hipMalloc(Q, n * sizeof(double2)));
    RMT_HIP(hipMemcpy(*Q, h.data(), n * sizeof(double2), hipMemcpyHostToDevice));
    return RMT_OK;
}

// mac.py:104-115 eigenvalues per axis: -2 (1 - cos(pi k / n)) / h**2 (h**2: libm pow, as a
// Python float)
static void mac_lambda(int n, double h, std::vector<double> &lam) {
    lam.resize(n);
    const double h2 = std::pow(h, 2.0);
    for (int k = 0; k < n; ++k) lam[k] = -2.0 * (1.0 - std::cos(M_PI * k / n)) / h2;
}

int dct2_plan(rmt_ctx *ctx, int ny, int nx, double dx, double dy) {
    Dct2Plan *P = ctx->dct2;
    if (P && P->ny == ny && P->nx == nx && P->dx == dx && P->dy == dy) return RMT_OK;
    if (P) { dct2_destroy(P); ctx->dct2 = nullptr; }
    P = new Dct2Plan;
    P->ny = ny; P->nx = nx; P->dx = dx; P->dy = dy;
    if ((nx & 1) || (ny & 1) || !factor(nx, P->radx, &P->npx) || !factor(ny, P->rady, &P->npy)) {
        delete P;
        set_error("DCT-II solve: N must be even, <= 8192, and factor into radices <= 23");
        return RMT_ENOTSUP;
    }
    for (int k = 0; k < P->npx; ++k) P->big |= P->radx[k] > 13;
    for (int k = 0; k < P->npy; ++k) P->big |= P->rady[k] > 13;
    ctx->dct2 = P;
    RMT_TRY(twiddles(nx, &P->Wx));
    RMT_TRY(twiddles(ny, &P->Wy));
    RMT_TRY(quarter_twiddles(nx, &P->Qx));
    RMT_TRY(quarter_twiddles(ny, &P->Qy));
    std::vector<double> lx, ly;
    mac_lambda(nx, dx, lx);
    mac_lambda(ny, dy, ly);
    RMT_HIP(hipMalloc(&P->lamx, nx * sizeof(double)));
    RMT_HIP(hipMalloc(&P->lamy, ny * sizeof(double)));
    RMT_HIP(hipMemcpy(P->lamx, lx.data(), nx * 8, hipMemcpyHostToDevice));
    RMT_HIP(hipMemcpy(P->lamy, ly.data(), ny * 8, hipMemcpyHostToDevice));
    RMT_HIP(hipMalloc(&P->T, (size_t)nx * ny * sizeof(double)));
    static bool attr = false;
    if (!attr) {
        const void *fs[6] = {(const void *)k_dct2<0, 0>, (const void *)k_dct2<1, 0>,
                             (const void *)k_dct2<2, 0>, (const void *)k_dct2<0, 1>,
                             (const void *)k_dct2<1, 1>, (const void *)k_dct2<2, 1>};
        for (auto f : fs)
            RMT_HIP(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize,
                                        DCT_MAXM * 16));
        attr = true;
    }
    return RMT_OK;
}

// one DCT-II pass over nrows rows along axis (0: length nx, 1: length ny; MODE 1 needs 1)
int dct2_pass(rmt_ctx *ctx, int mode, int axis, const double *src, double *dst,
                     int nrows, int row0) {
    Dct2Plan *P = ctx->dct2;
    const int n = axis == 0 ? P->nx : P->ny;
    const Radices rd = axis == 0 ? radices(P->radx, P->npx) : radices(P->rady, P->npy);
    const double2 *W = axis == 0 ? P->Wx : P->Wy, *Q = axis == 0 ? P->Qx : P->Qy;
    const size_t lds = (size_t)n * sizeof(double2);
    const unsigned g = (nrows + 1) / 2;
    hipStream_t st = ctx->stream;
#define DCT2_L(M, B) k_dct2<M, B><<<g, DCT_T, lds, st>>>(src, dst, nrows, n, W, Q, rd, P->lamx, P->lamy, row0, 1.0)
    if (P->big) {
        if (mode == 0) DCT2_L(0, 1); else if (mode == 1) DCT2_L(1, 1); else DCT2_L(2, 1);
    } else {
        if (mode == 0) DCT2_L(0, 0); else if (mode == 1) DCT2_L(1, 0); else DCT2_L(2, 0);
    }
#undef DCT2_L
    RMT_LAUNCHED();
    return RMT_OK;
}

// the caller's eigenvalues (eig = lam_x[None, :] + lam_y[:, None] of mac.py:104-115)
int dct2_set_lambda(rmt_ctx *ctx, const double *lamx, const double *lamy) {
    Dct2Plan *P = ctx->dct2;
    RMT_CHECK(P, RMT_EINVAL, "dct2_set_lambda: no plan");
    RMT_HIP(hipMemcpyAsync(P->lamx, lamx, P->nx * 8, hipMemcpyHostToDevice, ctx->stream));
    RMT_HIP(hipMemcpyAsync(P->lamy, lamy, P->ny * 8, hipMemcpyHostToDevice, ctx->stream));
    RMT_HIP(hipStreamSynchronize(ctx->stream));
    P->dx = P->dy = -1.0;   // next dct2_plan call recomputes the reference's own values
    return RMT_OK;
}

// mac.py:118-123: p = D^-1 (D rhs / eig), (0,0) -> 0; rhs and p are (ny, nx), may alias
int dct2_solve(rmt_ctx *ctx, const double *rhs, double *p) {
    Dct2Plan *P = ctx->dct2;
    RMT_CHECK(P, RMT_EINVAL, "dct2_solve: no plan");
    const int ny = P->ny, nx = P->nx;
    RMT_TRY(dct2_pass(ctx, 0, 0, rhs, p, ny, 0));
    transpose(ctx->stream, p, ny, nx, P->T);
    RMT_TRY(dct2_pass(ctx, 1, 1, P->T, P->T, nx, 0));
    transpose(ctx->stream, P->T, nx, ny, p);
    return dct2_pass(ctx, 2, 0, p, p, ny, 0);
}
}  // namespace rmt
