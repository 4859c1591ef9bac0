// poisson.hip -- functions.py:1091-1119 DCT-I Neumann Poisson solve on MI355X.
//
// p = idctn(dctn(rhs, type=1) / eig, type=1) - mean(p).  An unnormalised DCT-I of length
// n is the length-M = 2(n-1) DFT of the even extension [x0 .. x_{n-1}, x_{n-2} .. x1]
// (the construction pocketfft uses inside scipy); that DFT is real, so TWO rows packed as
// the real and imaginary parts of one complex sequence come back separated in Re and Im.
// scipy's inverse DCT-I is the forward one scaled by 1/(2(n-1)) per axis.
//
// Main path (n - 1 < 4096, a product of radices 2..23, 29, 31 -- the last two as matrix-form
// passes, fft_pass_mat): k_dct1 -- one workgroup per row,
// the row's even extension packed as a length-(n-1) complex sequence resident in LDS
// (<= 64 KB, two workgroups per CU), a mixed-radix Stockham FFT (radices grouped into
// in-register composite butterflies of up to 10; twiddles from a global per-pass table),
// then the packed-real split into the DCT-I.  A 2D solve is five launches:
//   rows (x)  ->  transpose  ->  columns: DCT, / eig, inverse DCT, fused  ->  transpose
//   ->  rows (x, inverse, + the row sums of the mean).
// HBM traffic: 10 planes per solve.  Reading the columns in place instead of transposing
// (strided, XCD-grouped workgroups) measured slower: 380 us for the fused column pass
// against 63 + 234 + 43 us with the transposes.  Other sizes: rocFFT R2C rounds.
#include "rmt_internal.hpp"
#include "dft_consts.hpp"
#include <algorithm>
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
    int mat = 0;                            // a matrix-form radix (29, 31) present
    double2 *Wx = nullptr, *Wy = nullptr;   // per-pass twiddle tables (twiddles())
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
    (void)hipFree(P->work); (void)hipFree(P->E); (void)hipFree(P->C); (void)hipFree(P->T);
    (void)hipFree(P->lamx); (void)hipFree(P->lamy);
    (void)hipFree(P->Wx); (void)hipFree(P->Wy);
    delete P;
}

// functions.py:1091-1104: lam = -2 (1 - cos(pi k / (n-1))) / h**2, eig = lam_x + lam_y,
// eig[0,0] = 1.  (h**2 of a numpy float64 scalar is libm pow.)
static void host_lambda(int n, double h, std::vector<double> &lam) {
    lam.resize(n);
    double h2 = std::pow(h, 2.0);
    for (int k = 0; k < n; ++k) lam[k] = -2.0 * (1.0 - std::cos(M_PI * k / (n - 1))) / h2;
}

constexpr int DCT_MAXM = 8192;    // complex LDS entries (128 KB)
constexpr int K1_MAXN = DCT_MAXM / 2;   // k_dct1's complex FFT length (n <= 4097)

// Radix plan of a length-M FFT: prime factors (2 .. 23), then 2s grouped into 8 / 4, 3s into
// 9, a leftover 2 with a 5 (10) or a 3 (6): M = 8190 = 2 3^2 5 7 13 runs as 9, 10, 7, 13 --
// four LDS passes instead of six.  mat: also 29 and 31, as matrix-form passes (fft_pass_mat;
// k_dct1 only).  false if a prime factor > 23 (> 31 with mat) remains.
static bool is_mat_radix(int R) { return R == 29 || R == 31; }
static bool factor(int M, int *rad, int *np, bool mat = false, bool desc = false) {
    if (M < 2 || M > DCT_MAXM) return false;
    int cnt[32] = {0}, m = M;
    for (int q : {2, 3, 5, 7, 11, 13, 17, 19, 23})
        while (m % q == 0) { ++cnt[q]; m /= q; }
    if (mat)
        for (int q : {29, 31})
            while (m % q == 0) { ++cnt[q]; m /= q; }
    if (m != 1) return false;
    int n = 0;
    auto put = [&](int r) { if (n < 16) rad[n++] = r; };
    while (cnt[2] >= 3) { put(8); cnt[2] -= 3; }
    if (cnt[2] == 2) { put(4); cnt[2] = 0; }
    while (cnt[3] >= 2) { put(9); cnt[3] -= 2; }
    if (cnt[2] && cnt[5]) { put(10); --cnt[2]; --cnt[5]; }
    if (cnt[2] && cnt[3]) { put(6); --cnt[2]; --cnt[3]; }
    for (int q : {2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31})
        while (cnt[q]) { put(q); --cnt[q]; }
    // ascending: the largest radix runs last, where Ns (the base-twiddle count) is M / R
    std::sort(rad, rad + n);
    if (desc) std::reverse(rad, rad + n);
    *np = n;
    return n < 16;
}

static bool big_radix(const int *rad, int np) {
    for (int k = 0; k < np; ++k) if (rad[k] > 13 && !is_mat_radix(rad[k])) return true;
    return false;
}
static bool mat_radix(const int *rad, int np) {
    for (int k = 0; k < np; ++k) if (is_mat_radix(rad[k])) return true;
    return false;
}

// Twiddles of the Stockham passes, in pass order: pass (R, Ns) holds e^{-2 pi i k r / (Ns R)}
// at [(r - 1) Ns + k], r = 1 .. R-1, k < Ns (M - 1 entries in all, L2-resident: every
// workgroup reads the same table), from long double, exact where k r / (Ns R) is a multiple
// of 1/4.  post: then k_dct1's packed-real split factors e^{-2 pi i k / (2M)}, k = 0 .. M.
static double2 unit_root(long t, long L) {
    const long double PI = 3.141592653589793238462643383279502884L;
    t %= L;
    if ((4 * t) % L == 0) {
        const int e = (int)(4 * t / L);
        const double c[4] = {1.0, 0.0, -1.0, 0.0}, sn[4] = {0.0, 1.0, 0.0, -1.0};
        return make_double2(c[e], -sn[e]);
    }
    const long double a = 2.0L * PI * t / L;
    return make_double2((double)cosl(a), (double)-sinl(a));
}
static int twiddles(int M, const int *rad, int np, double2 **W, bool post = false) {
    std::vector<double2> h;
    h.reserve(2 * (size_t)M + 2);
    int Ns = 1;
    for (int q = 0; q < np; ++q) {
        const int R = rad[q], L = Ns * R;
        for (int r = 1; r < R; ++r)
            for (int k = 0; k < Ns; ++k) h.push_back(unit_root((long)k * r, L));
        Ns = L;
    }
    if (post)
        for (long k = 0; k <= M; ++k) h.push_back(unit_root(k, 2L * M));
    h.push_back(make_double2(1.0, 0.0));
    RMT_HIP(hipMalloc(W, h.size() * sizeof(double2)));
    RMT_UPLOAD(*W, h.data(), h.size() * sizeof(double2));
    return RMT_OK;
}

// LDS budget of one FFT workgroup: the length-M sequence + 4 KB static
constexpr size_t FFT_LDS_MAX = 160 * 1024 - 4096;
static bool lds_fits(int M) { return (size_t)M * sizeof(double2) <= FFT_LDS_MAX; }

int dct_plan(rmt_ctx *ctx, double dx, double dy) {
    DctPlan *P = ctx->dct;
    if (P && P->dx == dx && P->dy == dy) return RMT_OK;
    if (!P) {
        P = ctx->dct = new DctPlan;
        P->ny = ctx->ny; P->nx = ctx->nx;
        // k_dct1's complex FFT length: N = n - 1 (half the even extension)
        const int Nx = P->nx - 1, Ny = P->ny - 1;
        P->lds = !ctx->opt.dct_rocfft && Nx >= 2 && Ny >= 2 && Nx < K1_MAXN && Ny < K1_MAXN &&
                 factor(Nx, P->radx, &P->npx, true, ctx->opt.dct_desc && Nx == 4095) &&
                 factor(Ny, P->rady, &P->npy, true, ctx->opt.dct_desc && Ny == 4095) &&
                 lds_fits(Nx) && lds_fits(Ny);
        P->big = big_radix(P->radx, P->npx) || big_radix(P->rady, P->npy);
        P->mat = mat_radix(P->radx, P->npx) || mat_radix(P->rady, P->npy);
        // (a matrix pass needs a second length-M buffer: both planes within the LDS budget)
        if (P->mat) P->lds = P->lds && lds_fits(2 * Nx + 64) && lds_fits(2 * Ny + 64);
    }
    if (!P->lds && !g_rocfft_ready) { RMT_TRY(rf(rocfft_setup(), "setup")); g_rocfft_ready = true; }
    if (P->lds && !P->Wx) {
        const size_t n = (size_t)P->ny * P->nx;
        RMT_TRY(twiddles(P->nx - 1, P->radx, P->npx, &P->Wx, true));
        RMT_TRY(twiddles(P->ny - 1, P->rady, P->npy, &P->Wy, true));
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
    RMT_UPLOAD(P->lamx, lx.data(), lx.size() * 8);
    RMT_UPLOAD(P->lamy, ly.data(), ly.size() * 8);
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
// Threads per workgroup: 1024 (16 waves, 128 VGPRs) for radices up to 13; 512 when a radix
// 17 / 19 / 23 pass is in the plan (its butterfly alone holds ~45 complex values).
template <int BIG> struct FftT { static constexpr int T = BIG ? 512 : 1024; };

__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
    return make_double2(__builtin_fma(a.x, b.x, -a.y * b.y), __builtin_fma(a.x, b.y, a.y * b.x));
}
__device__ __forceinline__ double2 cadd(double2 a, double2 b) { return make_double2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ double2 csub(double2 a, double2 b) { return make_double2(a.x - b.x, a.y - b.y); }

// a * e^{-2 pi i t / R}, t a constant after unrolling (exact for multiples of R / 4)
template <int R>
__device__ __forceinline__ double2 wmul(double2 a, int t) {
    t %= R;
    if (t == 0) return a;
    if (4 * t == R) return make_double2(a.y, -a.x);
    if (2 * t == R) return make_double2(-a.x, -a.y);
    if (4 * t == 3 * R) return make_double2(-a.y, a.x);
    const double c = Rc<R>::c[t], sn = Rc<R>::s[t];
    return make_double2(__builtin_fma(a.x, c, a.y * sn), __builtin_fma(a.y, c, -(a.x * sn)));
}

constexpr bool is_prime(int R) {
    for (int d = 2; d * d <= R; ++d) if (R % d == 0) return false;
    return R >= 2;
}
// first factor of a composite radix: 8 = 2 x 4, 9 = 3 x 3, 10 = 2 x 5, 6 = 2 x 3, 4 = 2 x 2
constexpr int split(int R) { return R % 2 == 0 ? 2 : 3; }

// forward DFT of length R in registers (e^{-2 pi i n k / R}), constants from dft_consts.hpp
template <int R>
__device__ __forceinline__ void dft(double2 *v) {
    if constexpr (R == 2) {
        const double2 a = v[0], b = v[1];
        v[0] = cadd(a, b); v[1] = csub(a, b);
    } else if constexpr (R == 4) {
        const double2 t0 = cadd(v[0], v[2]), t1 = csub(v[0], v[2]);
        const double2 t2 = cadd(v[1], v[3]), t3 = csub(v[1], v[3]);
        v[0] = cadd(t0, t2); v[2] = csub(t0, t2);
        v[1] = make_double2(t1.x + t3.y, t1.y - t3.x);   // t1 - i t3
        v[3] = make_double2(t1.x - t3.y, t1.y + t3.x);   // t1 + i t3
    } else if constexpr (is_prime(R)) {
        // odd prime: X_m = A_m -/+ i S_m from the symmetric / antisymmetric input pairs
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
                const double c = Rc<R>::c[(j * m) % R], sn = Rc<R>::s[(j * m) % R];
                A.x = __builtin_fma(a[j - 1].x, c, A.x);
                A.y = __builtin_fma(a[j - 1].y, c, A.y);
                S.x = __builtin_fma(b[j - 1].x, sn, S.x);
                S.y = __builtin_fma(b[j - 1].y, sn, S.y);
            }
            v[m] = make_double2(A.x + S.y, A.y - S.x);        // A - i S
            v[R - m] = make_double2(A.x - S.y, A.y + S.x);    // A + i S
        }
        v[0] = x0;
    } else {
        // R = A B: n = B n1 + n2, k = k1 + A k2; DFT_A over n1, twiddle w_R^{n2 k1}, DFT_B
        constexpr int A = split(R), B = R / A;
        double2 y[R];
#pragma unroll
        for (int n2 = 0; n2 < B; ++n2) {
            double2 t[A];
#pragma unroll
            for (int n1 = 0; n1 < A; ++n1) t[n1] = v[B * n1 + n2];
            dft<A>(t);
#pragma unroll
            for (int k1 = 0; k1 < A; ++k1) y[n2 * A + k1] = wmul<R>(t[k1], n2 * k1);
        }
#pragma unroll
        for (int k1 = 0; k1 < A; ++k1) {
            double2 t[B];
#pragma unroll
            for (int n2 = 0; n2 < B; ++n2) t[n2] = y[n2 * A + k1];
            dft<B>(t);
#pragma unroll
            for (int k2 = 0; k2 < B; ++k2) v[k1 + A * k2] = t[k2];
        }
    }
}

// Per pass: radix, Ns (product of the earlier radices), 1/Ns for divide-free index math, and
// the offset of the pass's twiddles in the table
struct Pass { int R, Ns; float inv; int tw; };
struct Radices { Pass p[16]; int n; };

// one Stockham pass of radix R over z[0..M): load every butterfly's twiddles (global table,
// issued first) and inputs, twiddle them -> barrier -> DFT_R -> write -> barrier
template <int R, int NT, int MAXN>
__device__ __forceinline__ void fft_pass(double2 *z, int M, const Pass &ps,
                                         const double2 *__restrict__ tw) {
    constexpr int BPT = (MAXN / R + NT - 1) / NT;      // butterflies per thread (max)
    const int nb = M / R, Ns = ps.Ns;
    // opaque per pass: the per-thread addresses below are not hoisted out of a caller's loop
    // (k_dct1's two transforms), where they would hold registers across every pass
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    double2 v[BPT][R];
    int o[BPT];
#pragma unroll
    for (int b = 0; b < BPT; ++b) {
        const int j = tid + b * NT;
        if (j < nb) {
            int g = (int)((float)j * ps.inv), k = j - g * Ns;   // j = g Ns + k
            if (k < 0) { --g; k += Ns; } else if (k >= Ns) { ++g; k -= Ns; }
            o[b] = g * Ns * R + k;
            double2 w[R - 1];
            if (Ns > 1) {
                const double2 *t = tw + ps.tw + k;
#pragma unroll
                for (int r = 1; r < R; ++r) w[r - 1] = t[(r - 1) * Ns];
            }
#pragma unroll
            for (int r = 0; r < R; ++r) v[b][r] = z[j + r * nb];
            if (Ns > 1)
#pragma unroll
                for (int r = 1; r < R; ++r) v[b][r] = cmul(v[b][r], w[r - 1]);
        }
    }
    __syncthreads();
#pragma unroll
    for (int b = 0; b < BPT; ++b) {
        const int j = tid + b * NT;
        if (j < nb) {
            dft<R>(v[b]);
#pragma unroll
            for (int r = 0; r < R; ++r) z[o[b] + r * Ns] = v[b][r];
        }
    }
    __syncthreads();
}

// A Stockham pass of an odd prime radix R too large for one butterfly per thread (29, 31:
// the radix-31 pass of M = 1023 has 33 butterflies, and a register butterfly holds 31 complex
// values), in matrix form: every (butterfly, input) pair stages its twiddled input in t, then
// every (butterfly, output pair m / R - m) forms dft<R>'s sums A_m, S_m from them -- the same
// operations in the same order as dft<R>, spread over the workgroup.  t: M + R complex LDS
// entries after z (the R roots of unity at t + M).
template <int R, int NT>
__device__ void fft_pass_mat(double2 *z, int M, const Pass &ps, const double2 *__restrict__ tw,
                             double2 *t) {
    constexpr int K = (R - 1) / 2;
    const int nb = M / R, Ns = ps.Ns;
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    double2 *cs = t + M;
    if (tid < R) cs[tid] = make_double2(Rc<R>::c[tid], Rc<R>::s[tid]);
    for (int q = tid; q < nb * R; q += NT) {
        const int j = q / R, r = q - j * R;
        double2 v = z[j + r * nb];
        if (Ns > 1 && r > 0) {
            const int k = j % Ns;
            v = cmul(v, tw[ps.tw + (r - 1) * Ns + k]);
        }
        t[q] = v;
    }
    __syncthreads();
    for (int q = tid; q < nb * (K + 1); q += NT) {
        const int j = q / (K + 1), m = q - j * (K + 1);
        const double2 *v = t + j * R;
        const int g = j / Ns, k = j - g * Ns, o = g * Ns * R + k;
        if (m == 0) {
            double2 x0 = v[0];
            for (int i = 1; i <= K; ++i) x0 = cadd(x0, cadd(v[i], v[R - i]));
            z[o] = x0;
        } else {
            double2 A = v[0], S = make_double2(0.0, 0.0);
            int e = 0;
            for (int i = 1; i <= K; ++i) {
                e += m;
                if (e >= R) e -= R;   // (i m) mod R
                const double2 a = cadd(v[i], v[R - i]), b = csub(v[i], v[R - i]), w = cs[e];
                A.x = __builtin_fma(a.x, w.x, A.x);
                A.y = __builtin_fma(a.y, w.x, A.y);
                S.x = __builtin_fma(b.x, w.y, S.x);
                S.y = __builtin_fma(b.y, w.y, S.y);
            }
            z[o + m * Ns] = make_double2(A.x + S.y, A.y - S.x);         // A - i S
            z[o + (R - m) * Ns] = make_double2(A.x - S.y, A.y + S.x);   // A + i S
        }
    }
    __syncthreads();
}

// the radix passes of rd over z[0..M), M <= MAXN, NT threads (scr: fft_pass_mat's buffer)
template <int BIG, int NT, int MAXN>
__device__ void fft_lds(double2 *z, int M, const Radices &rd, const double2 *__restrict__ tw,
                        double2 *scr = nullptr) {
    for (int q = 0; q < rd.n; ++q) {
        const Pass &ps = rd.p[q];
        switch (ps.R) {
            case 2: fft_pass<2, NT, MAXN>(z, M, ps, tw); break;
            case 3: fft_pass<3, NT, MAXN>(z, M, ps, tw); break;
            case 4: fft_pass<4, NT, MAXN>(z, M, ps, tw); break;
            case 5: fft_pass<5, NT, MAXN>(z, M, ps, tw); break;
            case 6: fft_pass<6, NT, MAXN>(z, M, ps, tw); break;
            case 7: fft_pass<7, NT, MAXN>(z, M, ps, tw); break;
            case 8: fft_pass<8, NT, MAXN>(z, M, ps, tw); break;
            case 9: fft_pass<9, NT, MAXN>(z, M, ps, tw); break;
            case 10: fft_pass<10, NT, MAXN>(z, M, ps, tw); break;
            case 11: fft_pass<11, NT, MAXN>(z, M, ps, tw); break;
            case 13: fft_pass<13, NT, MAXN>(z, M, ps, tw); break;
            case 29: fft_pass_mat<29, NT>(z, M, ps, tw, scr); break;
            case 31: fft_pass_mat<31, NT>(z, M, ps, tw, scr); break;
            default:
                if constexpr (BIG) {
                    switch (ps.R) {
                        case 17: fft_pass<17, NT, MAXN>(z, M, ps, tw); break;
                        case 19: fft_pass<19, NT, MAXN>(z, M, ps, tw); break;
                        case 23: fft_pass<23, NT, MAXN>(z, M, ps, tw); break;
                    }
                }
        }
    }
}

// The same Stockham pass with the radix, Ns and length known at compile time (the n = 4096
// plan, M = 4095 = 5 7 9 13): constant index math, no pass switch, the same arithmetic in the
// same order as fft_pass (bit-identical results)
template <int R, int NS, int NT, int M>
__device__ __forceinline__ void fft_pass_k(double2 *z, const double2 *__restrict__ tw) {
    constexpr int NB = M / R, BPT = (NB + NT - 1) / NT;
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    double2 v[BPT][R];
    int o[BPT];
#pragma unroll
    for (int b = 0; b < BPT; ++b) {
        const int j = tid + b * NT;
        if (j < NB) {
            const int g = j / NS, k = j - g * NS;
            o[b] = g * NS * R + k;
            double2 w[R - 1];
            if constexpr (NS > 1) {
#pragma unroll
                for (int r = 1; r < R; ++r) w[r - 1] = tw[(r - 1) * NS + k];
            }
#pragma unroll
            for (int r = 0; r < R; ++r) v[b][r] = z[j + r * NB];
            if constexpr (NS > 1) {
#pragma unroll
                for (int r = 1; r < R; ++r) v[b][r] = cmul(v[b][r], w[r - 1]);
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int b = 0; b < BPT; ++b) {
        const int j = tid + b * NT;
        if (j < NB) {
            dft<R>(v[b]);
#pragma unroll
            for (int r = 0; r < R; ++r) z[o[b] + r * NS] = v[b][r];
        }
    }
    __syncthreads();
}
// factor(4095)'s plan: radices 5, 7, 9, 13 (ascending), twiddle offsets 0, 4, 34, 314
template <int NT>
__device__ __forceinline__ void fft_4095(double2 *z, const double2 *__restrict__ W) {
    fft_pass_k<5, 1, NT, 4095>(z, W);
    fft_pass_k<7, 5, NT, 4095>(z, W + 4);
    fft_pass_k<9, 35, NT, 4095>(z, W + 34);
    fft_pass_k<13, 315, NT, 4095>(z, W + 314);
}
// descending (dct_desc): 13, 9, 7, 5, twiddle offsets 0, 12, 116, 818 -- the radix-13
// butterflies need no twiddles (Ns = 1), the radix-5 pass takes the large table
template <int NT>
__device__ __forceinline__ void fft_4095d(double2 *z, const double2 *__restrict__ W) {
    fft_pass_k<13, 1, NT, 4095>(z, W);
    fft_pass_k<9, 13, NT, 4095>(z, W + 12);
    fft_pass_k<7, 117, NT, 4095>(z, W + 116);
    fft_pass_k<5, 819, NT, 4095>(z, W + 818);
}

// DCT-I of one real row per workgroup.  The even extension e (length M = 2N, N = n - 1) is
// real, so its length-M DFT -- the unnormalised DCT-I -- comes from ONE length-N complex FFT
// of z_m = e_{2m} + i e_{2m+1} (the packed-real FFT): with Z = FFT_N(z), Z_N = Z_0 and
// W^k = e^{-2 pi i k / M} = c_k - i s_k,
//   X_k     = (S + c_k T - s_k D) / 2,   X_{N-k} = (S - c_k T + s_k D) / 2,
//   S = Re Z_k + Re Z_{N-k},  D = Re Z_k - Re Z_{N-k},  T = Im Z_k + Im Z_{N-k}.
// Read as doubles, z IS e (d[j] = e_j), so packing is the even extension itself.  N complex
// entries = 64 KB for n = 4096: two workgroups share a CU, one's HBM traffic hiding behind
// the other's LDS passes.  SOLVE: rows are x-frequencies kx of the transposed plane; forward
// DCT, / eig (functions.py:1091-1104: lam_x[kx] + lam_y[ky], (0,0) -> 1), inverse DCT.
// (launch bounds: two workgroups per CU -- 4 waves per SIMD at 512 threads, 128 VGPRs)
template <int BIG> struct K1T { static constexpr int T = BIG ? 256 : 512; };

// every load issued before the first LDS write: a dynamic-trip loop here compiled to one
// HBM round trip per iteration (load, wait, write), ~8 serial misses per row
template <int NT>
__device__ __forceinline__ void put_row_even(double *d, int N, const double *__restrict__ x) {
    constexpr int L = (K1_MAXN + NT) / NT;   // j <= N <= K1_MAXN
    double v[L];
#pragma unroll
    for (int t = 0; t < L; ++t) {
        const int j = threadIdx.x + t * NT;
        if (j <= N) v[t] = x[j];
    }
#pragma unroll
    for (int t = 0; t < L; ++t) {
        const int j = threadIdx.x + t * NT;
        if (j <= N) {
            d[j] = v[t];
            if (j >= 1 && j < N) d[2 * N - j] = v[t];
        }
    }
}

template <bool SOLVE, int BIG, int PLAN = 0>
__global__ void __launch_bounds__(K1T<BIG>::T, BIG ? 2 : 4) k_dct1(const double *__restrict__ src,
                                                      double *__restrict__ dst, int rows, int n,
                                                      const double2 *__restrict__ W,
                                                      Radices rd, double scale,
                                                      const double *__restrict__ lamr,
                                                      const double *__restrict__ lamk, int row0,
                                                      double *__restrict__ rs,
                                                      const unsigned char *__restrict__ rowmark,
                                                      int rm_inv = 0) {
    // only the listed rows (rm_inv: only the others)
    if (rowmark && (rowmark[blockIdx.x] != 0) == (rm_inv != 0)) return;
    constexpr int NT = K1T<BIG>::T;
    constexpr int PP = (K1_MAXN / 2 + NT - 1) / NT;   // (k, N - k) pairs per thread, N < K1_MAXN
    extern __shared__ double2 z[];
    __shared__ double red[256];
    // PLAN 1: n = 4096 (compile-time passes, fft_4095)
    const int N = PLAN == 1 || PLAN == 3 ? 4095 : n - 1, r = blockIdx.x;
    double *d = (double *)z;
    const double2 *Wq0 = W + (N - 1);   // after the N - 1 pass twiddles: W^k, k = 0 .. N
    put_row_even<NT>(d, N, src + (long)r * n);
    // SOLVE runs the transform twice (forward, then inverse on the divided spectrum): one
    // loop, so that the FFT is inlined once
#pragma unroll 1
    for (int it = 0; it < (SOLVE ? 2 : 1); ++it) {
        __syncthreads();
        if constexpr (PLAN == 1) fft_4095<NT>(z, W);
        else if constexpr (PLAN == 3) fft_4095d<NT>(z, W);
        else fft_lds<BIG, NT, K1_MAXN>(z, N, rd, W, z + N);
        // opaque per iteration: keeps the twiddle / eigenvalue loads below from being hoisted
        // above the FFT (they would hold ~40 registers across it)
        const double2 *Wq = Wq0;
        const double *lr = lamr, *lk = lamk;
        int tid = threadIdx.x;
        asm volatile("" : "+s"(Wq), "+s"(lr), "+s"(lk), "+v"(tid));
        double xa[PP], xb[PP];   // X_k, X_{N-k} for k = tid + t NT <= N / 2
#pragma unroll
        for (int t = 0; t < PP; ++t) {
            const int k = tid + t * NT;
            if (k <= N / 2) {
                const double2 A = z[k], B = z[k ? N - k : 0], w = Wq[k];
                const double S = A.x + B.x, D = A.x - B.x, T = A.y + B.y;
                const double c = w.x, sn = -w.y;
                xa[t] = 0.5 * (S + c * T - sn * D);
                xb[t] = 0.5 * (S - c * T + sn * D);
            }
        }
        if (SOLVE && it == 0) {
            const int kx = row0 + r;
            __syncthreads();   // every Z read
#pragma unroll
            for (int t = 0; t < PP; ++t) {
                const int k = tid + t * NT;
                if (k <= N / 2) {
                    const double ea = (kx == 0 && k == 0) ? 1.0 : lr[kx] + lk[k];
                    const double ya = xa[t] / ea;
                    d[k] = ya;
                    if (k >= 1) d[2 * N - k] = ya;
                    const int kb = N - k;
                    if (kb != k) {
                        const double yb = xb[t] / (lr[kx] + lk[kb]);
                        d[kb] = yb;
                        if (kb >= 1 && kb < N) d[2 * N - kb] = yb;
                    }
                }
                // one pair's divisions at a time: interleaved, their expansions spill
                __builtin_amdgcn_sched_barrier(0);
            }
            continue;
        }
        double *o = dst + (long)r * n;
#pragma unroll
        for (int t = 0; t < PP; ++t) {
            const int k = tid + t * NT;
            if (k <= N / 2) {
                o[k] = xa[t] * scale;
                if (N - k != k) o[N - k] = xb[t] * scale;
            }
        }
        if (rs) {
            // the sum k_rowsum would take of the row written: 256 strided partials, then the
            // halving tree (ops.hip)
            __syncthreads();
#pragma unroll
            for (int t = 0; t < PP; ++t) {
                const int k = tid + t * NT;
                if (k <= N / 2) { d[k] = xa[t] * scale; d[N - k] = xb[t] * scale; }
            }
            __syncthreads();
            if (tid < 256) {
                double acc = 0.0;
                for (int k = tid; k < n; k += 256) acc += d[k];
                red[tid] = acc;
            }
            __syncthreads();
            for (int w = 128; w > 0; w >>= 1) {
                if (tid < w) red[tid] = red[tid] + red[tid + w];
                __syncthreads();
            }
            if (tid == 0) rs[r] = red[0];
        }
    }
}

// out (C x R) = in (R x C) transposed, 64 x 64 tiles through LDS.  rowmark (nullable) with
// mode 1: only the 64-row blocks of in holding no marked row; mode 2: only those holding one
__global__ void __launch_bounds__(256) k_transpose(const double *__restrict__ in, int R, int C,
                                                   double *__restrict__ out,
                                                   const unsigned char *__restrict__ rowmark = nullptr,
                                                   int mode = 0) {
    __shared__ double t[64][65];
    const int c0 = blockIdx.x * 64, r0 = blockIdx.y * 64, tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    if (rowmark) {
        const bool any = __syncthreads_or(threadIdx.x < 64 && r0 + tx < R && rowmark[r0 + tx] != 0);
        if (any != (mode == 2)) return;
    }
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
    int Ns = 1, off = 0;
    for (int k = 0; k < np; ++k) {
        rd.p[k] = Pass{rad[k], Ns, (float)(1.0 / Ns), off};
        off += (rad[k] - 1) * Ns;
        Ns *= rad[k];
    }
    rd.n = np;
    return rd;
}

// One LDS DCT-I pass over nrows rows of length n (axis 0: n = nx, axis 1: n = ny).  SOLVE
// (axis 1 only): forward, / eig, inverse, with rows = x-frequencies row0 .. row0 + nrows.
int dct_pass(rmt_ctx *ctx, bool solve, int axis, const double *src, double *dst, int nrows,
             int row0, double scale, double *rs, const unsigned char *rowmark, bool unmarked) {
    DctPlan *P = ctx->dct;
    RMT_CHECK(P && P->lds, RMT_ENOTSUP, "dct_pass: no LDS DCT plan for this grid");
    RMT_CHECK(!solve || axis == 1, RMT_EINVAL, "dct_pass: the solve pass runs along y");
    RMT_CHECK(!rs || (!solve && nrows <= ctx->rsum_len), RMT_EINVAL, "dct_pass: row sums");
    RMT_CHECK(!rowmark || (!solve && !rs), RMT_EINVAL, "dct_pass: row marks on a plain row pass");
    static bool attr = false;
    if (!attr) {
        const void *fs[8] = {(const void *)k_dct1<false, 0>, (const void *)k_dct1<true, 0>,
                             (const void *)k_dct1<false, 1>, (const void *)k_dct1<true, 1>,
                             (const void *)k_dct1<false, 0, 1>, (const void *)k_dct1<true, 0, 1>,
                             (const void *)k_dct1<false, 0, 3>, (const void *)k_dct1<true, 0, 3>};
        for (auto f : fs)
            RMT_HIP(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize,
                                        (int)FFT_LDS_MAX));
        attr = true;
    }
    if (nrows <= 0) return RMT_OK;
    const int n = axis == 0 ? P->nx : P->ny;
    const int *rad = axis == 0 ? P->radx : P->rady, np = axis == 0 ? P->npx : P->npy;
    const Radices rd = radices(rad, np);
    const double2 *W = axis == 0 ? P->Wx : P->Wy;
    // (a matrix-form pass stages a second length-(n - 1) sequence and its R roots after the row)
    const size_t lds = (size_t)(P->mat ? 2 * (n - 1) + 32 : n - 1) * sizeof(double2);
    const unsigned g = (unsigned)nrows;   // one row per workgroup
    hipStream_t st = ctx->stream;
    const bool k4095 = n == 4096 && !P->big && np == 4 && rad[0] == 5 &&
                       rad[1] == 7 && rad[2] == 9 && rad[3] == 13;   // fft_4095's plan
    const bool k4095d = n == 4096 && !P->big && np == 4 && rad[0] == 13 &&
                        rad[1] == 9 && rad[2] == 7 && rad[3] == 5;   // fft_4095d's
    if (k4095d && solve)
        k_dct1<true, 0, 3><<<g, K1T<0>::T, lds, st>>>(src, dst, nrows, n, W, rd, scale, P->lamx, P->lamy, row0, nullptr, nullptr);
    else if (k4095d)
        k_dct1<false, 0, 3><<<g, K1T<0>::T, lds, st>>>(src, dst, nrows, n, W, rd, scale, nullptr, nullptr, 0, rs, rowmark, unmarked);
    else if (k4095 && solve)
        k_dct1<true, 0, 1><<<g, K1T<0>::T, lds, st>>>(src, dst, nrows, n, W, rd, scale, P->lamx, P->lamy, row0, nullptr, nullptr);
    else if (k4095)
        k_dct1<false, 0, 1><<<g, K1T<0>::T, lds, st>>>(src, dst, nrows, n, W, rd, scale, nullptr, nullptr, 0, rs, rowmark, unmarked);
    else if (solve) {
        if (P->big) k_dct1<true, 1><<<g, K1T<1>::T, lds, st>>>(src, dst, nrows, n, W, rd, scale, P->lamx, P->lamy, row0, nullptr, nullptr);
        else k_dct1<true, 0><<<g, K1T<0>::T, lds, st>>>(src, dst, nrows, n, W, rd, scale, P->lamx, P->lamy, row0, nullptr, nullptr);
    } else {
        if (P->big) k_dct1<false, 1><<<g, K1T<1>::T, lds, st>>>(src, dst, nrows, n, W, rd, scale, nullptr, nullptr, 0, rs, rowmark, unmarked);
        else k_dct1<false, 0><<<g, K1T<0>::T, lds, st>>>(src, dst, nrows, n, W, rd, scale, nullptr, nullptr, 0, rs, rowmark, unmarked);
    }
    RMT_LAUNCHED();
    return RMT_OK;
}

bool dct_lds_ready(rmt_ctx *ctx) { return ctx->dct && ctx->dct->lds; }

// k_transpose with 16-B accesses (R, C even, 16-B aligned planes): a lane moves a pair of
// adjacent doubles on both sides, through the same padded 64 x 64 LDS tile
__global__ void __launch_bounds__(256) k_transpose2(const double *__restrict__ in, int R, int C,
                                                    double *__restrict__ out,
                                                    const unsigned char *__restrict__ rowmark,
                                                    int mode) {
    __shared__ double t[64][65];
    const int c0 = blockIdx.x * 64, r0 = blockIdx.y * 64, tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
    if (rowmark) {
        const int l = threadIdx.x & 63;
        const bool any = __syncthreads_or(threadIdx.x < 64 && r0 + l < R && rowmark[r0 + l] != 0);
        if (any != (mode == 2)) return;
    }
    double2 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {   // rows ty + 8k, columns 2tx, 2tx + 1
        const int r = r0 + ty + 8 * k, c = c0 + 2 * tx;
        v[k] = (r < R && c < C) ? *(const double2 *)(in + (long)r * C + c) : make_double2(0.0, 0.0);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        t[ty + 8 * k][2 * tx] = v[k].x;
        t[ty + 8 * k][2 * tx + 1] = v[k].y;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 8; ++k) {   // output row c0 + ty + 8k, columns r0 + 2tx, + 1
        const int c = c0 + ty + 8 * k, r = r0 + 2 * tx;
        if (c < C && r < R)
            *(double2 *)(out + (long)c * R + r) = make_double2(t[2 * tx][ty + 8 * k], t[2 * tx + 1][ty + 8 * k]);
    }
}

void transpose(const rmt_ctx *ctx, hipStream_t st, const double *in, int R, int C, double *out,
               const unsigned char *rowmark, int mode) {
    // transpose2 = 0 (RMT_TRANSPOSE2=0): the 8-B kernel
    if (ctx->opt.transpose2 && R % 2 == 0 && C % 2 == 0 && ((uintptr_t)in & 15) == 0 && ((uintptr_t)out & 15) == 0)
        k_transpose2<<<dim3((C + 63) / 64, (R + 63) / 64), 256, 0, st>>>(in, R, C, out, rowmark, mode);
    else
        k_transpose<<<dim3((C + 63) / 64, (R + 63) / 64), 256, 0, st>>>(in, R, C, out, rowmark, mode);
}

static int dct_lds_solve(rmt_ctx *ctx, DctPlan *P, const double *rhs, double *p, double *rs) {
    const int ny = P->ny, nx = P->nx;
    hipStream_t st = ctx->stream;
    // forward along x: p <- DCT_x(rhs) (p doubles as scratch), then T <- p^T (nx x ny)
    RMT_TRY(dct_pass(ctx, false, 0, rhs, p, ny, 0, 1.0));
    transpose(ctx, st, p, ny, nx, P->T);
    // columns: DCT_y, / eig, inverse DCT_y (scaled), in place on T
    RMT_TRY(dct_pass(ctx, true, 1, P->T, P->T, nx, 0, 1.0 / (2.0 * (ny - 1))));
    transpose(ctx, st, P->T, nx, ny, p);
    // inverse along x, in place (+ the row sums of the result)
    RMT_TRY(dct_pass(ctx, false, 0, p, p, ny, 0, 1.0 / (2.0 * (nx - 1)), rs));
    RMT_LAUNCHED();
    return RMT_OK;
}

// the row blocks of pc whose rows are all unmarked are final before the marked rows are
// redone: transposed ahead (beside the extrapolation chain); dct_solve_after_rows with the
// same marks then transposes only the others
int dct_transpose_unmarked(rmt_ctx *ctx, const double *pc, const unsigned char *rowmark) {
    DctPlan *P = ctx->dct;
    RMT_CHECK(P && P->lds && rowmark, RMT_ENOTSUP, "dct_transpose_unmarked: LDS DCT plan needed");
    transpose(ctx, ctx->stream, pc, P->ny, P->nx, P->T, rowmark, 1);
    RMT_LAUNCHED();
    return RMT_OK;
}

int dct_solve_after_rows(rmt_ctx *ctx, double *pc, double *dev_root,
                         const unsigned char *early_marks) {
    DctPlan *P = ctx->dct;
    RMT_CHECK(P && P->lds && P->ny <= ctx->rsum_len, RMT_ENOTSUP,
              "dct_solve_after_rows: LDS DCT plan needed");
    const int ny = P->ny, nx = P->nx;
    transpose(ctx, ctx->stream, pc, ny, nx, P->T, early_marks, early_marks ? 2 : 0);
    RMT_TRY(dct_pass(ctx, true, 1, P->T, P->T, nx, 0, 1.0 / (2.0 * (ny - 1))));
    transpose(ctx, ctx->stream, P->T, nx, ny, pc);
    RMT_TRY(dct_pass(ctx, false, 0, pc, pc, ny, 0, 1.0 / (2.0 * (nx - 1)), ctx->rsum));
    return rowtree_sums(ctx, ny, dev_root);
}

int dct_solve(rmt_ctx *ctx, const double *rhs, double dx, double dy, double *p,
              double *dev_root) {
    RMT_TRY(dct_plan(ctx, dx, dy));
    DctPlan *P = ctx->dct;
    const int ny = P->ny, nx = P->nx;
    if (P->lds) {
        const bool fuse = dev_root && ny <= ctx->rsum_len;
        RMT_TRY(dct_lds_solve(ctx, P, rhs, p, fuse ? ctx->rsum : nullptr));
        if (fuse) return rowtree_sums(ctx, ny, dev_root);
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
    if (dev_root) RMT_HIP(hipMemsetAsync(dev_root, 0, sizeof(double), ctx->stream));
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

// factor(8192)'s plan: radices 2, 8, 8, 8, 8 (ascending), twiddle offsets 0, 1, 15, 127, 1023
template <int NT>
__device__ __forceinline__ void fft_8192(double2 *z, const double2 *__restrict__ W) {
    fft_pass_k<2, 1, NT, 8192>(z, W);
    fft_pass_k<8, 2, NT, 8192>(z, W + 1);
    fft_pass_k<8, 16, NT, 8192>(z, W + 15);
    fft_pass_k<8, 128, NT, 8192>(z, W + 127);
    fft_pass_k<8, 1024, NT, 8192>(z, W + 1023);
}

// PLAN 2: n = 8192 (compile-time passes, fft_8192: the same arithmetic as fft_lds)
template <int MODE, int BIG, int PLAN = 0>
__global__ void __launch_bounds__(FftT<BIG>::T) k_dct2(const double *__restrict__ src,
                                                       double *__restrict__ dst, int rows, int n,
                                                       const double2 *__restrict__ W,
                                                       const double2 *__restrict__ Wq, Radices rd,
                                                       const double *__restrict__ lamr,
                                                       const double *__restrict__ lamk, int row0,
                                                       double scale,
                                                       const double *__restrict__ mroot = nullptr,
                                                       double mcount = 1.0) {
    constexpr int DCT_T = FftT<BIG>::T;
    extern __shared__ double2 z[];
    constexpr int PER = DCT_MAXM / DCT_T;
    const int rA = 2 * blockIdx.x, rB = rA + 1, tid = threadIdx.x;
    const bool hasB = rB < rows;
    const double *sa = src + (long)rA * n, *sb = src + (long)rB * n;
    double *da = dst + (long)rA * n, *db = dst + (long)rB * n;
    if constexpr (MODE != 2) {
        // mroot (MODE 0, nullable): the rows' tree root -- x - root / count on the load, the
        // values k_sub_tree_mean would have left in src
        const double mean = mroot ? mroot[0] / mcount : 0.0;
        for (int m = tid; m < n; m += DCT_T) {
            const int q = mk_src(m, n);
            if (mroot) z[m] = make_double2(sa[q] - mean, hasB ? sb[q] - mean : 0.0);
            else z[m] = make_double2(sa[q], hasB ? sb[q] : 0.0);
        }
        __syncthreads();
        if constexpr (PLAN == 2) fft_8192<DCT_T>(z, W);
        else fft_lds<BIG, FftT<BIG>::T, DCT_MAXM>(z, n, rd, W);
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
    if constexpr (PLAN == 2) fft_8192<DCT_T>(z, W);
    else fft_lds<BIG, FftT<BIG>::T, DCT_MAXM>(z, n, rd, W);
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
    (void)hipFree(P->Wx); (void)hipFree(P->Wy); (void)hipFree(P->Qx); (void)hipFree(P->Qy);
    (void)hipFree(P->lamx); (void)hipFree(P->lamy); (void)hipFree(P->T);
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
    RMT_UPLOAD(*Q, h.data(), n * sizeof(double2));
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
    if ((nx & 1) || (ny & 1) || !factor(nx, P->radx, &P->npx) || !factor(ny, P->rady, &P->npy) ||
        !lds_fits(nx) || !lds_fits(ny)) {
        delete P;
        set_error("DCT-II solve: N must be even, <= 8192, and factor into radices <= 23");
        return RMT_ENOTSUP;
    }
    P->big = big_radix(P->radx, P->npx) || big_radix(P->rady, P->npy);
    ctx->dct2 = P;
    RMT_TRY(twiddles(nx, P->radx, P->npx, &P->Wx));
    RMT_TRY(twiddles(ny, P->rady, P->npy, &P->Wy));
    RMT_TRY(quarter_twiddles(nx, &P->Qx));
    RMT_TRY(quarter_twiddles(ny, &P->Qy));
    std::vector<double> lx, ly;
    mac_lambda(nx, dx, lx);
    mac_lambda(ny, dy, ly);
    RMT_HIP(hipMalloc(&P->lamx, nx * sizeof(double)));
    RMT_HIP(hipMalloc(&P->lamy, ny * sizeof(double)));
    RMT_UPLOAD(P->lamx, lx.data(), nx * 8);
    RMT_UPLOAD(P->lamy, ly.data(), ny * 8);
    RMT_HIP(hipMalloc(&P->T, (size_t)nx * ny * sizeof(double)));
    static bool attr = false;
    if (!attr) {
        const void *fs[9] = {(const void *)k_dct2<0, 0>, (const void *)k_dct2<1, 0>,
                             (const void *)k_dct2<2, 0>, (const void *)k_dct2<0, 1>,
                             (const void *)k_dct2<1, 1>, (const void *)k_dct2<2, 1>,
                             (const void *)k_dct2<0, 0, 2>, (const void *)k_dct2<1, 0, 2>,
                             (const void *)k_dct2<2, 0, 2>};
        for (auto f : fs)
            RMT_HIP(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize,
                                        (int)FFT_LDS_MAX));
        attr = true;
    }
    return RMT_OK;
}

// one DCT-II pass over nrows rows along axis (0: length nx, 1: length ny; MODE 1 needs 1)
int dct2_pass(rmt_ctx *ctx, int mode, int axis, const double *src, double *dst,
                     int nrows, int row0, const double *mroot, double mcount) {
    Dct2Plan *P = ctx->dct2;
    const int n = axis == 0 ? P->nx : P->ny;
    const Radices rd = axis == 0 ? radices(P->radx, P->npx) : radices(P->rady, P->npy);
    const double2 *W = axis == 0 ? P->Wx : P->Wy, *Q = axis == 0 ? P->Qx : P->Qy;
    const size_t lds = (size_t)n * sizeof(double2);
    const unsigned g = (nrows + 1) / 2;
    hipStream_t st = ctx->stream;
    RMT_CHECK(!mroot || mode == 0, RMT_EINVAL, "dct2_pass: the mean is taken on a forward pass");
#define DCT2_L(M, B) k_dct2<M, B><<<g, FftT<B>::T, lds, st>>>(src, dst, nrows, n, W, Q, rd, P->lamx, P->lamy, row0, 1.0, mroot, mcount)
#define DCT2_K(M) k_dct2<M, 0, 2><<<g, FftT<0>::T, lds, st>>>(src, dst, nrows, n, W, Q, rd, P->lamx, P->lamy, row0, 1.0, mroot, mcount)
    // n = 8192: the compile-time plan (factor(8192) is always 2, 8, 8, 8, 8)
    const bool k8192 = n == 8192 && rd.n == 5 && rd.p[0].R == 2 && rd.p[4].R == 8;
    if (k8192) {
        if (mode == 0) DCT2_K(0); else if (mode == 1) DCT2_K(1); else DCT2_K(2);
    } else if (P->big) {
        if (mode == 0) DCT2_L(0, 1); else if (mode == 1) DCT2_L(1, 1); else DCT2_L(2, 1);
    } else {
        if (mode == 0) DCT2_L(0, 0); else if (mode == 1) DCT2_L(1, 0); else DCT2_L(2, 0);
    }
#undef DCT2_L
#undef DCT2_K
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
int dct2_solve(rmt_ctx *ctx, const double *rhs, double *p, const double *mroot, double mcount) {
    Dct2Plan *P = ctx->dct2;
    RMT_CHECK(P, RMT_EINVAL, "dct2_solve: no plan");
    const int ny = P->ny, nx = P->nx;
    RMT_TRY(dct2_pass(ctx, 0, 0, rhs, p, ny, 0, mroot, mcount));
    transpose(ctx, ctx->stream, p, ny, nx, P->T);
    RMT_TRY(dct2_pass(ctx, 1, 1, P->T, P->T, nx, 0));
    transpose(ctx, ctx->stream, P->T, nx, ny, p);
    return dct2_pass(ctx, 2, 0, p, p, ny, 0);
}
}  // namespace rmt
