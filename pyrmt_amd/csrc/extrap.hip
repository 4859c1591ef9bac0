// extrap.hip -- functions.py:48-163 extrapolate_reference_map on MI355X, exact semantics.
//
// The reference fits targets in raster order and marks each accepted target "known"
// immediately (Gauss-Seidel).  Cramer's rule on absolute coordinates amplifies rounding,
// so any reordering changes results far above the rounding level, and a parallel
// fixed-point iteration needs as many sweeps as the dependency depth (measured: ~3000
// at N=4096).  The chain is therefore executed as a chain:
//   1. chip-wide: known = (phi < 0) byte plane; candidate band = interior unknown cells
//      within Chebyshev distance max_layers of a known cell, compacted in raster order
//      (count / scan / write, deterministic);
//   2. one wave: per layer, targets = candidates that are unknown with a known 3x3
//      neighbour; then targets in raster order, each fitted by the whole wave (lanes own
//      window cells; 12 lanes run the 12 ordered sums of functions.py:128-145), the value
//      written and the cell marked known before the next target.
#include "rmt_internal.hpp"
#include "exp_glibc.h"

namespace rmt {

constexpr int EX_CELLS_PER_BLOCK = 2048, EX_T = 256;

__global__ void k_ex_known(const double *__restrict__ phi, const double *__restrict__ X1,
                           const double *__restrict__ X2, long n, unsigned char *__restrict__ known,
                           double *__restrict__ X1o, double *__restrict__ X2o, int copy) {
    long c = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (c >= n) return;
    known[c] = phi[c] < 0;
    if (copy) { X1o[c] = X1[c]; X2o[c] = X2[c]; }
}

__device__ __forceinline__ bool ex_candidate(const unsigned char *__restrict__ known, long c,
                                             int ny, int nx, int L) {
    int j = (int)(c / nx), i = (int)(c % nx);
    if (j < 1 || j >= ny - 1 || i < 1 || i >= nx - 1 || known[c]) return false;
    int jlo = max(j - L, 0), jhi = min(j + L, ny - 1), ilo = max(i - L, 0), ihi = min(i + L, nx - 1);
    for (int jj = jlo; jj <= jhi; ++jj)
        for (int ii = ilo; ii <= ihi; ++ii)
            if (known[(long)jj * nx + ii]) return true;
    return false;
}

__global__ void __launch_bounds__(EX_T) k_ex_count(const unsigned char *__restrict__ known,
                                                   int ny, int nx, int L, int *__restrict__ counts) {
    __shared__ int s;
    if (threadIdx.x == 0) s = 0;
    __syncthreads();
    long base = (long)blockIdx.x * EX_CELLS_PER_BLOCK, n = (long)ny * nx;
    int cnt = 0;
    for (int q = threadIdx.x; q < EX_CELLS_PER_BLOCK; q += EX_T) {
        long c = base + q;
        if (c < n && ex_candidate(known, c, ny, nx, L)) ++cnt;
    }
    atomicAdd(&s, cnt);
    __syncthreads();
    if (threadIdx.x == 0) counts[blockIdx.x] = s;
}

// exclusive scan of nb counts by one 1024-thread block; total -> offsets[nb]
__global__ void __launch_bounds__(1024) k_ex_scan(const int *__restrict__ counts, int nb,
                                                  int *__restrict__ offsets) {
    __shared__ int s[1024];
    __shared__ int carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (int base = 0; base < nb; base += 1024) {
        int k = base + threadIdx.x;
        int x = k < nb ? counts[k] : 0;
        s[threadIdx.x] = x;
        __syncthreads();
        for (int w = 1; w < 1024; w <<= 1) {
            int y = threadIdx.x >= w ? s[threadIdx.x - w] : 0;
            __syncthreads();
            s[threadIdx.x] += y;
            __syncthreads();
        }
        if (k < nb) offsets[k] = carry + s[threadIdx.x] - x;
        __syncthreads();
        if (threadIdx.x == 1023) carry += s[1023];
        __syncthreads();
    }
    if (threadIdx.x == 0) offsets[nb] = carry;
}

__global__ void __launch_bounds__(EX_T) k_ex_write(const unsigned char *__restrict__ known,
                                                   int ny, int nx, int L,
                                                   const int *__restrict__ offsets,
                                                   int *__restrict__ cand) {
    __shared__ int s[EX_T];
    long base = (long)blockIdx.x * EX_CELLS_PER_BLOCK, n = (long)ny * nx;
    int out = offsets[blockIdx.x];
    for (int q0 = 0; q0 < EX_CELLS_PER_BLOCK; q0 += EX_T) {
        long c = base + q0 + threadIdx.x;
        int f = (c < n && ex_candidate(known, c, ny, nx, L)) ? 1 : 0;
        s[threadIdx.x] = f;
        __syncthreads();
        for (int w = 1; w < EX_T; w <<= 1) {
            int y = threadIdx.x >= w ? s[threadIdx.x - w] : 0;
            __syncthreads();
            s[threadIdx.x] += y;
            __syncthreads();
        }
        if (f) cand[out + s[threadIdx.x] - 1] = (int)c;
        int tot = s[EX_T - 1];
        __syncthreads();
        out += tot;
    }
}

// The sequential sweep: one wave (64 lanes).  Window cell q = 9*(jj-j+4) + (ii-i+4).
__global__ void __launch_bounds__(64) k_ex_sweep(double *__restrict__ X1e, double *__restrict__ X2e,
                                                 unsigned char *__restrict__ known,
                                                 const int *__restrict__ cand,
                                                 const int *__restrict__ ncand_p,
                                                 int *__restrict__ targets, int ny, int nx,
                                                 double dx, double dy, int max_layers,
                                                 int *__restrict__ stats) {
    __shared__ double term[81][12];
    __shared__ unsigned char inc[81];
    __shared__ int ntar;
    const int lane = threadIdx.x;
    const int ncand = *ncand_p;
    double r = 4 * sqrt(dx * dx + dy * dy);
    const double r2 = r * r;
    int filled = 0;
    for (int layer = 0; layer < max_layers; ++layer) {
        // targets among the candidates, in raster order (wave-wide ballot compaction)
        if (lane == 0) ntar = 0;
        __syncthreads();
        for (int b = 0; b < ncand; b += 64) {
            int k = b + lane;
            bool tgt = false;
            int c = 0;
            if (k < ncand) {
                c = cand[k];
                if (!known[c]) {
                    for (int dj = -1; dj <= 1 && !tgt; ++dj)
                        for (int di = -1; di <= 1; ++di)
                            if (known[c + (long)dj * nx + di]) { tgt = true; break; }
                }
            }
            unsigned long long m = __ballot(tgt);
            int pos = __popcll(m & ((1ull << lane) - 1));
            if (tgt) targets[ntar + pos] = c;
            __syncthreads();
            if (lane == 0) ntar += __popcll(m);
            __syncthreads();
        }
        const int nt = ntar;
        if (nt == 0) break;
        for (int t = 0; t < nt; ++t) {
            const int c = targets[t];
            const int j = c / nx, i = c % nx;
            const double x0 = dx * i, y0 = dy * j;
            for (int q = lane; q < 81; q += 64) {
                int jj = j - 4 + q / 9, ii = i - 4 + q % 9;
                bool in = jj >= 0 && jj < ny && ii >= 0 && ii < nx;
                long cc = (long)jj * nx + ii;
                in = in && known[cc];
                double xi = dx * ii, yi = dy * jj, d2 = 0.0;
                if (in) {
                    double ax = xi - x0, ay = yi - y0;
                    d2 = ax * ax + ay * ay;
                    in = d2 <= r2;
                }
                inc[q] = in;
                if (in) {
                    double w = exp_glibc(-d2 / r2);   // libm exp, bit for bit
                    double b1 = X1e[cc], b2 = X2e[cc];
                    double wa0 = w * 1.0, wa1 = w * xi, wa2 = w * yi;
                    term[q][0] = wa0 * b1; term[q][1] = wa1 * b1; term[q][2] = wa2 * b1;
                    term[q][3] = wa0 * b2; term[q][4] = wa1 * b2; term[q][5] = wa2 * b2;
                    term[q][6] = wa0 * 1.0; term[q][7] = wa0 * xi; term[q][8] = wa0 * yi;
                    term[q][9] = wa1 * xi; term[q][10] = wa1 * yi; term[q][11] = wa2 * yi;
                }
            }
            __syncthreads();
            // ordered sums (functions.py:128-145): lane k < 12 folds term[.][k] in loop order
            double acc = 0.0;
            int count = 0;
            if (lane < 12) {
                for (int q = 0; q < 81; ++q)
                    if (inc[q]) { acc += term[q][lane]; ++count; }
            }
            double B10 = __shfl(acc, 0), B11 = __shfl(acc, 1), B12 = __shfl(acc, 2);
            double B20 = __shfl(acc, 3), B21 = __shfl(acc, 4), B22 = __shfl(acc, 5);
            double A00 = __shfl(acc, 6), A01 = __shfl(acc, 7), A02 = __shfl(acc, 8);
            double A11 = __shfl(acc, 9), A12 = __shfl(acc, 10), A22 = __shfl(acc, 11);
            count = __shfl(count, 0);
            if (lane == 0 && count >= 3) {
                const double A[9] = {A00, A01, A02, A01, A11, A12, A02, A12, A22};
                double det = (A[0] * (A[4] * A[8] - A[5] * A[7])
                            - A[1] * (A[3] * A[8] - A[5] * A[6])
                            + A[2] * (A[3] * A[7] - A[4] * A[6]));
                if (fabs(det) > 1e-10) {
                    // utils.py:134-166 fast_solve_3x3 twice (same detA recomputed)
                    double detA = det, inv_det = 1.0 / detA;
                    double o[2];
                    const double bb[2][3] = {{B10, B11, B12}, {B20, B21, B22}};
                    for (int s = 0; s < 2; ++s) {
                        const double *b = bb[s];
                        double x = (b[0] * (A[4] * A[8] - A[5] * A[7]) -
                                    A[1] * (b[1] * A[8] - A[5] * b[2]) +
                                    A[2] * (b[1] * A[7] - A[4] * b[2])) * inv_det;
                        double y = (A[0] * (b[1] * A[8] - A[5] * b[2]) -
                                    b[0] * (A[3] * A[8] - A[5] * A[6]) +
                                    A[2] * (A[3] * b[2] - b[1] * A[6])) * inv_det;
                        double z = (A[0] * (A[4] * b[2] - b[1] * A[7]) -
                                    A[1] * (A[3] * b[2] - b[1] * A[6]) +
                                    b[0] * (A[3] * A[7] - A[4] * A[6])) * inv_det;
                        o[s] = x + y * x0 + z * y0;
                    }
                    X1e[c] = o[0];
                    X2e[c] = o[1];
                    known[c] = 1;
                    ++filled;
                }
            }
            __syncthreads();   // next target sees this value and flag
        }
    }
    if (lane == 0 && stats) stats[0] = filled;
}

int extrapolate(rmt_ctx *ctx, const double *X1, const double *X2, const double *phi, double dx,
                double dy, int max_layers, double *X1o, double *X2o, const int *dev_skip) {
    (void)dev_skip;
    const int ny = ctx->ny, nx = ctx->nx;
    const long n = (long)ny * nx;
    const int nb = (int)((n + EX_CELLS_PER_BLOCK - 1) / EX_CELLS_PER_BLOCK);
    // byte scratch: known plane | ints: counts[nb], offsets[nb+1], cand[n], targets[n], stats
    size_t kbytes = (n + 255) / 256 * 256;
    size_t need = kbytes + sizeof(int) * ((size_t)2 * nb + 2 * (size_t)n + 16);
    RMT_TRY(ensure_bytes(ctx, need));
    unsigned char *known = ctx->bytes;
    int *counts = (int *)(ctx->bytes + kbytes), *offsets = counts + nb, *cand = offsets + nb + 1;
    int *targets = cand + n, *stats = targets + n;
    if (max_layers <= 0) {
        if (X1o != X1) RMT_HIP(hipMemcpyAsync(X1o, X1, n * 8, hipMemcpyDeviceToDevice, ctx->stream));
        if (X2o != X2) RMT_HIP(hipMemcpyAsync(X2o, X2, n * 8, hipMemcpyDeviceToDevice, ctx->stream));
        return RMT_OK;
    }
    int copy = (X1o != X1) || (X2o != X2);
    k_ex_known<<<grid1d(n, 256), 256, 0, ctx->stream>>>(phi, X1, X2, n, known, X1o, X2o, copy);
    k_ex_count<<<nb, EX_T, 0, ctx->stream>>>(known, ny, nx, max_layers, counts);
    k_ex_scan<<<1, 1024, 0, ctx->stream>>>(counts, nb, offsets);
    k_ex_write<<<nb, EX_T, 0, ctx->stream>>>(known, ny, nx, max_layers, offsets, cand);
    if (ctx->prof) RMT_HIP(hipEventRecord(ctx->ev[2], ctx->stream));
    k_ex_sweep<<<1, 64, 0, ctx->stream>>>(X1o, X2o, known, cand, offsets + nb, targets, ny, nx, dx,
                                          dy, max_layers, stats);
    RMT_LAUNCHED();
    if (ctx->prof) RMT_HIP(hipEventRecord(ctx->ev[3], ctx->stream));
    return RMT_OK;
}

}  // namespace rmt

extern "C" int rmt_extrapolate_reference_map(rmt_ctx *ctx, const double *X1, const double *X2,
                                             const double *phi, double dx, double dy,
                                             int max_layers, double *X1_out, double *X2_out) {
    RMT_CHECK(ctx, RMT_EINVAL, "null ctx");
    return rmt::extrapolate(ctx, X1, X2, phi, dx, dy, max_layers, X1_out, X2_out);
}
