// extrap.hip -- functions.py:48-163 extrapolate_reference_map on MI355X, exact semantics.
//
// The reference (serial @njit: the prange at :95 runs serially) fits the targets of a layer in
// raster order and marks each accepted target "known" at once (Gauss-Seidel).  Cramer's rule on
// absolute coordinates amplifies rounding, so any reordering moves results far above rounding
// and a parallel fixed-point iteration needs as many sweeps as the dependency depth (DESIGN.md
// §5).  librmt executes the same dependency DAG, just not in one thread:
//
//   1. k_ex_bits / k_ex_dilate (chip-wide, bit planes): known = (phi < 0) as 64-cell words;
//      candidates = interior unknown cells within Chebyshev distance max_layers of a known cell
//      (the only cells that can ever become known), their layer byte set to "unknown".
//   2. k_ex_sweep (one workgroup of EXW waves): work item = (layer L, row j), taken from an LDS
//      ticket counter in order of j + 5L.  A target (L, j, i) reads the 9x9 window around it, so
//      at its fit the serial state is exactly reproduced when
//        - rows j-4..j+4 of layer L-1 are complete (the window and the 3x3 target test see the
//          state at the start of layer L), and
//        - rows j-1..j-4 of layer L have finished every target at column <= i+4 (the targets
//          before it in raster order that lie in its window); its own row runs in order.
//      Nothing later in raster order can be inside the window yet: row j+r of layer L waits for
//      row j to pass its columns, and layer L+1 waits for layer L.  Every wait is on a lower
//      ticket, so the lowest active ticket always proceeds.  Rows publish progress ("all my
//      targets left of column c are done") in an LDS ring; a layer byte per candidate cell
//      (0..: fitted in layer byte-1, 255: unknown) says whether a cell is known for layer L
//      (byte <= L) or at a fit inside layer L (byte <= L+1).
//   Each fit: lanes own window cells (geometry and glibc-exact weights computed before the
//   wait), 12 lanes fold the 12 sums of functions.py:128-145 in loop order, every lane runs
//   the 3x3 solve on the broadcast sums, lane 0 writes.
//
// Visibility: bytes written inside the sweep (layer bytes, fitted X values) are stored with
// plain stores drained by s_waitcnt vmcnt(0) before the LDS progress word is released, and
// read with sc1 (L2) loads after the acquire; bytes fixed before the launch use plain loads.
#include "rmt_internal.hpp"
#include "exp_glibc.h"

namespace rmt {

typedef unsigned long long u64;

constexpr int EXW = 16;                       // waves of the sweep workgroup
constexpr int EX_RING = 1024;                 // progress ring entries (tickets)
constexpr int EX_WIN = 81;                    // 9x9 window
constexpr unsigned EX_DONE = 0x7fffffffu;     // progress of a completed row
constexpr long EX_SPIN_LIMIT = 1L << 25;      // ~1-2 s of polling, then abort (bug guard)

// known bit plane: word (j, w) bit b <=> phi[j, 64w+b] < 0; row flags / row range reset
__global__ void __launch_bounds__(256) k_ex_bits(const double *__restrict__ phi, int ny, int nx,
                                                 int W, u64 *__restrict__ kbits,
                                                 unsigned char *__restrict__ rowcand,
                                                 int *__restrict__ jrange,
                                                 const double *__restrict__ X1,
                                                 const double *__restrict__ X2,
                                                 double *__restrict__ X1o,
                                                 double *__restrict__ X2o, int copy) {
    const int j = blockIdx.y, i = blockIdx.x * 256 + threadIdx.x;
    const long c = (long)j * nx + i;
    const bool in = i < nx;
    const bool k = in && phi[c] < 0;
    if (in && copy) { X1o[c] = X1[c]; X2o[c] = X2[c]; }
    const u64 m = __ballot(k);
    if ((threadIdx.x & 63) == 0 && (i >> 6) < W) kbits[(long)j * W + (i >> 6)] = m;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        rowcand[j] = 0;
        if (j == 0) { jrange[0] = 0x7fffffff; jrange[1] = -1; }
    }
}

// candidate bit plane: Chebyshev dilation of known by L, minus known, interior cells only
__global__ void __launch_bounds__(256) k_ex_dilate(const u64 *__restrict__ kbits, int ny, int nx,
                                                   int W, int L, u64 *__restrict__ cbits,
                                                   unsigned char *__restrict__ lay,
                                                   unsigned char *__restrict__ rowcand,
                                                   int *__restrict__ jrange) {
    const long t = blockIdx.x * 256L + threadIdx.x;
    if (t >= (long)ny * W) return;
    const int j = (int)(t / W), w = (int)(t % W);
    u64 cw = 0;
    const int i0 = 64 * w, lo = max(1, i0) - i0, hi = min(nx - 2, i0 + 63) - i0;
    if (j >= 1 && j <= ny - 2 && hi >= lo) {
        u64 d = 0;
        if (L >= 64) {
            d = ~0ull;   // superset: every interior unknown cell (exact, just more candidates)
        } else {
            for (int jj = max(0, j - L); jj <= min(ny - 1, j + L); ++jj) {
                const u64 *r = kbits + (long)jj * W;
                const u64 a = w > 0 ? r[w - 1] : 0, b = r[w], e = w + 1 < W ? r[w + 1] : 0;
                u64 h = b;
                for (int s = 1; s <= L; ++s)
                    h |= (b << s) | (a >> (64 - s)) | (b >> s) | (e << (64 - s));
                d |= h;
            }
        }
        const u64 cols = (~0ull >> (63 - hi)) & (~0ull << lo);
        cw = d & ~kbits[t] & cols;
    }
    cbits[t] = cw;
    if (cw) {
        rowcand[j] = 1;
        atomicMin(&jrange[0], j);
        atomicMax(&jrange[1], j);
        for (u64 m = cw; m; m &= m - 1) lay[(long)j * nx + i0 + __builtin_ctzll(m)] = 255;
    }
}

__device__ __forceinline__ unsigned char ld_sc1_u8(const unsigned char *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1_f64(const double *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ u64 readlane64(u64 v, int l) {
    unsigned lo = __builtin_amdgcn_readlane((unsigned)v, l);
    unsigned hi = __builtin_amdgcn_readlane((unsigned)(v >> 32), l);
    return ((u64)hi << 32) | lo;
}
__device__ __forceinline__ double readlane_f64(double v, int l) {
    u64 b = __double_as_longlong(v);
    return __longlong_as_double((long long)readlane64(b, l));
}

struct ExSweep {
    double *X1e, *X2e;
    unsigned char *lay;
    const u64 *kbits, *cbits;
    const unsigned char *rowcand;
    const int *jrange;
    int ny, nx, W, ML;
    double dx, dy;
    int *status;   // [0] fitted cells, [1] abort
};

struct ExState {
    u64 *ring;
    int *abort;
    int jlo, jhi, ML;
};

// progress of row j of layer L (EX_DONE if complete or outside the band's rows)
__device__ __forceinline__ unsigned ex_progress(const ExState &S, int L, int j) {
    if (j < S.jlo || j > S.jhi) return EX_DONE;
    const int T = (j + 5 * L - S.jlo) * S.ML + L;
    const u64 e = __hip_atomic_load(&S.ring[T & (EX_RING - 1)], __ATOMIC_ACQUIRE,
                                    __HIP_MEMORY_SCOPE_WORKGROUP);
    const int tag = (int)(e >> 32);
    return tag > T ? EX_DONE : (tag < T ? 0u : (unsigned)e);
}

__device__ __forceinline__ bool ex_spin(const ExState &S, long &spins) {
    if (++spins > EX_SPIN_LIMIT) {
        __hip_atomic_store(S.abort, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        return false;
    }
    if ((spins & 63) == 0 &&
        __hip_atomic_load(S.abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP))
        return false;
    __builtin_amdgcn_s_sleep(1);
    return true;
}

__device__ __forceinline__ void ex_publish(const ExState &S, int T, unsigned prog) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's stores reached L2
    __hip_atomic_store(&S.ring[T & (EX_RING - 1)], ((u64)(unsigned)T << 32) | prog,
                       __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// known_flag as the 3x3 target test sees it at the start of layer L (functions.py:81-90)
__device__ __forceinline__ bool ex_known_at_start(const ExSweep &A, int jj, int ii, int L) {
    const long wd = (long)jj * A.W + (ii >> 6);
    const u64 bit = 1ull << (ii & 63);
    if (A.kbits[wd] & bit) return true;
    if (!(A.cbits[wd] & bit)) return false;
    return ld_sc1_u8(A.lay + (long)jj * A.nx + ii) <= L;
}

// one window cell: geometry, weight and (static) value before the wait
struct ExCell {
    long cc;
    double xi, yi, w, b1, b2;
    bool geo;      // inside the grid and within the stencil radius
    bool kstat;    // known before the launch (solid)
    bool cand;     // may become known during the sweep
};

__device__ __forceinline__ ExCell ex_cell(const ExSweep &A, int q, int j, int i, double x0,
                                          double y0, double r2) {
    ExCell e{};
    const int jj = j - 4 + q / 9, ii = i - 4 + q % 9;
    const bool in = q < EX_WIN && jj >= 0 && jj < A.ny && ii >= 0 && ii < A.nx;
    e.geo = false; e.kstat = false; e.cand = false;
    e.cc = in ? (long)jj * A.nx + ii : 0;
    e.xi = A.dx * ii; e.yi = A.dy * jj;
    e.w = 0.0; e.b1 = 0.0; e.b2 = 0.0;
    if (in) {
        const double ax = e.xi - x0, ay = e.yi - y0;
        const double d2 = ax * ax + ay * ay;
        e.geo = d2 <= r2;
        if (e.geo) {
            const long wd = (long)jj * A.W + (ii >> 6);
            const u64 bit = 1ull << (ii & 63);
            e.kstat = (A.kbits[wd] & bit) != 0;
            e.cand = !e.kstat && (A.cbits[wd] & bit) != 0;
            if (e.kstat || e.cand) e.w = exp_glibc(-d2 / r2);   // libm exp, bit for bit
            if (e.kstat) { e.b1 = A.X1e[e.cc]; e.b2 = A.X2e[e.cc]; }
        }
    }
    return e;
}

// after the wait: is the cell known now, and its value (functions.py:105-119)
__device__ __forceinline__ bool ex_cell_live(const ExSweep &A, ExCell &e, int L) {
    if (!e.geo) return false;
    if (e.kstat) return true;
    if (!e.cand) return false;
    if (ld_sc1_u8(A.lay + e.cc) > L + 1) return false;
    e.b1 = ld_sc1_f64(A.X1e + e.cc);
    e.b2 = ld_sc1_f64(A.X2e + e.cc);
    return true;
}

__device__ __forceinline__ void ex_terms(double *t, int q, const ExCell &e, bool inc) {
    // t is the wave's [12][EX_WIN] buffer; excluded cells contribute +0.0 (exact: the sums
    // start at +0.0 and never become -0.0)
    double v[12];
    if (inc) {
        const double wa0 = e.w * 1.0, wa1 = e.w * e.xi, wa2 = e.w * e.yi;
        v[0] = wa0 * e.b1; v[1] = wa1 * e.b1; v[2] = wa2 * e.b1;
        v[3] = wa0 * e.b2; v[4] = wa1 * e.b2; v[5] = wa2 * e.b2;
        v[6] = wa0 * 1.0; v[7] = wa0 * e.xi; v[8] = wa0 * e.yi;
        v[9] = wa1 * e.xi; v[10] = wa1 * e.yi; v[11] = wa2 * e.yi;
    } else {
#pragma unroll
        for (int k = 0; k < 12; ++k) v[k] = 0.0;
    }
#pragma unroll
    for (int k = 0; k < 12; ++k) t[k * EX_WIN + q] = v[k];
}

// fit target (j, i) of layer L; returns true if the cell became known
__device__ bool ex_fit(const ExSweep &A, const ExState &S, double *tbuf, int T, int L, int j,
                       int i, double r2, int lane, bool &ok) {
    const double x0 = A.dx * i, y0 = A.dy * j;
    ExCell c0 = ex_cell(A, lane, j, i, x0, y0, r2);
    ExCell c1 = ex_cell(A, lane + 64, j, i, x0, y0, r2);
    // wait for rows j-1..j-4 of this layer to pass column i+4
    const unsigned need = (unsigned)(i + 5);
    long spins = 0;
    for (int r = 1; r <= 4; ++r)
        while (ex_progress(S, L, j - r) < need)
            if (!ex_spin(S, spins)) { ok = false; return false; }
    const bool inc0 = ex_cell_live(A, c0, L), inc1 = ex_cell_live(A, c1, L);
    ex_terms(tbuf, lane, c0, inc0);
    if (lane < EX_WIN - 64) ex_terms(tbuf, lane + 64, c1, inc1);
    const int count = __popcll(__ballot(inc0)) + __popcll(__ballot(inc1 && lane < EX_WIN - 64));
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    double acc = 0.0;
    if (lane < 12) {
        const double *t = tbuf + lane * EX_WIN;
#pragma unroll
        for (int q = 0; q < EX_WIN; ++q) acc += t[q];   // functions.py:128-145 loop order
    }
    __builtin_amdgcn_wave_barrier();
    if (count < 3) return false;
    const double B10 = readlane_f64(acc, 0), B11 = readlane_f64(acc, 1), B12 = readlane_f64(acc, 2);
    const double B20 = readlane_f64(acc, 3), B21 = readlane_f64(acc, 4), B22 = readlane_f64(acc, 5);
    const double A00 = readlane_f64(acc, 6), A01 = readlane_f64(acc, 7), A02 = readlane_f64(acc, 8);
    const double A11 = readlane_f64(acc, 9), A12 = readlane_f64(acc, 10), A22 = readlane_f64(acc, 11);
    const double M[9] = {A00, A01, A02, A01, A11, A12, A02, A12, A22};
    const double det = (M[0] * (M[4] * M[8] - M[5] * M[7])
                      - M[1] * (M[3] * M[8] - M[5] * M[6])
                      + M[2] * (M[3] * M[7] - M[4] * M[6]));
    if (!(fabs(det) > 1e-10)) return false;
    // utils.py:134-166 fast_solve_3x3, once per right-hand side
    const double inv_det = 1.0 / det;
    double o[2];
    const double bb[2][3] = {{B10, B11, B12}, {B20, B21, B22}};
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        const double *b = bb[s];
        const double x = (b[0] * (M[4] * M[8] - M[5] * M[7]) -
                          M[1] * (b[1] * M[8] - M[5] * b[2]) +
                          M[2] * (b[1] * M[7] - M[4] * b[2])) * inv_det;
        const double y = (M[0] * (b[1] * M[8] - M[5] * b[2]) -
                          b[0] * (M[3] * M[8] - M[5] * M[6]) +
                          M[2] * (M[3] * b[2] - b[1] * M[6])) * inv_det;
        const double z = (M[0] * (M[4] * b[2] - b[1] * M[7]) -
                          M[1] * (M[3] * b[2] - b[1] * M[6]) +
                          b[0] * (M[3] * M[7] - M[4] * M[6])) * inv_det;
        o[s] = x + y * x0 + z * y0;
    }
    if (lane == 0) {
        const long c = (long)j * A.nx + i;
        A.X1e[c] = o[0];
        A.X2e[c] = o[1];
        A.lay[c] = (unsigned char)(L + 1);
    }
    return true;
}

__global__ void __launch_bounds__(EXW * 64) k_ex_sweep(ExSweep A) {
    __shared__ u64 ring[EX_RING];
    __shared__ double term[EXW][12 * EX_WIN];
    __shared__ int s_ticket, s_abort;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int s = threadIdx.x; s < EX_RING; s += blockDim.x)
        ring[s] = ((u64)(unsigned)(s - EX_RING) << 32) | EX_DONE;   // virtual done tickets
    if (threadIdx.x == 0) { s_ticket = 0; s_abort = 0; }
    __syncthreads();
    ExState S{ring, &s_abort, A.jrange[0], A.jrange[1], A.ML};
    if (S.jhi < S.jlo) return;   // no candidates at all
    const int ML = A.ML;
    const int ntick = (S.jhi - S.jlo + 1 + 5 * (ML - 1)) * ML;
    double r = 4 * sqrt(A.dx * A.dx + A.dy * A.dy);
    const double r2 = r * r;
    double *tbuf = term[wv];
    int filled = 0;
    bool ok = true;
    for (;;) {
        int T = 0;
        if (lane == 0) T = atomicAdd(&s_ticket, 1);
        T = __builtin_amdgcn_readfirstlane(T);
        if (T >= ntick) break;
        const int L = T % ML, j = S.jlo + T / ML - 5 * L;
        // the ring slot's previous ticket must be complete before it is reused
        long spins = 0;
        const int Tp = T - EX_RING;
        for (;;) {
            const u64 e = __hip_atomic_load(&ring[T & (EX_RING - 1)], __ATOMIC_ACQUIRE,
                                            __HIP_MEMORY_SCOPE_WORKGROUP);
            const int tag = (int)(e >> 32);
            if (tag == Tp && (unsigned)e == EX_DONE) break;
            if (!ex_spin(S, spins)) { ok = false; break; }
        }
        if (!ok) break;
        const bool active = j >= S.jlo && j <= S.jhi && A.rowcand[j];
        if (!active) { ex_publish(S, T, EX_DONE); continue; }
        ex_publish(S, T, 0);
        // rows j-4..j+4 of the previous layer complete
        if (L > 0) {
            for (int rr = -4; rr <= 4 && ok; ++rr)
                while (ex_progress(S, L - 1, j + rr) != EX_DONE)
                    if (!ex_spin(S, spins)) { ok = false; break; }
            if (!ok) break;
        }
        // targets of row j, in column order (functions.py:81-90 then :95-96)
        for (int wb = 0; wb < A.W && ok; wb += 64) {
            const int w = wb + lane;
            const u64 cw = w < A.W ? A.cbits[(long)j * A.W + w] : 0;
            u64 tw = 0;
            for (u64 m = cw; m; m &= m - 1) {
                const int b = __builtin_ctzll(m), i = 64 * w + b;
                if (ld_sc1_u8(A.lay + (long)j * A.nx + i) <= L) continue;   // known already
                bool nb = false;
                for (int dj = -1; dj <= 1 && !nb; ++dj)
                    for (int di = -1; di <= 1 && !nb; ++di)
                        nb = ex_known_at_start(A, j + dj, i + di, L);
                if (nb) tw |= 1ull << b;
            }
            for (u64 lanes = __ballot(tw != 0); lanes && ok; lanes &= lanes - 1) {
                const int src = __builtin_ctzll(lanes);
                for (u64 t = readlane64(tw, src); t && ok; t &= t - 1) {
                    const int i = 64 * (wb + src) + __builtin_ctzll(t);
                    ex_publish(S, T, (unsigned)i);   // every target left of i is done
                    if (ex_fit(A, S, tbuf, T, L, j, i, r2, lane, ok)) ++filled;
                }
            }
        }
        if (!ok) break;
        ex_publish(S, T, EX_DONE);
    }
    if (lane == 0) {
        atomicAdd(&A.status[0], filled);
        if (!ok) atomicExch(&A.status[1], 1);
    }
}

size_t extrap_workspace(int ny, int nx) {
    const size_t n = (size_t)ny * nx, W = (nx + 63) / 64;
    return 2 * (size_t)ny * W * 8 + (n + 255) / 256 * 256 + ((size_t)ny + 255) / 256 * 256 + 64;
}

int extrapolate(rmt_ctx *ctx, const double *X1, const double *X2, const double *phi, double dx,
                double dy, int max_layers, double *X1o, double *X2o, int *dev_status) {
    const int ny = ctx->ny, nx = ctx->nx;
    const long n = (long)ny * nx;
    const int W = (nx + 63) / 64;
    if (max_layers <= 0) {
        if (X1o != X1) RMT_HIP(hipMemcpyAsync(X1o, X1, n * 8, hipMemcpyDeviceToDevice, ctx->stream));
        if (X2o != X2) RMT_HIP(hipMemcpyAsync(X2o, X2, n * 8, hipMemcpyDeviceToDevice, ctx->stream));
        return RMT_OK;
    }
    RMT_CHECK(ny >= 3 && nx >= 3 && ny < (1 << 20), RMT_EINVAL, "extrapolation grid size");
    RMT_TRY(ensure_bytes(ctx, extrap_workspace(ny, nx)));
    // byte workspace: kbits | cbits | layer bytes | row flags | jrange[2], status[4]
    u64 *kbits = (u64 *)ctx->bytes, *cbits = kbits + (size_t)ny * W;
    unsigned char *lay = (unsigned char *)(cbits + (size_t)ny * W);
    unsigned char *rowcand = lay + (n + 255) / 256 * 256;
    int *jrange = (int *)(rowcand + ((size_t)ny + 255) / 256 * 256), *status = jrange + 2;
    const int copy = (X1o != X1) || (X2o != X2);
    k_ex_bits<<<dim3((nx + 255) / 256, ny), 256, 0, ctx->stream>>>(phi, ny, nx, W, kbits, rowcand,
                                                                   jrange, X1, X2, X1o, X2o, copy);
    k_ex_dilate<<<grid1d((long)ny * W, 256), 256, 0, ctx->stream>>>(kbits, ny, nx, W, max_layers,
                                                                    cbits, lay, rowcand, jrange);
    RMT_HIP(hipMemsetAsync(status, 0, 4 * sizeof(int), ctx->stream));
    if (ctx->prof) RMT_HIP(hipEventRecord(ctx->ev[2], ctx->stream));
    ExSweep A{X1o, X2o, lay, kbits, cbits, rowcand, jrange, ny, nx, W, max_layers, dx, dy, status};
    k_ex_sweep<<<1, EXW * 64, 0, ctx->stream>>>(A);
    RMT_LAUNCHED();
    if (ctx->prof) RMT_HIP(hipEventRecord(ctx->ev[3], ctx->stream));
    if (dev_status)
        RMT_HIP(hipMemcpyAsync(dev_status, status, 2 * sizeof(int), hipMemcpyDeviceToDevice,
                               ctx->stream));
    return RMT_OK;
}

}  // namespace rmt

extern "C" int rmt_extrapolate_reference_map(rmt_ctx *ctx, const double *X1, const double *X2,
                                             const double *phi, double dx, double dy,
                                             int max_layers, double *X1_out, double *X2_out) {
    RMT_CHECK(ctx, RMT_EINVAL, "null ctx");
    return rmt::extrapolate(ctx, X1, X2, phi, dx, dy, max_layers, X1_out, X2_out, nullptr);
}
