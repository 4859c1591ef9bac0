// extrap_chain.hip -- functions.py:48-163 extrapolate_reference_map, geometry first.
//
// The reference fits the targets of a layer in raster order and marks each one known at once,
// so a fit sees every earlier accepted fit of its layer (Gauss-Seidel).  Everything a fit
// computes EXCEPT its right-hand sides is value-independent: which window cells are known
// (acceptance: count >= 3 and det > 1e-10 depends on the known set only), the weights
// w = exp(-d^2/r^2), the normal matrix Aw, its det and Cramer cofactors.  Only the sums
// Bw = sum w*a*X over the window (functions.py:128-133) read values that earlier fits produce.
// So the exact serial result is computed in three stages:
//
//   1. per layer, chip-wide: targets (k_tg_rows/scan/emit: bit planes, raster-order ids),
//      then one wave per target (k_ex_geom) computes the fit assuming every earlier target of
//      its layer was accepted, and emits a RECORD: Cramer constants, the partial sums of the
//      static (phi < 0) terms before the first value an earlier fit produces, and for every
//      later included cell either its 6 products w*a*X (static) or its 3 coefficients w*a
//      plus the id of the fit that produces X (dynamic).  Speculation is exact unless a target
//      is rejected: k_ex_fix then re-fits, Jacobi-style, every later target whose window holds
//      a rejected one until acceptance is a fixed point -- the DAG's unique fixed point is the
//      serial answer (acceptance only flows forward in raster order).
//   2. chain order (k_ex_order/chainidx/relink): fits are numbered in order of (j + 5L, L, i),
//      a topological order of the true dependency DAG (a layer-L fit reads layer L rows j-4..j
//      and layer L-1 rows j-4..j+4), and record sources are rewritten to chain indices.
//   3. k_ex_chain, one workgroup: waves take chain indices round-robin; a fit waits for its
//      dynamic sources in an LDS value ring (tag == chain index), forms their products, folds
//      the 6 ordered sums over its record terms (lanes 0-5) and runs the 3x3 solve of
//      utils.py:134-166 with the precomputed cofactors -- the same operations, in the same
//      order, as the reference, on the same values.
//
// Capacity limits (ids, record arena, fix-up lists, ring distance) set ctl[EXC_FALLBACK]
// on the device; extrap.hip then runs the row-ticket sweep instead.
#include "extrap.hpp"
#include "exp_glibc.h"
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

namespace rmt {

constexpr int EXS = 82;   // term-buffer row stride of the geometry fold (16-B aligned rows)
constexpr long long CH_CRIT = 1LL << 16;   // dyn entry term field: the fit's latest local source

__device__ __forceinline__ u64 ld_l2(const u64 *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int wave_incl_scan(int v, int lane) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int t = __shfl_up(v, d);
        if (lane >= d) v += t;
    }
    return v;
}
__device__ __forceinline__ u64 rl64(u64 v, int l) {
    const unsigned lo = __builtin_amdgcn_readlane((unsigned)v, l);
    const unsigned hi = __builtin_amdgcn_readlane((unsigned)(v >> 32), l);
    return ((u64)hi << 32) | lo;
}
__device__ __forceinline__ double rlf(double v, int l) {
    return __longlong_as_double((long long)rl64((u64)__double_as_longlong(v), l));
}
// raster rank -> id of the layer-Ls target at word o, bit mask `bit`
__device__ __forceinline__ int ex_id(const ExWs &ws, int ny, int Ls, int jj, long o, u64 bit) {
    return ws.ctl[EXC_BASE + Ls] + ws.rowoff[(long)Ls * (ny + 1) + jj] +
           ws.wordoff[(long)Ls * ws.plane + o] + __popcll(ws.T[(long)Ls * ws.plane + o] & (bit - 1));
}

// ------------------------------------------------------------------ 1. targets -----
// functions.py:79-90: targets of layer L = interior cells unknown at the start of L with a
// known 3x3 neighbour.  Known at the start of L: kbits (L = 0) or KN[L-1] = KN[L-2] | ACC[L-1],
// materialised here row by row.  One wave per row, lanes over 64-cell words; ACC[L] starts as
// T[L] (speculation), wordoff = exclusive popcount within the row, rowcnt = row total.
__global__ void __launch_bounds__(256) k_tg_rows(ExWs ws, int ny, int nx, int W, int L) {
    const int lane = threadIdx.x & 63, j = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (j >= ny) return;
    const long plane = ws.plane;
    const u64 *Kpp = L >= 2 ? ws.KN + (long)(L - 2) * plane : ws.kbits;
    const u64 *Ap = L >= 1 ? ws.ACC + (long)(L - 1) * plane : nullptr;
    auto K = [&](int jj, int w) -> u64 {
        if (jj < 0 || jj >= ny || w < 0 || w >= W) return 0;
        const long o = (long)jj * W + w;
        return Ap ? (Kpp[o] | Ap[o]) : Kpp[o];
    };
    int run = 0;
    for (int w0 = 0; w0 < W; w0 += 64) {
        const int w = w0 + lane;
        u64 t = 0;
        if (w < W) {
            u64 d = 0;
            for (int r = -1; r <= 1; ++r) {
                const u64 a = K(j + r, w - 1), b = K(j + r, w), c = K(j + r, w + 1);
                d |= b | (b << 1) | (a >> 63) | (b >> 1) | (c << 63);
            }
            const u64 k0 = K(j, w);
            const long o = (long)j * W + w;
            if (L >= 1) ws.KN[(long)(L - 1) * plane + o] = k0;
            const int i0 = 64 * w, lo = max(1, i0) - i0, hi = min(nx - 2, i0 + 63) - i0;
            u64 cols = hi >= lo ? (~0ull >> (63 - hi)) & (~0ull << lo) : 0;
            if (j < 1 || j > ny - 2) cols = 0;
            t = d & ~k0 & cols;
            ws.T[(long)L * plane + o] = t;
            ws.ACC[(long)L * plane + o] = t;
        }
        const int c = __popcll(t), inc = wave_incl_scan(c, lane);
        if (w < W) ws.wordoff[(long)L * plane + (long)j * W + w] = run + inc - c;
        run += __shfl(inc, 63);
    }
    if (lane == 0) ws.rowcnt[(long)L * ny + j] = run;
}

// exclusive scan of the row counts -> rowoff[L][j]; ids of layer L are base[L] + raster rank
__global__ void __launch_bounds__(1024) k_tg_scan(ExWs ws, int ny, int L) {
    __shared__ int part[1024];
    const int t = threadIdx.x, per = (ny + 1023) / 1024;
    const int j0 = min(ny, t * per), j1 = min(ny, j0 + per);
    const int *rc = ws.rowcnt + (long)L * ny;
    int s = 0;
    for (int j = j0; j < j1; ++j) s += rc[j];
    part[t] = s;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {
        const int v = t >= d ? part[t - d] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    int run = part[t] - s;
    int *ro = ws.rowoff + (long)L * (ny + 1);
    for (int j = j0; j < j1; ++j) { ro[j] = run; run += rc[j]; }
    if (t == 1023) {
        const int total = part[1023], b = ws.ctl[EXC_BASE + L];
        ro[ny] = total;
        ws.ctl[EXC_BASE + L + 1] = b + total;
        if ((long)b + total > ws.maxt) ws.ctl[EXC_FALLBACK] = 1;
    }
}

__global__ void __launch_bounds__(256) k_tg_emit(ExWs ws, int ny, int nx, int W, int L) {
    const int lane = threadIdx.x & 63, j = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (j >= ny || ws.ctl[EXC_FALLBACK]) return;
    const int base = ws.ctl[EXC_BASE + L] + ws.rowoff[(long)L * (ny + 1) + j];
    for (int w = lane; w < W; w += 64) {
        const long o = (long)L * ws.plane + (long)j * W + w;
        u64 t = ws.T[o];
        int id = base + ws.wordoff[o];
        for (; t; t &= t - 1, ++id) {
            ws.tcell[id] = (long)j * nx + 64 * w + __builtin_ctzll(t);
            ws.dmark[id] = -1;
        }
    }
}

// ------------------------------------------------------------------ 1. geometry ----
struct ExGeoArgs {
    ExWs ws;
    const double *X1, *X2;   // static values (phi < 0 cells are never written)
    int ny, nx, W, L;
    double dx, dy, r2;
    int norec;               // acceptance only, no record (the parallel mode)
};

// One wave fits target `id` of layer A.L.  Same-layer acceptance of earlier targets is read
// from T (FIX = false: speculation) or from ACC through L2 (FIX = true: k_ex_fix, where ACC
// changes inside the launch).  Emits the record's geometry if accepted (Cramer constants, the
// term layout, the dynamic sources and their coefficients -- everything the known plane
// decides); the values of the static terms (P and the static products) are filled in by
// k_ex_vals once the map is advected.  Returns acceptance (uniform).
template <bool FIX>
__device__ bool ex_geom(const ExGeoArgs &A, int id, double *tb, const u64 *tab, int lane) {
    const ExWs &ws = A.ws;
    const int L = A.L, W = A.W, nx = A.nx, ny = A.ny;
    const long plane = ws.plane, c = ws.tcell[id];
    const int j = (int)(c / nx), i = (int)(c % nx);
    const u64 *Kst = L == 0 ? ws.kbits : ws.KN + (long)(L - 1) * plane;
    const u64 *SL = (FIX ? ws.ACC : ws.T) + (long)L * plane;
    const double x0 = A.dx * i, y0 = A.dy * j;
    bool inc[2], st[2];
    double w[2], xi[2], yi[2];
    int src[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int q = lane + 64 * h, jj = j - 4 + q / 9, ii = i - 4 + q % 9;
        inc[h] = false; st[h] = false;
        w[h] = 0.0; src[h] = -1;
        xi[h] = A.dx * ii; yi[h] = A.dy * jj;
        if (q < 81 && jj >= 0 && jj < ny && ii >= 0 && ii < nx) {
            const double ax = xi[h] - x0, ay = yi[h] - y0, d2 = ax * ax + ay * ay;
            if (d2 <= A.r2) {
                const long o = (long)jj * W + (ii >> 6);
                const u64 bit = 1ull << (ii & 63);
                const bool ks = (Kst[o] & bit) != 0;
                bool sl = false;
                if (!ks && (jj < j || (jj == j && ii < i)))
                    sl = ((FIX ? ld_l2(SL + o) : SL[o]) & bit) != 0;
                inc[h] = ks || sl;
                if (inc[h]) {
                    w[h] = exp_glibc_tab(-d2 / A.r2, tab);   // libm exp, bit for bit
                    st[h] = (ws.kbits[o] & bit) != 0;
                    if (!st[h]) {
                        int Ls = L;
                        if (!sl)
                            for (Ls = 0; Ls < L; ++Ls)
                                if (ws.ACC[(long)Ls * plane + o] & bit) break;
                        src[h] = ex_id(ws, ny, Ls, jj, o, bit);
                    }
                }
            }
        }
    }
    // first dynamic window position (the static prefix before it is pre-summed)
    const u64 dl = __ballot(inc[0] && !st[0]), dh = __ballot(inc[1] && !st[1] && lane < 17);
    const int qf = dl ? __builtin_ctzll(dl) : (dh ? 64 + __builtin_ctzll(dh) : 81);
    // terms of functions.py:140-145: Aw over every included cell; excluded cells contribute
    // +0.0 (exact)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int q = lane + 64 * h;
        if (q >= 81) break;
        const double wa0 = w[h] * 1.0, wa1 = w[h] * xi[h], wa2 = w[h] * yi[h];
        tb[0 * EXS + q] = inc[h] ? wa0 * 1.0 : 0.0;
        tb[1 * EXS + q] = inc[h] ? wa0 * xi[h] : 0.0;
        tb[2 * EXS + q] = inc[h] ? wa0 * yi[h] : 0.0;
        tb[3 * EXS + q] = inc[h] ? wa1 * xi[h] : 0.0;
        tb[4 * EXS + q] = inc[h] ? wa1 * yi[h] : 0.0;
        tb[5 * EXS + q] = inc[h] ? wa2 * yi[h] : 0.0;
    }
    const u64 il = __ballot(inc[0]), ih = __ballot(inc[1] && lane < 17);
    const int count = __popcll(il) + __popcll(ih);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    double acc = 0.0;
    if (lane < 6) {
        const double2 *t2 = (const double2 *)(tb + lane * EXS);
        double2 t[40];
#pragma unroll
        for (int q2 = 0; q2 < 40; ++q2) t[q2] = t2[q2];
        const double last = tb[lane * EXS + 80];
#pragma unroll
        for (int q2 = 0; q2 < 40; ++q2) { acc += t[q2].x; acc += t[q2].y; }
        acc += last;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    const double A00 = rlf(acc, 0), A01 = rlf(acc, 1), A02 = rlf(acc, 2);
    const double A11 = rlf(acc, 3), A12 = rlf(acc, 4), A22 = rlf(acc, 5);
    const double M[9] = {A00, A01, A02, A01, A11, A12, A02, A12, A22};
    const double det = (M[0] * (M[4] * M[8] - M[5] * M[7])
                      - M[1] * (M[3] * M[8] - M[5] * M[6])
                      + M[2] * (M[3] * M[7] - M[4] * M[6]));
    const bool accept = count >= 3 && fabs(det) > 1e-10;
    if (!accept) {
        if (lane == 0) ws.recoff[id] = -1;
        return false;
    }
    if (A.norec) return true;
    // record: compact the included cells from qf on (static: 6 products; dynamic: 3 coefs)
    const u64 lt = (1ull << lane) - 1;
    const u64 tl = il & ~((qf >= 64) ? ~0ull : ((1ull << qf) - 1));
    const u64 th = ih & ~((qf >= 64) ? ((1ull << (qf - 64)) - 1) : 0ull);
    const int n = __popcll(tl) + __popcll(th), npad = (n + 7) & ~7;
    const int nd = __popcll(dl) + __popcll(dh);
    const long long bytes = ((8LL * (CH_HDR + 4 * nd + 6 * npad)) + 63) & ~63LL;
    unsigned long long off = 0;
    if (nd > 64) {   // k_ex_chain forms one product per lane
        if (lane == 0) { ws.ctl[EXC_FALLBACK] = 1; ws.recoff[id] = -1; }
        return true;
    }
    if (ws.slots) {
        off = (unsigned long long)id * CH_MAXREC;   // bytes <= CH_MAXREC (nd <= 64)
    } else {
        if (lane == 0) {
            off = atomicAdd((unsigned long long *)(ws.ctl + EXC_ARENA), (unsigned long long)bytes);
            if ((long long)(off + bytes) > ws.arena_bytes) ws.ctl[EXC_FALLBACK] = 1;
        }
        off = rl64(off, 0);
    }
    if ((long long)(off + bytes) > ws.arena_bytes) {
        if (lane == 0) ws.recoff[id] = -1;
        return true;   // (fallback sweep recomputes everything)
    }
    double *rec = (double *)(ws.arena + off);
    double *dyn = rec + CH_HDR;           // nd entries {(k, src), w*1, w*x, w*y}
    double *tv = dyn + 4 * nd;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const bool term = h ? ((th >> lane) & 1) && lane < 17 : (tl >> lane) & 1;
        if (!term) continue;
        const int k = h ? __popcll(tl) + __popcll(th & lt) : __popcll(tl & lt);
        const double wa0 = w[h] * 1.0, wa1 = w[h] * xi[h], wa2 = w[h] * yi[h];
        if (!st[h]) {   // (static products: k_ex_vals)
            const int dk = h ? __popcll(dl) + __popcll(dh & lt) : __popcll(dl & lt);
            dyn[4 * dk] = __longlong_as_double(((long long)src[h] << 32) | (unsigned)k);
            dyn[4 * dk + 1] = wa0; dyn[4 * dk + 2] = wa1; dyn[4 * dk + 3] = wa2;
        }
    }
    if (lane < 6 * (npad - n)) tv[(lane / (npad - n)) * npad + n + lane % (npad - n)] = 0.0;
    if (lane == 0) {
        rec[0] = __longlong_as_double((long long)c);
        rec[1] = __longlong_as_double(((long long)nd << 32) | (unsigned)npad);
        rec[2] = x0; rec[3] = y0;
        for (int k = 0; k < 9; ++k) rec[4 + k] = M[k];
        rec[13] = M[4] * M[8] - M[5] * M[7];
        rec[14] = M[3] * M[8] - M[5] * M[6];
        rec[15] = M[3] * M[7] - M[4] * M[6];
        rec[16] = 1.0 / det;
        rec[23] = 0.0;
    }
    if (lane == 0) ws.recoff[id] = ((long long)(bytes >> 6) << 32) | (long long)(off >> 6);
    return true;
}

__global__ void __launch_bounds__(256) k_ex_geom(ExGeoArgs A) {
    __shared__ u64 tab[256];
    __shared__ __attribute__((aligned(16))) double tb[4][6 * EXS];
    for (int s = threadIdx.x; s < 256; s += blockDim.x) tab[s] = kExpTab[s];
    __syncthreads();
    const ExWs &ws = A.ws;
    if (ws.ctl[EXC_FALLBACK]) return;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int b0 = ws.ctl[EXC_BASE + A.L], b1 = ws.ctl[EXC_BASE + A.L + 1];
    for (int id = b0 + blockIdx.x * 4 + wv; id < b1; id += gridDim.x * 4) {
        if (ex_geom<false>(A, id, tb[wv], tab, lane) || lane != 0) continue;
        const long c = ws.tcell[id];
        const int j = (int)(c / A.nx), i = (int)(c % A.nx);
        atomicAnd(ws.ACC + (long)A.L * ws.plane + (long)j * A.W + (i >> 6), ~(1ull << (i & 63)));
        const int r = atomicAdd(ws.ctl + EXC_REJ + A.L, 1);
        if (r < EX_MAXREJ) ws.rej[A.L * EX_MAXREJ + r] = id;
        else ws.ctl[EXC_FALLBACK] = 1;
    }
}


__device__ __forceinline__ int ch_base(const int *ctl, int p);


// ------------------------------------------------------------------ 1. values ------
// The value half of a record (k_ex_geom wrote the geometry): P[0..5] = the ordered sums of
// the static terms before the first dynamic one (functions.py:128-138, window order), and
// the 6 products w*a*X of every static term from there on, at the record's term slots.  The
// same window analysis as ex_geom (final same-layer acceptance from ACC), the same operands.
// One wave per accepted fit, every layer in one launch.
__global__ void __launch_bounds__(256) k_ex_vals(ExGeoArgs A, int ML) {
    __shared__ u64 tab[256];
    __shared__ __attribute__((aligned(16))) double tb[4][6 * EXS];
    for (int s = threadIdx.x; s < 256; s += blockDim.x) tab[s] = kExpTab[s];
    __syncthreads();
    const ExWs &ws = A.ws;
    if (ws.ctl[EXC_FALLBACK]) return;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int total = ws.ctl[EXC_BASE + ML];
    const int W = A.W, nx = A.nx, ny = A.ny;
    const long plane = ws.plane;
    double *T = tb[wv];
    for (int id = blockIdx.x * 4 + wv; id < total; id += gridDim.x * 4) {
        const long long r = ws.recoff[id];
        if (r < 0) continue;
        int L = ML - 1;
        while (L > 0 && id < ws.ctl[EXC_BASE + L]) --L;
        const long c = ws.tcell[id];
        const int j = (int)(c / nx), i = (int)(c % nx);
        const u64 *Kst = L == 0 ? ws.kbits : ws.KN + (long)(L - 1) * plane;
        const u64 *SL = ws.ACC + (long)L * plane;
        const double x0 = A.dx * i, y0 = A.dy * j;
        bool inc[2], st[2];
        double w[2], xi[2], yi[2], b1[2], b2[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int q = lane + 64 * h, jj = j - 4 + q / 9, ii = i - 4 + q % 9;
            inc[h] = false; st[h] = false;
            w[h] = 0.0; b1[h] = 0.0; b2[h] = 0.0;
            xi[h] = A.dx * ii; yi[h] = A.dy * jj;
            if (q < 81 && jj >= 0 && jj < ny && ii >= 0 && ii < nx) {
                const double ax = xi[h] - x0, ay = yi[h] - y0, d2 = ax * ax + ay * ay;
                if (d2 <= A.r2) {
                    const long o = (long)jj * W + (ii >> 6);
                    const u64 bit = 1ull << (ii & 63);
                    const bool ks = (Kst[o] & bit) != 0;
                    bool sl = false;
                    if (!ks && (jj < j || (jj == j && ii < i))) sl = (SL[o] & bit) != 0;
                    inc[h] = ks || sl;
                    if (inc[h]) {
                        st[h] = (ws.kbits[o] & bit) != 0;
                        if (st[h]) {
                            w[h] = exp_glibc_tab(-d2 / A.r2, tab);   // libm exp, bit for bit
                            const long cc = (long)jj * nx + ii;
                            b1[h] = A.X1[cc]; b2[h] = A.X2[cc];
                        }
                    }
                }
            }
        }
        const u64 dl = __ballot(inc[0] && !st[0]), dh = __ballot(inc[1] && !st[1] && lane < 17);
        const int qf = dl ? __builtin_ctzll(dl) : (dh ? 64 + __builtin_ctzll(dh) : 81);
        // the Bw prefix: static cells before qf (functions.py:133-138 order), +0.0 elsewhere
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int q = lane + 64 * h;
            if (q >= 81) break;
            const double wa0 = w[h] * 1.0, wa1 = w[h] * xi[h], wa2 = w[h] * yi[h];
            const bool pre = st[h] && q < qf;
            T[0 * EXS + q] = pre ? wa0 * b1[h] : 0.0;
            T[1 * EXS + q] = pre ? wa1 * b1[h] : 0.0;
            T[2 * EXS + q] = pre ? wa2 * b1[h] : 0.0;
            T[3 * EXS + q] = pre ? wa0 * b2[h] : 0.0;
            T[4 * EXS + q] = pre ? wa1 * b2[h] : 0.0;
            T[5 * EXS + q] = pre ? wa2 * b2[h] : 0.0;
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        double acc = 0.0;
        if (lane < 6) {
            const double2 *t2 = (const double2 *)(T + lane * EXS);
            double2 t[40];
#pragma unroll
            for (int q2 = 0; q2 < 40; ++q2) t[q2] = t2[q2];
            const double last = T[lane * EXS + 80];
#pragma unroll
            for (int q2 = 0; q2 < 40; ++q2) { acc += t[q2].x; acc += t[q2].y; }
            acc += last;
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        // static products from qf on, at the compact term slots of ex_geom's record
        double *rec = (double *)(ws.arena + ((r & 0xffffffffLL) << 6));
        const long long meta = __double_as_longlong(rec[1]);
        const int npad = (int)(meta & 0xffffffff), nd = (int)((meta >> 32) & 0x7fffffff);
        double *tv = rec + CH_HDR + 4 * nd;
        const u64 il = __ballot(inc[0]), ih = __ballot(inc[1] && lane < 17);
        const u64 lt = (1ull << lane) - 1;
        const u64 tl = il & ~((qf >= 64) ? ~0ull : ((1ull << qf) - 1));
        const u64 th = ih & ~((qf >= 64) ? ((1ull << (qf - 64)) - 1) : 0ull);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const bool term = h ? ((th >> lane) & 1) && lane < 17 : (tl >> lane) & 1;
            if (!term || !st[h]) continue;
            const int k = h ? __popcll(tl) + __popcll(th & lt) : __popcll(tl & lt);
            const double wa0 = w[h] * 1.0, wa1 = w[h] * xi[h], wa2 = w[h] * yi[h];
            tv[0 * npad + k] = wa0 * b1[h]; tv[1 * npad + k] = wa1 * b1[h];
            tv[2 * npad + k] = wa2 * b1[h]; tv[3 * npad + k] = wa0 * b2[h];
            tv[4 * npad + k] = wa1 * b2[h]; tv[5 * npad + k] = wa2 * b2[h];
        }
        if (lane < 6) rec[17 + lane] = acc;   // P[0..5]
    }
}

// ------------------------------------------------------------------ 1. fix-up ------
constexpr int FIXW = 8;

// append the later same-layer targets whose window holds target `id` (dedup by dmark)
__device__ void ex_add_dependents(const ExGeoArgs &A, int id, int *dlist, int *dn) {
    const ExWs &ws = A.ws;
    const long c = ws.tcell[id];
    const int j = (int)(c / A.nx), i = (int)(c % A.nx);
    const u64 *T = ws.T + (long)A.L * ws.plane;
    for (int jj = j; jj <= min(A.ny - 1, j + 4); ++jj)
        for (int ii = max(0, i - 4); ii <= min(A.nx - 1, i + 4); ++ii) {
            if (jj == j && ii <= i) continue;
            const long o = (long)jj * A.W + (ii >> 6);
            const u64 bit = 1ull << (ii & 63);
            if (!(T[o] & bit)) continue;
            const int d = ex_id(ws, A.ny, A.L, jj, o, bit);
            if (atomicExch(ws.dmark + d, 1) == 1) continue;
            const int p = atomicAdd(dn, 1);
            if (p < EX_DCAP) dlist[p] = d;
        }
}

// Jacobi re-fits of the targets downstream of rejections until acceptance is a fixed point.
__global__ void __launch_bounds__(FIXW * 64) k_ex_fix(ExGeoArgs A) {
    __shared__ u64 tab[256];
    __shared__ __attribute__((aligned(16))) double tb[FIXW][6 * EXS];
    __shared__ int dlist[EX_DCAP];
    __shared__ unsigned char dres[EX_DCAP];
    __shared__ int dn, nflip;
    const ExWs &ws = A.ws;
    const int nrej = ws.ctl[EXC_REJ + A.L];
    if (nrej == 0 || ws.ctl[EXC_FALLBACK]) return;
    for (int s = threadIdx.x; s < 256; s += blockDim.x) tab[s] = kExpTab[s];
    if (threadIdx.x == 0) dn = 0;
    __syncthreads();
    for (int r = threadIdx.x; r < min(nrej, EX_MAXREJ); r += blockDim.x)
        ex_add_dependents(A, ws.rej[A.L * EX_MAXREJ + r], dlist, &dn);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const u64 *ACC = ws.ACC + (long)A.L * ws.plane;
    for (int iter = 0;; ++iter) {
        __syncthreads();
        const int m = dn;
        if (m > EX_DCAP || iter > (1 << 20)) {
            if (threadIdx.x == 0) ws.ctl[EXC_FALLBACK] = 1;
            return;
        }
        for (int e = wv; e < m; e += FIXW) {
            const bool a = ex_geom<true>(A, dlist[e], tb[wv], tab, lane);
            if (lane == 0) dres[e] = a;
        }
        if (threadIdx.x == 0) nflip = 0;
        __syncthreads();
        for (int e = threadIdx.x; e < m; e += blockDim.x) {
            const long c = ws.tcell[dlist[e]];
            const int j = (int)(c / A.nx), i = (int)(c % A.nx);
            const long o = (long)j * A.W + (i >> 6);
            const u64 bit = 1ull << (i & 63);
            const bool cur = (ld_l2(ACC + o) & bit) != 0;
            if (cur != (bool)(dres[e] & 1)) {
                atomicXor((u64 *)ACC + o, bit);
                dres[e] |= 2;
                atomicAdd(&nflip, 1);
            }
        }
        __threadfence();
        __syncthreads();
        if (nflip == 0) break;
        for (int e = threadIdx.x; e < m; e += blockDim.x)
            if (dres[e] & 2) ex_add_dependents(A, dlist[e], dlist, &dn);
        __threadfence();
    }
}

// ------------------------------------------------------------------ 2. chain order -
// chain order (k = j + 5L, L, i): exclusive scan of the row counts over (k, L) slots
__global__ void __launch_bounds__(1024) k_ex_order(ExWs ws, int ny, int ML) {
    __shared__ int part[1024];
    if (ws.ctl[EXC_FALLBACK]) return;
    const int t = threadIdx.x, nslot = (ny + 5 * (ML - 1)) * ML, per = (nslot + 1023) / 1024;
    const int s0 = min(nslot, t * per), s1 = min(nslot, s0 + per);
    auto cnt = [&](int s) {
        const int L = s % ML, j = s / ML - 5 * L;
        return j >= 0 && j < ny ? ws.rowcnt[(long)L * ny + j] : 0;
    };
    int sum = 0;
    for (int s = s0; s < s1; ++s) sum += cnt(s);
    part[t] = sum;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {
        const int v = t >= d ? part[t - d] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    int run = part[t] - sum;
    for (int s = s0; s < s1; ++s) {
        const int L = s % ML, j = s / ML - 5 * L;
        if (j >= 0 && j < ny) ws.cbase[(long)L * ny + j] = run;
        run += cnt(s);
    }
}

// chain parts: split column = middle of the targets' column range (ncol == 2), so the two
// sides of the band run apart; the few fits near the split column hand their values across
// through L2 / the fabric, as every fit read by a later layer group does
__global__ void __launch_bounds__(1024) k_ex_split(ExWs ws, int nx, int ML, int ncol, int nlg) {
    __shared__ int smin[1024], smax[1024];
    const int t = threadIdx.x, total = ws.ctl[EXC_BASE + ML];
    int mn = 0x7fffffff, mx = -1;
    for (int id = t; id < total; id += 1024) {
        const int i = (int)(ws.tcell[id] % nx);
        mn = min(mn, i); mx = max(mx, i);
    }
    smin[t] = mn; smax[t] = mx;
    __syncthreads();
    for (int w = 512; w > 0; w >>= 1) {
        if (t < w) { smin[t] = min(smin[t], smin[t + w]); smax[t] = max(smax[t], smax[t + w]); }
        __syncthreads();
    }
    if (t == 0) {
        ws.ctl[EXC_CMIN] = smin[0];
        ws.ctl[EXC_CMAX] = smax[0] >= smin[0] ? smax[0] - smin[0] + 1 : 1;   // span
        ws.ctl[EXC_NCOL] = ncol;
        ws.ctl[EXC_NLG] = nlg;
        ws.ctl[EXC_NPART + CH_MAXP] = ncol * nlg;
    }
}
// column range of a target column: EXC_NCOL equal ranges over the targets' span
__device__ __forceinline__ int ch_col_of(const int *ctl, int i) {
    const int np = ctl[EXC_NCOL];
    if (np <= 1) return 0;
    const long q = (long)(i - ctl[EXC_CMIN]) * np / ctl[EXC_CMAX];
    return (int)min((long)np - 1, max(0L, q));
}

__global__ void __launch_bounds__(256) k_ex_chainidx(ExWs ws, int ny, int nx, int ML,
                                                     int *status) {
    if (ws.ctl[EXC_FALLBACK]) return;
    const int id = blockIdx.x * 256 + threadIdx.x, total = ws.ctl[EXC_BASE + ML];
    bool acc = false;
    if (id < total) {
        int L = ML - 1;
        while (L > 0 && id < ws.ctl[EXC_BASE + L]) --L;
        const int j = (int)(ws.tcell[id] / nx);
        const int x = ws.cbase[(long)L * ny + j] +
                      (id - ws.ctl[EXC_BASE + L] - ws.rowoff[(long)L * (ny + 1) + j]);
        ws.chain_of[id] = x;
        // part = (column range, layer group): a layer's fits read the previous layers' only
        // ~5 rows ahead of their own chain position (k_ex_order), so a layer group on a
        // workgroup of its own hands values over off the critical path
        const int nlg = ws.ctl[EXC_NLG];
        ws.part[x] = (unsigned char)(ch_col_of(ws.ctl, (int)(ws.tcell[id] % nx)) * nlg +
                                     L * nlg / ML);
        const long long r = ws.recoff[id];
        ws.rec_by_chain[x] = r;
        acc = r >= 0;
    }
    const u64 b = __ballot(acc);
    if ((threadIdx.x & 63) == 0 && b) atomicAdd(status, __popcll(b));
}

// ordinals within the parts (chain order kept inside each part), their inverse, the part
// sizes (ctl[EXC_NPART + p]); resets the cross-part hand-off tags.  One block.
__global__ void __launch_bounds__(1024) k_ex_local(ExWs ws, int ML) {
    __shared__ int sc[CH_MAXP][1024];
    if (ws.ctl[EXC_FALLBACK]) return;
    const int t = threadIdx.x, total = ws.ctl[EXC_BASE + ML], per = (total + 1023) / 1024;
    const int a = min(total, t * per), b = min(total, a + per);
    int cnt[CH_MAXP];
#pragma unroll
    for (int p = 0; p < CH_MAXP; ++p) cnt[p] = 0;
    for (int x = a; x < b; ++x) {
        const int px = ws.part[x];
#pragma unroll
        for (int p = 0; p < CH_MAXP; ++p) cnt[p] += px == p;
    }
#pragma unroll
    for (int p = 0; p < CH_MAXP; ++p) sc[p][t] = cnt[p];
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {
        int v[CH_MAXP];
#pragma unroll
        for (int p = 0; p < CH_MAXP; ++p) v[p] = t >= d ? sc[p][t - d] : 0;
        __syncthreads();
#pragma unroll
        for (int p = 0; p < CH_MAXP; ++p) sc[p][t] += v[p];
        __syncthreads();
    }
    int base[CH_MAXP], run[CH_MAXP];
    int acc = 0;
#pragma unroll
    for (int p = 0; p < CH_MAXP; ++p) {
        base[p] = acc; acc += sc[p][1023];
        run[p] = sc[p][t] - cnt[p];
    }
    for (int x = a; x < b; ++x) {
        const int px = ws.part[x];
        int l = 0, bs = 0;
#pragma unroll
        for (int p = 0; p < CH_MAXP; ++p)
            if (px == p) { l = run[p]++; bs = base[p]; }
        ws.loc[x] = l;
        ws.inv[bs + l] = x;
        ((u64 *)ws.gval)[2 * x] = CH_GSENT;      // (slots 0 .. total - 1 in any order)
        ((u64 *)ws.gval)[2 * x + 1] = CH_GSENT;
    }
    if (t == 1023) {
#pragma unroll
        for (int p = 0; p < CH_MAXP; ++p) { ws.ctl[EXC_NPART + p] = sc[p][1023]; }
    }
}
__device__ __forceinline__ int ch_base(const int *ctl, int p) {
    int b = 0;
    for (int q = 0; q < p; ++q) b += ctl[EXC_NPART + q];
    return b;
}

// Wave assignment of part blockIdx.x: ordinal l on wave l % CH_W (round robin: a fit's record
// staging and prefix fold overlap its predecessors' waits; giving each row run of fits to one
// wave measured slower in round 3, 4.32 vs 3.0 ms at N=4096).  One block per part.
__global__ void __launch_bounds__(1024) k_ex_runs(ExWs ws) {
    if (ws.ctl[EXC_FALLBACK]) return;
    const int p = blockIdx.x, t = threadIdx.x;
    if (p >= ws.ctl[EXC_NPART + CH_MAXP]) return;
    const int np = ws.ctl[EXC_NPART + p], base = ch_base(ws.ctl, p);
    int *wst = ws.ctl + EXC_WSTART + p * CH_W;
    for (int l = t; l < np; l += 1024) ws.wnext[base + l] = l + CH_W;
    if (t < CH_W) wst[t] = min(t, np);
}

// record sources: fit ids -> ring tags within the fit's part (the ring needs every source
// < CH_R/2 back), or -(global slot + 1) for a source in the other part (marked for the HBM
// hand-off); header word 23 <- (ordinal, record) of the next accepted fit of the same chain
// wave of the part
// One wave per fit, lanes over its dynamic sources (the per-source lookups are independent
// dependent-load chains: a thread per fit walked them serially, ~90 us at N=4096).
__global__ void __launch_bounds__(256) k_ex_relink(ExWs ws, int ML) {
    if (ws.ctl[EXC_FALLBACK]) return;
    const int lane = threadIdx.x & 63, total = ws.ctl[EXC_BASE + ML];
    for (int id = blockIdx.x * 4 + (int)(threadIdx.x >> 6); id < total; id += gridDim.x * 4) {
        const long long r = ws.recoff[id];
        if (r < 0) continue;
        double *rec = (double *)(ws.arena + ((r & 0xffffffffLL) << 6));
        // meta bit 63 (set here by the readers in other parts): publish to HBM as well
        const long long meta = __double_as_longlong(rec[1]);
        const int nd = (int)((meta >> 32) & 0x7fffffff);
        int2 *dyn = (int2 *)(rec + CH_HDR);   // entry d at int2 index 2d: (k, src)
        const int x = ws.chain_of[id], p = ws.part[x], l = ws.loc[x];
        const int np = ws.ctl[EXC_NPART + p], base = ch_base(ws.ctl, p);
        int lmax = -1, dmax = -1;   // the latest local source: its ordinal, entry
        for (int d = lane; d < nd; d += 64) {
            const int src = dyn[4 * d].y;
            const int xs = ws.chain_of[src];
            dyn[4 * d].x &= 0xffff;
            if (xs >= x) { ws.ctl[EXC_ABORT] = 1; exa_report(ws.status, exa_code(EXA_RELINK, p, l)); }   // a bug
            if (ws.part[xs] == p) {
                const int ls = ws.loc[xs];
                dyn[4 * d].y = ls;
                if (ls > lmax) { lmax = ls; dmax = d; }
                if (l - ls >= CH_R / 2) ws.ctl[EXC_FALLBACK] = 1;
            } else {
                const int g = ch_base(ws.ctl, ws.part[xs]) + ws.loc[xs];
                dyn[4 * d].y = -(g + 1);
                const long long rs = ws.rec_by_chain[xs];
                double *srec = (double *)(ws.arena + ((rs & 0xffffffffLL) << 6));
                atomicOr((unsigned long long *)&srec[1], 1ull << 63);
            }
        }
        {
            // mark the latest local source (ordinals of distinct fits differ)
            int m = lmax;
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) m = max(m, __shfl_xor(m, off));
            if (m >= 0 && lmax == m) dyn[4 * dmax].x |= (int)CH_CRIT;
        }
        if (lane == 0) {
            int ln = ws.wnext[base + l];
            while (ln < np && ws.rec_by_chain[ws.inv[base + ln]] < 0) ln = ws.wnext[base + ln];
            const long long rn = ln < np ? ws.rec_by_chain[ws.inv[base + ln]] : 0;   // (size64 << 32) | off64
            const unsigned r32 = (unsigned)(rn & 0xffffffffLL) | ((unsigned)(rn >> 32) << 25);
            rec[23] = __longlong_as_double(((long long)ln << 32) | r32);
        }
    }
}

// ------------------------------------------------------------------ 3. the chain ---
constexpr int CH_XL2 = 3;   // the lane of a fit's X2 result (ch_fit)
#ifndef RMT_CH_POLL_PRIO
#define RMT_CH_POLL_PRIO 3   // wave priority while polling a fit's critical source (the
#endif                       // highest: 0 measured 2.19 ms per chain, 2 2.15, 3 2.15)
#ifndef RMT_CH_WORK_PRIO
#define RMT_CH_WORK_PRIO 1   // ... during a fit's pre-arrival work (0: 2.17 ms, no better)
#endif
#ifndef RMT_CH_ABL
#define RMT_CH_ABL 0   // timing ablations (wrong results, A/B only): 1 no tail fold, 2 no
#endif                 // solve, 4 no waits for sources
constexpr int CH_BUFD = CH_MAXREC / 8 + 32;   // doubles per wave record buffer (+ the tail
                                              // prefetch's NRT = 24 reads past a short record)
constexpr long CH_SPIN_LIMIT = 1L << 25;

struct ChainArgs {
    ExWs ws;
    double *X1e, *X2e;
    int ML;
    int *status;
    long long *trace;   // PROF diagnostic: per fit {start, ready, published, critical source,
                        // wave, cell} (s_memrealtime), indexed by global chain slot
};

// record r (packed: 64-B units of offset | size << 25) -> five 16-B pieces per lane; every
// lane issues the same 5 loads (lanes past the record re-read its last piece, same line).
// Plain named registers, not an aggregate: an aggregate gets promoted to LDS, which turns the
// prefetch into a synchronous copy.
#define CH_LOAD(r)                                                                   \
    do {                                                                             \
        const double2 *p_ = (const double2 *)(arena + ((size_t)((r) & 0x1ffffff) << 6)); \
        const int l_ = (int)(((r) >> 25) << 2) - 1;                                  \
        d0 = p_[min(lane, l_)];        d1 = p_[min(64 + lane, l_)];                  \
        d2 = p_[min(128 + lane, l_)];  d3 = p_[min(192 + lane, l_)];                 \
        d4 = p_[min(256 + lane, l_)];                                                \
    } while (0)
#define CH_STAGE(r)                                                                  \
    do {                                                                             \
        const int n_ = (int)(((r) >> 25) << 2);                                      \
        double2 *B2 = (double2 *)B;                                                  \
        if (lane < n_) B2[lane] = d0;                                                \
        if (64 + lane < n_) B2[64 + lane] = d1;                                      \
        if (128 + lane < n_) B2[128 + lane] = d2;                                    \
        if (192 + lane < n_) B2[192 + lane] = d3;                                    \
        if (256 + lane < n_) B2[256 + lane] = d4;                                    \
    } while (0)

// One fit of the chain: chain index x whose record is staged in this wave's buffer B.
// LDS hand-offs: a fit writes its value pair, then its tag; a reader that sees the tag reads
// the values afterwards (one wave's LDS operations are performed in issue order), so no
// fence is needed -- and none is wanted: a workgroup fence would also drain the record
// prefetch in flight.  Returns false on a timeout (bug guard).
#define CH_STAMP(k)                                                    \
    if constexpr (PROF) {                                              \
        const long long t_ = __builtin_amdgcn_s_memtime();             \
        pr[k] += t_ - tl; tl = t_;                                     \
    }
// fold row[8*c0 .. 8*c1) into acc in order: 4-term groups, four groups of reads in flight
// (a group's 4 dependent adds, 32 clk, against an LDS read latency of ~70-100 clk).  The
// reads run up to three groups past the end unconditionally (unused; LDS reads never fault):
// conditional reads made the compiler copy registers and drain every read at each copy.
__device__ __forceinline__ double ch_fold(double acc, const double *row, int c0, int c1) {
    if (c0 >= c1) return acc;
    const double2 *r2 = (const double2 *)row;
    const int g0 = 2 * c0, g1 = 2 * c1;   // 4-term groups: double2 pairs 2g, 2g + 1
    double2 s0a = r2[2 * g0], s0b = r2[2 * g0 + 1];
    double2 s1a = r2[2 * g0 + 2], s1b = r2[2 * g0 + 3];
    double2 s2a = r2[2 * g0 + 4], s2b = r2[2 * g0 + 5];
    double2 s3a = r2[2 * g0 + 6], s3b = r2[2 * g0 + 7];
    __builtin_amdgcn_sched_barrier(0);
    for (int g = g0;; g += 4) {
        acc += s0a.x; acc += s0a.y; acc += s0b.x; acc += s0b.y;
        if (g + 1 >= g1) break;
        s0a = r2[2 * g + 8]; s0b = r2[2 * g + 9];
        __builtin_amdgcn_sched_barrier(0);   // the reads stay issued here, ahead of use
        acc += s1a.x; acc += s1a.y; acc += s1b.x; acc += s1b.y;
        if (g + 2 >= g1) break;
        s1a = r2[2 * g + 10]; s1b = r2[2 * g + 11];
        __builtin_amdgcn_sched_barrier(0);
        acc += s2a.x; acc += s2a.y; acc += s2b.x; acc += s2b.y;
        if (g + 3 >= g1) break;
        s2a = r2[2 * g + 12]; s2b = r2[2 * g + 13];
        __builtin_amdgcn_sched_barrier(0);
        acc += s3a.x; acc += s3a.y; acc += s3b.x; acc += s3b.y;
        if (g + 4 >= g1) break;
        s3a = r2[2 * g + 14]; s3b = r2[2 * g + 15];
        __builtin_amdgcn_sched_barrier(0);
    }
    return acc;
}


__device__ __forceinline__ double dpp_shl(double v, int ctrl) {
    // row_shl:1 = 0x101, row_shl:2 = 0x102 (lanes read lane + k within their 16-lane row)
    const int lo = __double2loint(v), hi = __double2hiint(v);
    const int l2 = ctrl == 1 ? __builtin_amdgcn_update_dpp(0, lo, 0x101, 0xf, 0xf, false)
                             : __builtin_amdgcn_update_dpp(0, lo, 0x102, 0xf, 0xf, false);
    const int h2 = ctrl == 1 ? __builtin_amdgcn_update_dpp(0, hi, 0x101, 0xf, 0xf, false)
                             : __builtin_amdgcn_update_dpp(0, hi, 0x102, 0xf, 0xf, false);
    return __hiloint2double(h2, l2);
}

// terms [lo, hi) of the 8-term chunk c of row (lo, hi within the chunk), in order: the chunk's
// four 16-byte reads issued together
__device__ __forceinline__ double ch_part(double acc, const double *row, int c, int lo, int hi) {
    const double2 *r2 = (const double2 *)(row + 8 * c);
    const double2 a = r2[0], b = r2[1], d = r2[2], e = r2[3];
    const double t[8] = {a.x, a.y, b.x, b.y, d.x, d.y, e.x, e.y};
    lo -= 8 * c; hi -= 8 * c;
#pragma unroll
    for (int k = 0; k < 8; ++k)
        if (k >= lo && k < hi) acc += t[k];
    return acc;
}
// row[a .. b) in order: partial head chunk, whole chunks (ch_fold: 4-term groups, three
// groups of reads ahead), partial last chunk
__device__ __forceinline__ double ch_fold_span(double acc, const double *row, int a, int b) {
    if (a >= b) return acc;
    const int ca = a >> 3, cb = b >> 3;
    if (ca == cb) return ch_part(acc, row, ca, a, b);
    if (a & 7) acc = ch_part(acc, row, ca, a, 8 * ca + 8);
    acc = ch_fold(acc, row, (a + 7) >> 3, cb);
    if (b & 7) acc = ch_part(acc, row, cb, 8 * cb, b);
    return acc;
}

// One fit of the chain, chain index x, its record staged in this wave's buffer B.  The fit's latest local source in chain order (marked CH_CRIT by
// k_ex_relink) is the one its predecessor link hands over; everything else is done before it
// arrives: the other sources' products (written to the staged record's term rows as they
// arrive), the fold of the terms before the critical one's window position kc, and the
// first reads of the terms after it.  The critical value is polled with one broadcast LDS
// read of its tag and value (issued back to back: a wave's LDS operations are performed in
// order, and the producer writes the value before the tag), its product is added in
// registers -- never written to LDS -- and the terms after kc follow: the reference's order,
// the same operations.
template <bool PROF>
__device__ __forceinline__ bool ch_fit(int x, int lane, double *B, double2 *val, int *tag,
                                        int *cur, int &wm, double &o_out, long &c_out,
                                        long long *pr, long long &tl, double *gval,
                                        int gslot, long long *trace = nullptr, int base = 0) {
    long long tr_start = 0, tr_ready = 0;
    int tr_crit = -1, tr_far = -1;   // the critical local ordinal / far global slot (PROF)
    long spins = 0;
    while (x - CH_R / 2 >= wm) {
        int m = 0x7fffffff;
        for (int k = 0; k < CH_W; ++k)
            m = min(m, __hip_atomic_load(&cur[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
        wm = m;
        if (x - CH_R / 2 >= wm) {
            if (++spins > CH_SPIN_LIMIT) return false;
            __builtin_amdgcn_s_sleep(1);
        }
    }
    CH_STAMP(1);
    if constexpr (PROF) tr_start = __builtin_amdgcn_s_memrealtime();
    const long long meta = __double_as_longlong(B[1]);
    const int npad = __builtin_amdgcn_readfirstlane((int)(meta & 0xffffffff));
    const int nd = __builtin_amdgcn_readfirstlane((int)((meta >> 32) & 0x7fffffff));
    const bool pub = __builtin_amdgcn_readfirstlane((int)((unsigned long long)meta >> 63)) != 0;
    if (npad > CH_TVS || nd > 64 || npad < 0 || nd < 0) return false;   // bug guard
    const double *dyn = B + CH_HDR;
    double *tv = B + CH_HDR + 4 * nd;
    // wave-uniform solve constants, kept in SGPRs (scalar loads of the global record measured
    // no faster: their lgkm waits merge with the LDS ones)
    auto U = [&](int k) {
        const double v = B[k];
        return __hiloint2double(__builtin_amdgcn_readfirstlane(__double2hiint(v)),
                                __builtin_amdgcn_readfirstlane(__double2loint(v)));
    };
    const double x0 = U(2), y0 = U(3), M0 = U(4), M1 = U(5), M2 = U(6), M3 = U(7), M4 = U(8);
    const double M5 = U(9), M6 = U(10), M7 = U(11), M8 = U(12), C0 = U(13), C1 = U(14);
    const double C2 = U(15), inv_det = U(16);
    // fold lanes: one per ordered sum (row of the term table: X1's three, then X2's three)
    const int fs = lane % 3, fc = lane >= 3 ? 1 : 0, frow = lane;
    const bool fl = lane < 6;
    constexpr int XL2 = CH_XL2;   // the lane holding X2's result
    double acc = 0.0;
    if (fl) acc = B[17 + frow];
    const bool has = lane < nd;
    int2 e = make_int2(0, -1);
    bool crit = false;
    double cf[3] = {0.0, 0.0, 0.0};
    if (has) {
        const double2 q0 = ((const double2 *)dyn)[2 * lane], q1 = ((const double2 *)dyn)[2 * lane + 1];
        const long long kk = __double_as_longlong(q0.x);
        crit = (kk & CH_CRIT) != 0;
        e = make_int2((int)(kk & 0xffff), (int)(kk >> 32));
        cf[0] = q0.y; cf[1] = q1.x; cf[2] = q1.y;
    }
    const int slot = e.y & (CH_R - 1);
    // the other parts' sources first: 8-byte granules (X1, X2) stored write-through by their
    // producers, read with agent-scope loads (no L1, no fence: the value is its own flag)
    const bool far = has && e.y < 0;
    bool done = !has || crit;
    if (__ballot(far)) {
        long sp = 0;
        const u64 *gv = (const u64 *)gval + 2 * (long)(-e.y - 1);
        for (;;) {
            if (far && !done) {
                const u64 bx = __hip_atomic_load(gv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const u64 by = __hip_atomic_load(gv + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (bx != CH_GSENT && by != CH_GSENT) {
                    const double vx = __longlong_as_double((long long)bx);
                    const double vy = __longlong_as_double((long long)by);
#pragma unroll
                    for (int s = 0; s < 6; ++s) tv[s * npad + e.x] = cf[s % 3] * (s < 3 ? vx : vy);
                    done = true;
                }
            }
            if (__ballot(far && !done) == 0 || (RMT_CH_ABL & 4)) break;
            if constexpr (PROF) {   // the far source still missing with the latest slot
                int g = far && !done ? -e.y - 1 : -1;
#pragma unroll
                for (int off = 32; off > 0; off >>= 1) g = max(g, __shfl_xor(g, off));
                tr_far = g;
            }
            if (++sp > CH_SPIN_LIMIT) return false;
            __builtin_amdgcn_s_sleep(1);
        }
        if constexpr (PROF)
            if (sp) tr_ready = __builtin_amdgcn_s_memrealtime();
    }
    // the critical source: its term position, slot, tag and coefficients (uniform)
    const u64 cm = __ballot(crit);
    const int cl = cm ? __builtin_ctzll(cm) : 0;
    const int kc = cm ? __builtin_amdgcn_readlane(e.x, cl) : npad;
    const int eyc = __builtin_amdgcn_readlane(e.y, cl);
    const int slc = eyc & (CH_R - 1);
    const double cc0 = rlf(cf[0], cl), cc1 = rlf(cf[1], cl), cc2 = rlf(cf[2], cl);
    const double cfc = fs == 0 ? cc0 : (fs == 1 ? cc1 : cc2);   // fold lane: w * a_s
    // pass 1: products of the other sources already published
    {
        const bool ready = !done && __hip_atomic_load(&tag[slot], __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_WORKGROUP) == e.y;
        asm volatile("" ::: "memory");
        if (ready) {
            const double2 v = val[slot];
#pragma unroll
            for (int s = 0; s < 6; ++s) tv[s * npad + e.x] = cf[s % 3] * (s < 3 ? v.x : v.y);
            done = true;
        }
    }
    // fold up to the first missing term (or kc), then wait for the other sources
    u64 pend = __ballot(!done);
    int kmiss = pend ? __builtin_amdgcn_readlane(e.x, __builtin_ctzll(pend)) : kc;
    if (kmiss > kc) kmiss = kc;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    if (fl) acc = ch_fold_span(acc, tv + frow * npad, 0, kmiss);
    CH_STAMP(3);
    if (pend) {
        long sp = 0;
        __builtin_amdgcn_s_setprio(0);
        for (;;) {
            if (!done && __hip_atomic_load(&tag[slot], __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_WORKGROUP) == e.y) {
                asm volatile("" ::: "memory");
                const double2 v = val[slot];
#pragma unroll
                for (int s = 0; s < 6; ++s) tv[s * npad + e.x] = cf[s % 3] * (s < 3 ? v.x : v.y);
                done = true;
            }
            if (__ballot(!done) == 0 || (RMT_CH_ABL & 4)) break;
            if (++sp > CH_SPIN_LIMIT) return false;
        }
        __builtin_amdgcn_s_setprio(3);
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
    if (fl) acc = ch_fold_span(acc, tv + frow * npad, kmiss, kc);
    if (cm) {
        // the terms after kc: their head chunk and the next two in registers before the
        // critical value arrives (pure VALU adds after it), the rest from LDS.  Rows are padded
        // with +0.0 to whole chunks (exact: a sum that starts at +0.0 is never -0.0).
        // (lanes 0-5 only: 64 lanes at a row stride would conflict on every LDS bank)
        const double *row = tv + frow * npad;
        const int h0 = (kc + 1) >> 3, hs = kc + 1 - 8 * h0, nch = npad >> 3;
        // (the profiled build keeps one chunk: its counters need the registers)
        constexpr int NRT = PROF ? 8 : 24;
        double rt[NRT];
        if (fl) {
            const double2 *r2 = (const double2 *)(row + 8 * h0);
#pragma unroll
            for (int k = 0; k < NRT / 2; ++k) {
                const double2 q = r2[k];
                rt[2 * k] = q.x; rt[2 * k + 1] = q.y;
            }
            // pinned here: the compiler would otherwise sink these reads past the poll loop
#pragma unroll
            for (int k = 0; k < NRT; ++k) asm volatile("" : "+v"(rt[k]));
        }
        double2 vc;
        long sp = 0;
        // the tag and the value read back to back in one LDS round trip (relaxed atomic
        // loads: a plain value load would be sunk out of the loop)
        const unsigned long long *vq = (const unsigned long long *)&val[slc];
        __builtin_amdgcn_s_setprio(RMT_CH_POLL_PRIO);   // polling the critical source
        for (;;) {
            const int tg = __hip_atomic_load(&tag[slc], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            asm volatile("" ::: "memory");             // the tag read is issued first
            __builtin_amdgcn_sched_barrier(0);
            vc.x = __longlong_as_double((long long)__hip_atomic_load(vq, __ATOMIC_RELAXED,
                                                                     __HIP_MEMORY_SCOPE_WORKGROUP));
            vc.y = __longlong_as_double((long long)__hip_atomic_load(vq + 1, __ATOMIC_RELAXED,
                                                                     __HIP_MEMORY_SCOPE_WORKGROUP));
            __builtin_amdgcn_sched_barrier(0);   // all three reads issued, then the tag test
            if (__builtin_amdgcn_readfirstlane(tg) == eyc || (RMT_CH_ABL & 4)) break;
            if (++sp > CH_SPIN_LIMIT) return false;
        }
        if constexpr (PROF) {
            if (sp) tr_crit = eyc;
            pr[7] += sp;
            CH_STAMP(2);
            tr_ready = __builtin_amdgcn_s_memrealtime();
        }
        __builtin_amdgcn_s_setprio(3);   // from the arrival through the publish
        if (fl) {
            acc += cfc * (fc == 0 ? vc.x : vc.y);
            do {   // (straight-line: rt indexed statically)
                if (RMT_CH_ABL & 1) break;   // timing ablation (wrong results): no tail
                if (h0 >= nch) break;   // kc was the last term
#pragma unroll
                for (int k = 0; k < 8; ++k)
                    if (k >= hs) acc += rt[k];
                if constexpr (NRT > 8) {
                    if (h0 + 1 >= nch) break;
                    acc += rt[8]; acc += rt[9]; acc += rt[10]; acc += rt[11];
                    acc += rt[12]; acc += rt[13]; acc += rt[14]; acc += rt[15];
                }
                if constexpr (NRT > 16) {
                    if (h0 + 2 >= nch) break;
                    acc += rt[16]; acc += rt[17]; acc += rt[18]; acc += rt[19];
                    acc += rt[20]; acc += rt[21]; acc += rt[22]; acc += rt[23];
                }
                acc = ch_fold(acc, row, h0 + NRT / 8, nch);
            } while (0);
        }
    }
    if constexpr (PROF) asm volatile("" : "+v"(acc));
    CH_STAMP(4);
    double bb1 = dpp_shl(acc, 1), bb2 = dpp_shl(acc, 2);
    if constexpr (PROF) asm volatile("" : "+v"(bb1), "+v"(bb2));
    CH_STAMP(8);
    if (lane == 0 || lane == 3) {
        const double b0 = acc, b1 = bb1, b2 = bb2;
        const double xs = (b0 * C0 - M1 * (b1 * M8 - M5 * b2) + M2 * (b1 * M7 - M4 * b2)) * inv_det;
        const double ys = (M0 * (b1 * M8 - M5 * b2) - b0 * C1 + M2 * (M3 * b2 - b1 * M6)) * inv_det;
        const double zs = (M0 * (M4 * b2 - b1 * M7) - M1 * (M3 * b2 - b1 * M6) + b0 * C2) * inv_det;
        // (ablation 2: no solve -- the identity map's value, still after acc)
        double o = (RMT_CH_ABL & 2) ? (lane == 0 ? x0 : y0) + 0.0 * acc : xs + ys * x0 + zs * y0;
        if constexpr (PROF) asm volatile("" : "+v"(o));
        CH_STAMP(9);
        ((double *)&val[x & (CH_R - 1)])[lane == 0 ? 0 : 1] = o;
        o_out = o;
    }
    asm volatile("" ::: "memory");
    if (lane == 0)
        __hip_atomic_store(&tag[x & (CH_R - 1)], x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (pub && (lane == 0 || lane == XL2))   // after the LDS hand-off: the local reader first
        __hip_atomic_store((u64 *)gval + 2L * gslot + (lane == 0 ? 0 : 1),
                           (u64)__double_as_longlong(o_out), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    if constexpr (PROF) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    CH_STAMP(10);
    __builtin_amdgcn_s_setprio(RMT_CH_WORK_PRIO);   // the next fit's pre-arrival work
    c_out = __double_as_longlong(B[0]);
    if constexpr (PROF) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    CH_STAMP(5);
    if constexpr (PROF) {
        if (trace && lane == 0) {
            const long long tp = __builtin_amdgcn_s_memrealtime();
            long long *t = trace + 6L * gslot;
            t[0] = tr_start; t[1] = tr_ready ? tr_ready : tr_start; t[2] = tp;
            t[3] = tr_crit >= 0 ? base + tr_crit : tr_far;
            t[4] = (threadIdx.x >> 6) | (blockIdx.x << 8); t[5] = c_out;
        }
    }
    return true;
}

template <bool PROF>
__global__ void __launch_bounds__(CH_W * 64) k_ex_chain(ChainArgs C, long long *gprof) {
    __shared__ double2 val[CH_R];
    __shared__ int tag[CH_R];
    __shared__ __attribute__((aligned(16))) double buf[CH_W][CH_BUFD];
    __shared__ int cur[CH_W];
    const int *ctl = C.ws.ctl;
    const char *arena = C.ws.arena;
    double *X1e = C.X1e, *X2e = C.X2e;
    for (int s = threadIdx.x; s < CH_R; s += blockDim.x) tag[s] = -1;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (threadIdx.x < CH_W) cur[threadIdx.x] = 0;
    __syncthreads();
    if (ctl[EXC_FALLBACK] || ctl[EXC_ABORT]) return;
    // this workgroup runs part blockIdx.x; x below is the ordinal within the part
    const int part = blockIdx.x, base = ch_base(ctl, part);
    const int total = ctl[EXC_NPART + part];
    double *B = buf[wv];
    // this wave's first accepted fit (k_ex_runs); every record names the wave's next one
    // (k_ex_relink)
    int x = ctl[EXC_WSTART + part * CH_W + wv];
    long long r0 = -1;
    while (x < total && (r0 = C.ws.rec_by_chain[C.ws.inv[base + x]]) < 0) x = C.ws.wnext[base + x];
    unsigned r = (unsigned)(r0 & 0xffffffffLL) | (unsigned)((r0 >> 32) << 25);
    double2 d0, d1, d2, d3, d4;
    if (x < total) CH_LOAD(r);
    int wm = 0;
    bool ok = true;
    long long pr[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, tl = 0;
    if constexpr (PROF) tl = __builtin_amdgcn_s_memtime();
    double o = 0.0;      // previous fit's value (lane 0: X1, lane 3: X2) and cell
    long c = -1;
    while (x < total) {
        __hip_atomic_store(&cur[wv], x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        CH_STAGE(r);
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        CH_STAMP(0);
        // the previous fit's stores go out BEFORE the prefetch, so that waiting for the
        // prefetched record next trip never waits on a younger store
        if (c >= 0 && (lane == 0 || lane == CH_XL2)) (lane == 0 ? X1e : X2e)[c] = o;
        // prefetch the next record of this wave into the registers just staged
        const long long nx = __double_as_longlong(B[23]);
        const int x2 = __builtin_amdgcn_readfirstlane((int)(nx >> 32));
        const unsigned r2 = (unsigned)__builtin_amdgcn_readfirstlane((int)(nx & 0xffffffff));
        if (x2 <= x) { ok = false; break; }   // bug guard: the wave's sequence must advance
        if (x2 < total) CH_LOAD(r2);
        CH_STAMP(6);
        const bool fit_ok = ch_fit<PROF>(x, lane, B, val, tag, cur, wm, o, c, pr, tl,
                                         C.ws.gval, base + x, C.trace, base);
        if (!fit_ok) { ok = false; break; }
        x = x2; r = r2;
    }
    if constexpr (PROF)
        if (lane == 0)
            for (int k = 0; k < 12; ++k) atomicAdd((unsigned long long *)&gprof[k], pr[k]);
    if (ok && c >= 0 && (lane == 0 || lane == CH_XL2)) (lane == 0 ? X1e : X2e)[c] = o;
    __hip_atomic_store(&cur[wv], 0x7fffffff, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (!ok && lane == 0) {   // the abort word names this part and the waiting fit (extrap.hpp)
        C.ws.ctl[EXC_ABORT] = 1;
        exa_report(C.status, exa_code(EXA_CHAIN, part, x));
    }
}
// ------------------------------------------------------------------ host side ------
// the chain's workgroups: column ranges x layer groups (rmt_ctx::ch_cols, ch_lgroups)
static int chain_parts(const rmt_ctx *ctx, int ML, int *ncol, int *nlg) {
    *ncol = std::min(CH_MAXP, std::max(1, ctx->opt.ch_cols));
    int g = ctx->opt.ch_lgroups > 0 ? ctx->opt.ch_lgroups : ML;
    *nlg = std::max(1, std::min({g, ML, CH_MAXP / *ncol}));
    return *ncol * *nlg;
}

bool extrap_chain_supported(int ny, int nx, int ML) {
    return ML >= 1 && ML <= EX_MAXL && ny >= 3 && nx >= 3;
}

// the chip-wide passes that turn the band into chain records (the chain kernel itself is
// extrap_chain_run, launched after the fallback sweep's launch so that the sweep -- an
// early exit unless a capacity limit tripped -- does not wait behind the chain)
int extrap_chain_prep(rmt_ctx *ctx, const ExWs &ws, const double *X1o, const double *X2o,
                      double dx, double dy, int ML) {
    const int ny = ctx->ny, nx = ctx->nx, W = (nx + 63) / 64;
    hipStream_t st = ctx->stream;
    const unsigned rows = grid1d(ny, 4);
    double r = 4 * std::sqrt(dx * dx + dy * dy);
    ExGeoArgs A{ws, X1o, X2o, ny, nx, W, 0, dx, dy, r * r, 0};
    const unsigned gblocks = (unsigned)std::min<long>(4096, std::max<long>(1, ws.maxt / 4));
    for (int L = 0; L < ML; ++L) {
        A.L = L;
        k_tg_rows<<<rows, 256, 0, st>>>(ws, ny, nx, W, L);
        k_tg_scan<<<1, 1024, 0, st>>>(ws, ny, L);
        k_tg_emit<<<rows, 256, 0, st>>>(ws, ny, nx, W, L);
        k_ex_geom<<<gblocks, 256, 0, st>>>(A);
        k_ex_fix<<<1, FIXW * 64, 0, st>>>(A);
        RMT_LAUNCHED();
    }
    int ncol, nlg;
    const int nparts = chain_parts(ctx, ML, &ncol, &nlg);
    k_ex_order<<<1, 1024, 0, st>>>(ws, ny, ML);
    k_ex_split<<<1, 1024, 0, st>>>(ws, nx, ML, ncol, nlg);
    const unsigned idb = grid1d(ws.maxt, 256);
    k_ex_chainidx<<<idb, 256, 0, st>>>(ws, ny, nx, ML, ws.status);
    k_ex_local<<<1, 1024, 0, st>>>(ws, ML);
    k_ex_runs<<<nparts, 1024, 0, st>>>(ws);
    k_ex_relink<<<std::min<unsigned>(grid1d(ws.maxt, 4), 2048), 256, 0, st>>>(ws, ML);
    RMT_LAUNCHED();
    return RMT_OK;
}

// the parallel mode's half of the prep: targets and final acceptance per layer, no records
int extrap_chain_prep_px(rmt_ctx *ctx, const ExWs &ws, double dx, double dy, int ML) {
    const int ny = ctx->ny, nx = ctx->nx, W = (nx + 63) / 64;
    hipStream_t st = ctx->stream;
    const unsigned rows = grid1d(ny, 4);
    double r = 4 * std::sqrt(dx * dx + dy * dy);
    ExGeoArgs A{ws, nullptr, nullptr, ny, nx, W, 0, dx, dy, r * r, 1};
    const unsigned gblocks = (unsigned)std::min<long>(4096, std::max<long>(1, ws.maxt / 4));
    for (int L = 0; L < ML; ++L) {
        A.L = L;
        k_tg_rows<<<rows, 256, 0, st>>>(ws, ny, nx, W, L);
        k_tg_scan<<<1, 1024, 0, st>>>(ws, ny, L);
        k_tg_emit<<<rows, 256, 0, st>>>(ws, ny, nx, W, L);
        k_ex_geom<<<gblocks, 256, 0, st>>>(A);
        k_ex_fix<<<1, FIXW * 64, 0, st>>>(A);
        RMT_LAUNCHED();
    }
    return RMT_OK;
}

// the value half of the records (after the map is advected; k_ex_vals)
int extrap_chain_values(rmt_ctx *ctx, const ExWs &ws, const double *X1o, const double *X2o,
                        double dx, double dy, int ML) {
    const int ny = ctx->ny, nx = ctx->nx, W = (nx + 63) / 64;
    const double r = 4 * std::sqrt(dx * dx + dy * dy);
    ExGeoArgs A{ws, X1o, X2o, ny, nx, W, 0, dx, dy, r * r, 0};
    const unsigned gblocks = (unsigned)std::min<long>(4096, std::max<long>(1, ws.maxt / 4));
    RMT_HIP(launch_done(ctx, k_ex_vals, dim3(gblocks), dim3(256), 0, ctx->stream,
                        ctx->ev_chain_vals ? ctx->ev_chain : nullptr, A, ML));
    return RMT_OK;
}

int extrap_chain_run(rmt_ctx *ctx, const ExWs &ws, const double *X1o, const double *X2o,
                     int ML) {
    hipStream_t st = ctx->stream;
    int ncol, nlg;
    const int nparts = chain_parts(ctx, ML, &ncol, &nlg);
    if (ctx->prof) RMT_HIP(hipEventRecord(ctx->ev[2], st));
    if (ctx->ev_chain && !ctx->ev_chain_vals) RMT_HIP(hipEventRecord(ctx->ev_chain, st));
    ChainArgs C{ws, (double *)X1o, (double *)X2o, ML, ws.status, nullptr};
    if (!ctx->opt.ex_profile) {
        k_ex_chain<false><<<nparts, CH_W * 64, 0, st>>>(C, nullptr);
        RMT_LAUNCHED();
    } else {
        // diagnostic: per-phase shader clocks summed over the chain waves
        long long *gp = nullptr, hp[12];
        RMT_HIP(hipMalloc(&gp, sizeof(hp)));
        RMT_HIP(hipMemsetAsync(gp, 0, sizeof(hp), st));
        hipEvent_t e0, e1;
        RMT_HIP(hipEventCreate(&e0)); RMT_HIP(hipEventCreate(&e1));
        // RMT_EX_TRACE=<path>: per-fit timestamps of the first profiled call, raw int64
        // (tools/chain_trace.py reconstructs the critical path)
        static const char *tpath = getenv("RMT_EX_TRACE");
        static bool traced = false;
        long long *dtr = nullptr;
        if (tpath && !traced) {
            RMT_HIP(hipMalloc(&dtr, 6 * sizeof(long long) * ws.maxt));
            RMT_HIP(hipMemsetAsync(dtr, 0, 6 * sizeof(long long) * ws.maxt, st));
            C.trace = dtr;
        }
        RMT_HIP(hipEventRecord(e0, st));
        k_ex_chain<true><<<nparts, CH_W * 64, 0, st>>>(C, gp);
        RMT_LAUNCHED();
        RMT_HIP(hipEventRecord(e1, st));
        RMT_HIP(hipMemcpyAsync(hp, gp, sizeof(hp), hipMemcpyDeviceToHost, st));
        int hs[2];
        RMT_HIP(hipMemcpyAsync(hs, ws.status, sizeof(hs), hipMemcpyDeviceToHost, st));
        RMT_HIP(hipStreamSynchronize(st));
        float ms = 0;
        RMT_HIP(hipEventElapsedTime(&ms, e0, e1));
        fprintf(stderr, "[chain-prof] %.3f ms fits=%d | stage %.3g throttle %.3g wait %.3g "
                "products %.3g fold %.3g solve+publish %.3g store+prefetch %.3g (Mclk, all "
                "waves) polls %lld | post split (clk/fit): fold %.0f dpp %.0f solve %.0f "
                "publish %.0f\n", ms, hs[0], hp[0] / 1e6, hp[1] / 1e6, hp[2] / 1e6,
                hp[3] / 1e6, hp[4] / 1e6, hp[5] / 1e6, hp[6] / 1e6, hp[7],
                (double)hp[4] / std::max(1, hs[0]), (double)hp[8] / std::max(1, hs[0]),
                (double)hp[9] / std::max(1, hs[0]), (double)hp[10] / std::max(1, hs[0]));
        if (dtr) {
            std::vector<long long> h(6 * ws.maxt);
            int tot = 0;
            RMT_HIP(hipMemcpy(&tot, ws.ctl + EXC_BASE + ML, sizeof(int), hipMemcpyDeviceToHost));
            RMT_HIP(hipMemcpy(h.data(), dtr, 6 * sizeof(long long) * tot, hipMemcpyDeviceToHost));
            FILE *f = fopen(tpath, "wb");
            if (f) { fwrite(h.data(), sizeof(long long), 6 * (size_t)tot, f); fclose(f); }
            (void)hipFree(dtr);
            traced = true;
        }
        (void)hipEventDestroy(e0); (void)hipEventDestroy(e1); (void)hipFree(gp);
    }
    if (ctx->prof) RMT_HIP(hipEventRecord(ctx->ev[3], st));
    return RMT_OK;
}

}  // namespace rmt
