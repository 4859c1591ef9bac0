// extrap_par.hip -- functions.py:48-163 extrapolate_reference_map, parallel mode (opt-in:
// rmt_extrap_set_parallel / RMT_EXTRAP_PARALLEL=1).  NOT bit-exact: see below.
//
// The reference fits a layer's targets in raster order and marks each known at once, so a
// fit reads the fits before it (a Gauss-Seidel chain ~3000 fits deep at N = 4096: the exact
// path, extrap_chain.hip, runs it in ~3 ms on one CU).  Every fit is linear in the map
// values it reads, with coefficients fixed by the known set alone: in integer offsets
// (di, dj) from the target, the weighted least-squares plane's value at the target is
//     x_t = sum_s beta_ts X_s,   beta_ts = w_s (y0 + y1 di_s + y2 dj_s),
// (y0, y1, y2) = first column of the inverse of the centred normal matrix sum w [1 di dj]^T
// [1 di dj] (w = exp(-d^2/r^2) exactly as the reference, exp_glibc.h).  The plane's value at
// the target does not depend on the coordinate origin, so this is the reference's fit in
// exact arithmetic; the reference evaluates it by Cramer's rule on absolute coordinates
// (utils.py:134-166) with det ~ 1e-10, which loses ~6 digits at N = 4096 (SURVEY App. A.2:
// 1.9e-6 from the exact plane).  This mode therefore differs from the reference by the
// reference's own rounding of each fit -- the same order as what 1-ulp noise in the weights
// does to it (tools/noise_floor.py, profiles/r03/noise/); acceptance (count >= 3,
// det(Aw) > 1e-10 in the reference's arithmetic), the weights, the known sets and the
// raster-order semantics are the reference's exactly (extrap_chain.hip's passes).
//
// A layer's fits then form a sparse unit-lower-triangular system x = c + B x (c: the static
// sources -- solid cells and earlier layers' fits; B: same-layer fits, raster order).  It is
// solved by segments of PX_K consecutive fits:
//   geometry (value-independent; beside the previous step's projection in the fused step):
//     k_px_beta   one wave per fit: sources and beta (window order, static first)
//     k_px_seg    one wave per segment: its frontier F (earlier same-layer fits it reads,
//                 ~13 at N = 4096, <= PX_F or the segment is solved serially), and its
//                 affine response x_seg = M f_F + N c_seg by forward substitution
//     k_px_pack   one wave per segment: the rows a later frontier reads ("live", ~13) and
//                 their M rows, packed into one contiguous block for the sequential pass
//   values, per layer (critical path):
//     k_px_c      one wave per fit: c_t = sum over static sources beta X
//     k_px_d      one wave per segment: d = N c (and d of the live rows into the block)
//     k_px_comb   one workgroup, sequential over the layer's segments: wave 0 computes the
//                 live rows, x = d + M f (~13 x 13 FMAs per segment) from an LDS value ring;
//                 15 producer waves stream the next segments' blocks into LDS slots ahead
//                 of it (intra-workgroup flags), so its ~0.2 us per segment is not HBM latency
//     k_px_out    one wave per segment: every fit, x = d + M f, written to the map
// tools/pex_proto.py restates the algorithm in numpy (segment solve = serial forward
// substitution to 7e-16 at N = 4096; frontier sizes); oracle/rmt_oracle.c mode 2 computes the
// same fits serially (the GPU agrees to rounding: tests/test_gpu_extrap_par.py).
#include "extrap.hpp"
#include "exp_glibc.h"
#include <cstdlib>

namespace rmt {

static int g_par = -1;   // -1: from RMT_EXTRAP_PARALLEL

bool extrap_par_enabled() {
    if (g_par < 0) g_par = getenv("RMT_EXTRAP_PARALLEL") && atoi(getenv("RMT_EXTRAP_PARALLEL"));
    return g_par > 0;
}

__device__ __forceinline__ double px_wsum(double v) {   // butterfly: every lane gets the sum
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
__device__ __forceinline__ double px_rl(double v, int l) {
    const long long b = __double_as_longlong(v);
    const unsigned lo = __builtin_amdgcn_readlane((unsigned)b, l);
    const unsigned hi = __builtin_amdgcn_readlane((unsigned)(b >> 32), l);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
__device__ __forceinline__ int px_layer_of(const int *ctl, int ML, int id) {
    int L = ML - 1;
    while (L > 0 && id < ctl[EXC_BASE + L]) --L;
    return L;
}
// segments of layer L: first global index s0, count ns
__device__ __forceinline__ void px_segs(const int *ctl, int L, int &s0, int &ns) {
    s0 = 0;
    for (int q = 0; q < L; ++q) s0 += (ctl[EXC_BASE + q + 1] - ctl[EXC_BASE + q] + PX_K - 1) / PX_K;
    ns = (ctl[EXC_BASE + L + 1] - ctl[EXC_BASE + L] + PX_K - 1) / PX_K;
}

// ------------------------------------------------------------------ geometry -------
// One wave per target id (all layers): the window of ex_geom (extrap_chain.hip) with the
// final acceptance (ACC after k_ex_fix), the centred fit's beta per included cell.
__global__ void __launch_bounds__(256) k_px_beta(ExWs ws, int ny, int nx, int W, int ML,
                                                 double dx, double dy, double r2) {
    __shared__ u64 tab[256];
    for (int s = threadIdx.x; s < 256; s += blockDim.x) tab[s] = kExpTab[s];
    __syncthreads();
    if (ws.ctl[EXC_FALLBACK]) return;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int total = ws.ctl[EXC_BASE + ML];
    const long plane = ws.plane;
    for (int id = blockIdx.x * 4 + wv; id < total; id += gridDim.x * 4) {
        const int L = px_layer_of(ws.ctl, ML, id);
        const long c = ws.tcell[id];
        const int j = (int)(c / nx), i = (int)(c % nx);
        const u64 *ACC = ws.ACC + (long)L * plane;
        const bool accepted = (ACC[(long)j * W + (i >> 6)] >> (i & 63)) & 1;
        if (!accepted) {
            if (lane == 0) { ws.pns[id] = 0; ws.pnd[id] = 0; ws.pval[id] = make_double2(0.0, 0.0); }
            continue;
        }
        const u64 *Kst = L == 0 ? ws.kbits : ws.KN + (long)(L - 1) * plane;
        const double x0 = dx * i, y0 = dy * j;
        bool inc[2], same[2];
        double w[2], di[2], dj[2];
        int key[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int q = lane + 64 * h, jj = j - 4 + q / 9, ii = i - 4 + q % 9;
            inc[h] = false; same[h] = false; w[h] = 0.0; key[h] = 0;
            di[h] = (double)(ii - i); dj[h] = (double)(jj - j);
            if (q < 81 && jj >= 0 && jj < ny && ii >= 0 && ii < nx) {
                const double xi = dx * ii, yi = dy * jj;
                const double ax = xi - x0, ay = yi - y0, d2 = ax * ax + ay * ay;
                if (d2 <= r2) {
                    const long o = (long)jj * W + (ii >> 6);
                    const u64 bit = 1ull << (ii & 63);
                    const bool ks = (Kst[o] & bit) != 0;
                    bool sl = false;
                    if (!ks && (jj < j || (jj == j && ii < i))) sl = (ACC[o] & bit) != 0;
                    inc[h] = ks || sl;
                    if (inc[h]) {
                        w[h] = exp_glibc_tab(-d2 / r2, tab);   // the reference's weight
                        if (ws.kbits[o] & bit) {
                            key[h] = (int)((long)jj * nx + ii);   // solid: the map value
                        } else {
                            int Ls = L;
                            if (!sl)
                                for (Ls = 0; Ls < L; ++Ls)
                                    if (ws.ACC[(long)Ls * plane + o] & bit) break;
                            const int sid = ws.ctl[EXC_BASE + Ls] +
                                            ws.rowoff[(long)Ls * (ny + 1) + jj] +
                                            ws.wordoff[(long)Ls * plane + o] +
                                            __popcll(ws.T[(long)Ls * plane + o] & (bit - 1));
                            key[h] = -(sid + 1);
                            same[h] = sl;
                        }
                    }
                }
            }
        }
        // centred normal matrix (fixed butterfly order: deterministic)
        double s0 = 0, sx = 0, sy = 0, sxx = 0, sxy = 0, syy = 0;
#pragma unroll
        for (int h = 0; h < 2; ++h)
            if (inc[h]) {
                const double a = di[h], b = dj[h], ww = w[h];
                s0 += ww; sx += ww * a; sy += ww * b;
                sxx += ww * a * a; sxy += ww * a * b; syy += ww * b * b;
            }
        s0 = px_wsum(s0); sx = px_wsum(sx); sy = px_wsum(sy);
        sxx = px_wsum(sxx); sxy = px_wsum(sxy); syy = px_wsum(syy);
        const double c00 = sxx * syy - sxy * sxy, c01 = sx * syy - sxy * sy,
                     c02 = sx * sxy - sxx * sy;
        const double dc = s0 * c00 - sx * c01 + sy * c02;
        const double y0c = c00 / dc, y1c = -c01 / dc, y2c = c02 / dc;
        // compact in window order: static sources first, then same-layer fits
        const u64 lt = (1ull << lane) - 1;
        const u64 st0 = __ballot(inc[0] && !same[0]), st1 = __ballot(inc[1] && !same[1] && lane < 17);
        const u64 dy0 = __ballot(inc[0] && same[0]), dy1 = __ballot(inc[1] && same[1] && lane < 17);
        const int ns = __popcll(st0) + __popcll(st1), nd = __popcll(dy0) + __popcll(dy1);
        int *kb = ws.pkey + (long)id * PX_S;
        double *bb = ws.pbeta + (long)id * PX_S;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            if (!inc[h] || (h && lane >= 17)) continue;
            int k;
            if (!same[h]) k = h ? __popcll(st0) + __popcll(st1 & lt) : __popcll(st0 & lt);
            else k = ns + (h ? __popcll(dy0) + __popcll(dy1 & lt) : __popcll(dy0 & lt));
            kb[k] = key[h];
            bb[k] = w[h] * (y0c + y1c * di[h] + y2c * dj[h]);
        }
        if (lane == 0) {
            ws.pns[id] = ns; ws.pnd[id] = nd;
            atomicAdd(ws.status, 1);   // fitted cells (rmt's dev_status[0])
        }
    }
}

// hash set of frontier ids in LDS (512 slots, open addressing)
constexpr int PX_HT = 512;
__device__ __forceinline__ unsigned px_h(int id) { return ((unsigned)id * 2654435761u) >> 23; }

// One wave per segment (all layers): frontier, then the forward substitution of the
// segment's rows over the columns [frontier | segment fits] (lanes = columns):
//   row_r = e_r (N part) + sum over same-layer sources s of fit lo + r, window order:
//           beta * (s in F ? e_F(s) : row_(s - lo))
struct PxSegLds {
    int tab[PX_HT], pos[PX_HT];
    int F[PX_F];
    double M[PX_K][PX_F + 1];   // +1: the transposed write-out reads columns
    double N[PX_K][PX_K + 1];
};
__global__ void __launch_bounds__(64) k_px_seg(ExWs ws, int ML) {
    __shared__ PxSegLds S;
    if (ws.ctl[EXC_FALLBACK]) return;
    const int g = blockIdx.x, lane = threadIdx.x;
    int L = -1, s0 = 0, ns = 0;
    for (int q = 0; q < ML; ++q) {
        px_segs(ws.ctl, q, s0, ns);
        if (g >= s0 && g < s0 + ns) { L = q; break; }
    }
    if (L < 0) return;
    const int b0 = ws.ctl[EXC_BASE + L], b1 = ws.ctl[EXC_BASE + L + 1];
    const int lo = b0 + (g - s0) * PX_K, hi = min(b1, lo + PX_K), n = hi - lo;
    for (int k = lane; k < PX_HT; k += 64) S.tab[k] = -1;
    __syncthreads();
    // 1. frontier: same-layer sources before lo (lane = row: the rows' loads in parallel)
    if (lane < n) {
        const int t = lo + lane, nst = ws.pns[t], nd = ws.pnd[t];
        const int *kb = ws.pkey + (long)t * PX_S + nst;
        for (int k = 0; k < nd; ++k) {
            const int s = -kb[k] - 1;
            if (s < lo) {
                unsigned h = px_h(s) & (PX_HT - 1);
                int probe = 0;
                for (; probe < PX_HT; ++probe, h = (h + 1) & (PX_HT - 1)) {
                    const int old = atomicCAS(&S.tab[h], -1, s);
                    if (old == -1 || old == s) break;
                }
                // table full (never at the configs' sizes): the exact sweep takes over
                if (probe == PX_HT) atomicExch(ws.ctl + EXC_FALLBACK, 1);
            }
        }
    }
    __syncthreads();
    int cnt = 0;
    for (int k = 8 * lane; k < 8 * lane + 8; ++k) cnt += S.tab[k] >= 0;
    int inc = cnt;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int v = __shfl_up(inc, d);
        if (lane >= d) inc += v;
    }
    const int nF = __shfl(inc, 63);
    int *hdr = ws.shdr + (long)g * PX_H;
    const bool serial = nF > PX_F;
    if (lane == 0) {
        hdr[0] = lo; hdr[1] = hi; hdr[2] = L; hdr[3] = serial ? 0 : nF; hdr[4] = serial;
    }
    // every frontier fit is computed by k_px_comb before this segment is reached
    for (int k = lane; k < PX_HT; k += 64)
        if (S.tab[k] >= 0) ws.live[S.tab[k]] = 1;
    if (serial) return;   // k_px_comb solves this segment fit by fit
    {
        int p = inc - cnt;
        for (int k = 8 * lane; k < 8 * lane + 8; ++k)
            if (S.tab[k] >= 0) S.F[p++] = S.tab[k];
    }
    __syncthreads();
    // sort F ascending (rank = number of smaller ids), record each id's column
    const int v = lane < nF ? S.F[lane] : 0x7fffffff;
    int rank = 0;
    for (int q = 0; q < nF; ++q) rank += __shfl(v, q) < v;
    __syncthreads();
    if (lane < nF) {
        S.F[rank] = v;
        ws.sF[(long)g * PX_F + rank] = v;
        unsigned h = px_h(v) & (PX_HT - 1);
        while (S.tab[h] != v) h = (h + 1) & (PX_HT - 1);
        S.pos[h] = rank;
    }
    __syncthreads();
    // 2. forward substitution, one row per fit (the next row's sources loaded ahead)
    int nxt_nd = 0, nxt_key = 0;
    double nxt_beta = 0.0;
    auto load_row = [&](int r) {
        const int t = lo + r, nst = ws.pns[t];
        nxt_nd = ws.pnd[t];
        const long kb = (long)t * PX_S + nst;
        nxt_key = lane < nxt_nd ? ws.pkey[kb + lane] : 0;
        nxt_beta = lane < nxt_nd ? ws.pbeta[kb + lane] : 0.0;
    };
    if (n > 0) load_row(0);
    for (int r = 0; r < n; ++r) {
        const int nd = nxt_nd, mykey = nxt_key;
        const double mybeta = nxt_beta;
        if (r + 1 < n) load_row(r + 1);
        double m = 0.0, nn = lane == r ? 1.0 : 0.0;
        for (int k = 0; k < nd; ++k) {
            const int s = -__builtin_amdgcn_readlane(mykey, k) - 1;
            const double b = px_rl(mybeta, k);
            if (s < lo) {
                unsigned h = px_h(s) & (PX_HT - 1);
                while (S.tab[h] != s) h = (h + 1) & (PX_HT - 1);
                if (lane == S.pos[h]) m += b;
            } else {
                const int rs = s - lo;
                m += b * S.M[rs][lane];
                nn += b * S.N[rs][lane];
            }
        }
        S.M[r][lane] = m;
        S.N[r][lane] = nn;
        __syncthreads();
    }
    // 3. write M^T [c][r] and N^T [r'][r] (lane = r: coalesced reads in the value passes)
    double *MT = ws.sMT + (long)g * PX_F * PX_K, *NT = ws.sNT + (long)g * PX_K * PX_K;
    for (int c = 0; c < nF; ++c) MT[c * PX_K + lane] = lane < n ? S.M[lane][c] : 0.0;
    for (int q = 0; q < n; ++q) NT[q * PX_K + lane] = lane < n ? S.N[lane][q] : 0.0;
}

// packed block of segment g (doubles): [0] nF, [1] nL, [2] kind (0 packed, 1 serial, 2 too
// large: k_px_comb reads M and d from their own arrays), [3] lo, [4] n, [8, 72) frontier ids,
// [72, 136) live rows, [136, 264) d of the live rows (k_px_d), [264, PX_PB) M of the live
// rows at a fixed stride: M[r_k][c] at 264 + c PXB_S + k (nF <= PXB_C, nL <= PXB_S; larger
// segments are kind 2).  Fixed addresses let k_px_comb read a whole block in one LDS round
// trip, before its header is known.
constexpr int PXB_F = 8, PXB_R = 72, PXB_D = 136, PXB_M = 264, PXB_S = 20, PXB_C = 24;
static_assert(PXB_M + PXB_C * PXB_S <= PX_PB, "packed block");
__global__ void __launch_bounds__(64) k_px_pack(ExWs ws, int ML) {
    if (ws.ctl[EXC_FALLBACK]) return;
    const int g = blockIdx.x, lane = threadIdx.x;
    int L = -1, s0 = 0, ns = 0;
    for (int q = 0; q < ML; ++q) {
        px_segs(ws.ctl, q, s0, ns);
        if (g >= s0 && g < s0 + ns) { L = q; break; }
    }
    if (L < 0) return;
    const int *hdr = ws.shdr + (long)g * PX_H;
    const int lo = hdr[0], n = hdr[1] - lo, nF = hdr[3], serial = hdr[4];
    double *B = ws.spk + (long)g * PX_PB;
    const bool lv = !serial && lane < n && ws.live[lo + lane];
    const u64 lm = __ballot(lv);
    const int nL = __popcll(lm);
    const int kind = serial ? 1 : (nF > PXB_C || nL > PXB_S ? 2 : 0);
    if (lane == 0) { B[0] = nF; B[1] = nL; B[2] = kind; B[3] = lo; B[4] = n; }
    if (serial) return;
    if (lane < nF) B[PXB_F + lane] = ws.sF[(long)g * PX_F + lane];
    const int k = __popcll(lm & ((1ull << lane) - 1));
    if (lv) B[PXB_R + k] = lane;
    if (kind != 0) return;
    const double *MT = ws.sMT + (long)g * PX_F * PX_K;
    for (int c = 0; c < nF; ++c)
        if (lv) B[PXB_M + c * PXB_S + k] = MT[c * PX_K + lane];
}

// ------------------------------------------------------------------ values ---------
// c_t = sum over the static sources (solid: the advected map; earlier layers: their fits)
// of beta X, one wave per fit of layer L (butterfly sum)
__global__ void __launch_bounds__(256) k_px_c(ExWs ws, int L, const double *__restrict__ X1,
                                              const double *__restrict__ X2) {
    if (ws.ctl[EXC_FALLBACK]) return;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int b0 = ws.ctl[EXC_BASE + L], b1 = ws.ctl[EXC_BASE + L + 1];
    for (int id = b0 + blockIdx.x * 4 + wv; id < b1; id += gridDim.x * 4) {
        const int nst = ws.pns[id];
        double a1 = 0.0, a2 = 0.0;
        for (int k = lane; k < nst; k += 64) {
            const int key = ws.pkey[(long)id * PX_S + k];
            const double b = ws.pbeta[(long)id * PX_S + k];
            double v1, v2;
            if (key >= 0) { v1 = X1[key]; v2 = X2[key]; }
            else { const double2 p = ws.pval[-key - 1]; v1 = p.x; v2 = p.y; }
            a1 += b * v1; a2 += b * v2;
        }
        a1 = px_wsum(a1); a2 = px_wsum(a2);
        if (lane == 0) ws.pc[id] = make_double2(a1, a2);
    }
}

// d = N c per segment of layer L: lane = row, the 64 columns split over 4 waves (16 each,
// combined in wave order), the live rows' d also into the packed block
__global__ void __launch_bounds__(256) k_px_d(ExWs ws, int L) {
    __shared__ double part[4][2][64];
    if (ws.ctl[EXC_FALLBACK]) return;
    int s0, ns;
    px_segs(ws.ctl, L, s0, ns);
    if ((int)blockIdx.x >= ns) return;
    const int g = s0 + blockIdx.x, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int *hdr = ws.shdr + (long)g * PX_H;
    if (hdr[4]) return;
    const int lo = hdr[0], n = hdr[1] - lo;
    const double *NT = ws.sNT + (long)g * PX_K * PX_K;
    double nq[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int q = wv * 16 + k;
        nq[k] = q < n ? NT[q * PX_K + lane] : 0.0;
    }
    const double2 cr = lane < n ? ws.pc[lo + lane] : make_double2(0.0, 0.0);
    double d1 = 0.0, d2 = 0.0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int q = wv * 16 + k;
        d1 += nq[k] * px_rl(cr.x, q);
        d2 += nq[k] * px_rl(cr.y, q);
    }
    part[wv][0][lane] = d1; part[wv][1][lane] = d2;
    __syncthreads();
    if (wv) return;
    d1 = ((part[0][0][lane] + part[1][0][lane]) + part[2][0][lane]) + part[3][0][lane];
    d2 = ((part[0][1][lane] + part[1][1][lane]) + part[2][1][lane]) + part[3][1][lane];
    if (lane < n) ws.sd[(long)g * PX_K + lane] = make_double2(d1, d2);
    const bool lv = lane < n && ws.live[lo + lane];
    const u64 lm = __ballot(lv);
    if (lv) {
        double *B = ws.spk + (long)g * PX_PB + PXB_D;
        const int k = __popcll(lm & ((1ull << lane) - 1));
        B[2 * k] = d1; B[2 * k + 1] = d2;
    }
}

// x = d + M f for one row (lane): the same operation order in k_px_comb and k_px_out
__device__ __forceinline__ double2 px_row(const double *__restrict__ MT, int nF, double2 d,
                                          double f1, double f2, int lane) {
    double x1 = d.x, x2 = d.y;
    for (int c = 0; c < nF; ++c) {
        const double m = MT[c * PX_K + lane];
        x1 += m * px_rl(f1, c);
        x2 += m * px_rl(f2, c);
    }
    return make_double2(x1, x2);
}

// The layer's segments in order, one workgroup: wave 0 (the consumer) computes each
// segment's live rows from an LDS value ring by fit id; waves 1..PX_NP (producers) copy the
// segments' packed blocks into PX_NS LDS slots ahead of it.  A slot is handed over by LDS flags
// (a wave's LDS operations complete in order, so the flag written after the data orders it);
// all waves of a workgroup are resident, so the spins terminate; a bug guard caps them and
// reports an abort (dev_status[1]).  A frontier id more than PX_RING behind its segment is
// read through L2 after a fence (the consumer wrote it to pval).
constexpr int PX_RING = 4096, PX_NS = 10, PX_NP = 15;
constexpr int PX_FR = 24;   // frontier columns the consumer holds in registers
constexpr size_t PX_COMB_LDS = PX_RING * 16 + (size_t)PX_NS * PX_PB * 8 + 2 * PX_NS * 4;
__device__ __forceinline__ double2 px_far(const double2 *p) {
    const double *q = (const double *)p;
    return make_double2(__hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                        __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__global__ void __launch_bounds__(64 * (PX_NP + 1)) k_px_comb(ExWs ws, int L,
                                                             double *__restrict__ X1,
                                                             double *__restrict__ X2) {
    extern __shared__ double px_lds[];
    double2 *ring = (double2 *)px_lds;
    double *slots = px_lds + 2 * PX_RING;
    volatile int *ready = (volatile int *)(slots + (size_t)PX_NS * PX_PB);
    volatile int *freeg = ready + PX_NS;
    if (ws.ctl[EXC_FALLBACK]) return;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    int s0, ns;
    px_segs(ws.ctl, L, s0, ns);
    if (threadIdx.x < PX_NS) { ready[threadIdx.x] = -1; freeg[threadIdx.x] = threadIdx.x; }
    __syncthreads();
    constexpr long SPIN = 1L << 26;
    if (wv > 0) {   // producer
        for (int gi = wv - 1; gi < ns; gi += PX_NP) {
            const int slot = gi % PX_NS;
            long spin = 0;
            while (freeg[slot] != gi) {
                __builtin_amdgcn_s_sleep(1);
                if (++spin > SPIN) { if (lane == 0) exa_report(ws.status, exa_code(EXA_PAR, 0, 0)); return; }
            }
            const double *src = ws.spk + (long)(s0 + gi) * PX_PB;
            double v[PX_PB / 64];
#pragma unroll
            for (int q = 0; q < PX_PB / 64; ++q) v[q] = src[q * 64 + lane];
            double *dst = slots + (size_t)slot * PX_PB;
#pragma unroll
            for (int q = 0; q < PX_PB / 64; ++q) dst[q * 64 + lane] = v[q];
            if (lane == 0) ready[slot] = gi;
        }
        return;
    }
    static_assert(PXB_C == PX_FR, "the consumer holds a packed block's M in registers");
    const int ml = lane < PXB_S ? lane : 0;
    for (int gi = 0; gi < ns; ++gi) {   // consumer (wave 0)
        const int slot = gi % PX_NS, g = s0 + gi;
        const double *B = slots + (size_t)slot * PX_PB;
        // the ready flag, then the whole block at fixed addresses, in one LDS round trip (a
        // wave's LDS operations execute in order: if the flag read sees gi, the reads after it
        // see the producer's block); read again after a wait if the producer was not done
        int rd;
        double h0, h1, h2, h3, h4, sd, rdd;
        double2 xd;
        double m[PX_FR];
        auto read_block = [&]() {
            rd = ready[slot];
            asm volatile("" ::: "memory");
            h0 = B[0]; h1 = B[1]; h2 = B[2]; h3 = B[3]; h4 = B[4];
            sd = B[PXB_F + lane]; rdd = B[PXB_R + lane];
            xd = make_double2(B[PXB_D + 2 * lane], B[PXB_D + 2 * lane + 1]);
#pragma unroll
            for (int c = 0; c < PX_FR; ++c) m[c] = B[PXB_M + c * PXB_S + ml];
        };
        read_block();
        if (rd != gi) {
            long spin = 0;
            while (ready[slot] != gi)
                if (++spin > SPIN) { if (lane == 0) exa_report(ws.status, exa_code(EXA_PAR, 0, 0)); return; }
            read_block();
        }
        const int nF = (int)h0, nL = (int)h1, kind = (int)h2, lo = (int)h3, n = (int)h4;
        if (kind == 1) {
            // serial segment, fit by fit: x_t = c_t + sum over same-layer sources beta x_s
            for (int r = 0; r < n; ++r) {
                const int t = lo + r, nst = ws.pns[t], nd = ws.pnd[t];
                int sr = 0;
                double b = 0.0, a1 = 0.0, a2 = 0.0;
                if (lane < nd) {
                    sr = -ws.pkey[(long)t * PX_S + nst + lane] - 1;
                    b = ws.pbeta[(long)t * PX_S + nst + lane];
                }
                const bool far = lane < nd && t - sr > PX_RING;
                if (__ballot(far)) __threadfence();
                if (lane < nd) {
                    const double2 v = far ? px_far(&ws.pval[sr]) : ring[sr & (PX_RING - 1)];
                    a1 = b * v.x; a2 = b * v.y;
                }
                a1 = px_wsum(a1); a2 = px_wsum(a2);
                const double2 c = ws.pc[t];
                const double2 x = make_double2(c.x + a1, c.y + a2);
                if (lane == 0 && nst + nd > 0) {
                    ring[t & (PX_RING - 1)] = x;
                    ws.pval[t] = x;
                    const long cell = ws.tcell[t];
                    X1[cell] = x.x; X2[cell] = x.y;
                }
            }
        } else if (nL > 0) {
            // the frontier's values: the one read that waits on earlier segments
            const int sf = lane < nF ? (int)sd : lo;
            const int r = lane < nL ? (int)rdd : 0;
            double f1 = 0.0, f2 = 0.0;
            {
                const bool far = lane < nF && lo - sf > PX_RING;
                if (__ballot(far)) __threadfence();
                if (lane < nF) {
                    const double2 v = far ? px_far(&ws.pval[sf]) : ring[sf & (PX_RING - 1)];
                    f1 = v.x; f2 = v.y;
                }
            }
            double2 x;
            if (kind == 0) {   // the FMAs back to back in px_row's order
                x = lane < nL ? xd : make_double2(0.0, 0.0);
#pragma unroll
                for (int c = 0; c < PX_FR; ++c) {
                    if (c < nF) {
                        const double mc = lane < nL ? m[c] : 0.0;
                        x.x += mc * px_rl(f1, c);
                        x.y += mc * px_rl(f2, c);
                    }
                }
            } else {   // block too small for this segment's M: its own arrays (same order)
                x = px_row(ws.sMT + (long)g * PX_F * PX_K, nF, ws.sd[(long)g * PX_K + r], f1, f2,
                           r);
            }
            if (lane < nL) {
                ring[(lo + r) & (PX_RING - 1)] = x;
                ws.pval[lo + r] = x;
            }
        }
        // every read of the slot is done: hand it back (LDS operations stay in order)
        if (lane == 0) freeg[slot] = gi + PX_NS;
    }
}

// every fit of the (non-serial) segments of layer L: x = d + M f, into the map
__global__ void __launch_bounds__(64) k_px_out(ExWs ws, int L, double *__restrict__ X1,
                                               double *__restrict__ X2) {
    if (ws.ctl[EXC_FALLBACK]) return;
    int s0, ns;
    px_segs(ws.ctl, L, s0, ns);
    if ((int)blockIdx.x >= ns) return;
    const int g = s0 + blockIdx.x, lane = threadIdx.x;
    const int *hdr = ws.shdr + (long)g * PX_H;
    if (hdr[4]) return;
    const int lo = hdr[0], n = hdr[1] - lo, nF = hdr[3];
    double f1 = 0.0, f2 = 0.0;
    if (lane < nF) {
        const double2 v = ws.pval[ws.sF[(long)g * PX_F + lane]];
        f1 = v.x; f2 = v.y;
    }
    const double2 d = lane < n ? ws.sd[(long)g * PX_K + lane] : make_double2(0.0, 0.0);
    const double2 x = px_row(ws.sMT + (long)g * PX_F * PX_K, nF, d, f1, f2, lane);
    if (lane < n && ws.pns[lo + lane] + ws.pnd[lo + lane] > 0) {
        ws.pval[lo + lane] = x;
        const long cell = ws.tcell[lo + lane];
        X1[cell] = x.x; X2[cell] = x.y;
    }
}

// ------------------------------------------------------------------ host side ------
int extrap_par_geometry(rmt_ctx *ctx, const ExWs &ws, double dx, double dy, int ML) {
    const int ny = ctx->ny, nx = ctx->nx, W = (nx + 63) / 64;
    hipStream_t st = ctx->stream;
    const double r = 4 * std::sqrt(dx * dx + dy * dy);
    RMT_HIP(hipMemsetAsync(ws.live, 0, ws.maxt, st));
    const unsigned gb = (unsigned)std::min<long>(4096, std::max<long>(1, ws.maxt / 4));
    k_px_beta<<<gb, 256, 0, st>>>(ws, ny, nx, W, ML, dx, dy, r * r);
    k_px_seg<<<(unsigned)ws.maxseg, 64, 0, st>>>(ws, ML);
    k_px_pack<<<(unsigned)ws.maxseg, 64, 0, st>>>(ws, ML);
    RMT_LAUNCHED();
    return RMT_OK;
}

int extrap_par_values(rmt_ctx *ctx, const ExWs &ws, double *X1o, double *X2o, int ML) {
    hipStream_t st = ctx->stream;
    static bool attr = false;
    if (!attr) {
        RMT_HIP(hipFuncSetAttribute((const void *)k_px_comb,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, PX_COMB_LDS));
        attr = true;
    }
    const unsigned gb = (unsigned)std::min<long>(4096, std::max<long>(1, ws.maxt / 4));
    const unsigned sb = (unsigned)ws.maxseg;
    for (int L = 0; L < ML; ++L) {
        k_px_c<<<gb, 256, 0, st>>>(ws, L, X1o, X2o);
        k_px_d<<<sb, 256, 0, st>>>(ws, L);
        k_px_comb<<<1, 64 * (PX_NP + 1), PX_COMB_LDS, st>>>(ws, L, X1o, X2o);
        k_px_out<<<sb, 64, 0, st>>>(ws, L, X1o, X2o);
        RMT_LAUNCHED();
    }
    return RMT_OK;
}

}  // namespace rmt

extern "C" int rmt_extrap_set_parallel(int on) {
    if ((on ? 1 : 0) != (rmt::extrap_par_enabled() ? 1 : 0)) rmt::extrap_config_changed();
    rmt::g_par = on ? 1 : 0;
    return RMT_OK;
}
