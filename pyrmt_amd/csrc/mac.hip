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
#include "extrap.hpp"
#include <algorithm>
#include <climits>
#include <cmath>
#include <vector>

namespace rmt {

constexpr int MAC_MAXD = 8;
// Box mode (rmt_mac_sim_step): disc k's map is zero and its phi = disc_phi(0, 0) > 0 outside
// the cells b[k] = {j0, j1, i0, i1} (half-open); n = 0: no boxes (every cell may hold
// anything).  contact: every disc_phi(0, 0) >= eps too, so a contact pair is +0.0 outside
// either disc's box and the stress S is +0.0 outside the union of the boxes.
struct SBox {
    int n, contact;
    int b[MAC_MAXD][4];
    __device__ __forceinline__ bool in(int k, int j, int i, int r = 0) const {
        return j >= b[k][0] - r && j < b[k][1] + r && i >= b[k][2] - r && i < b[k][3] + r;
    }
    // S may be nonzero within r cells of (j, i)
    __device__ __forceinline__ bool near(int j, int i, int r) const {
        if (!n || !contact) return true;
        for (int k = 0; k < n; ++k)
            if (in(k, j, i, r)) return true;
        return false;
    }
};
struct DiscSet {
    const double *X1[MAC_MAXD], *X2[MAC_MAXD], *phi[MAC_MAXD];
    int K;
    SBox bx;
};

// Index math of the per-cell / per-face kernels in 32 bits (a 64-bit division by a runtime
// divisor is a long emulated sequence): every index fits, N <= 32768 (rmt_mac_sim_create).
__device__ __forceinline__ int dv32(long x, int d) { return (int)((unsigned)x / (unsigned)d); }

// Every kernel takes global row ranges and global-index plane pointers (pointer - lo * row
// length), so the slab-decomposed step (rmt_mac_slab below) runs the same per-element code.
__global__ void k_mac_centres(const double *__restrict__ u, const double *__restrict__ v, int N,
                              double *__restrict__ uc, double *__restrict__ vc, int *bad, int jb,
                              int je) {
    const long c = (long)jb * N + blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (c >= (long)je * N) return;
    const int j = dv32(c, N), i = (int)(c - (long)j * N);
    const double a = 0.5 * (u[(long)j * (N + 1) + i] + u[(long)j * (N + 1) + i + 1]);
    const double b = 0.5 * (v[c] + v[c + N]);
    uc[c] = a; vc[c] = b;
    if (!(isfinite(a) && isfinite(b))) atomicOr(bad, 1);
}

// big (nullable): set when a phi is NaN, infinite or >= 2^928 in magnitude (k_mac_stress)
// one workgroup: the NaN-propagating max of G partials (NAN_MAX: nanmax, else k_reduce_p1<3>'s
// rule -- either is exact in any order) into *out
template <bool NAN_MAX>
__global__ void __launch_bounds__(1024) k_max_partials(const double *__restrict__ part, int G,
                                                      double init, double *__restrict__ out) {
    __shared__ double s[1024];
    double acc = init;
    for (int k = threadIdx.x; k < G; k += 1024) {
        const double y = part[k];
        acc = NAN_MAX ? nanmax(acc, y) : ((y > acc || y != y) ? y : acc);
    }
    s[threadIdx.x] = acc;
    __syncthreads();
    for (int w = 512; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) {
            const double y = s[threadIdx.x + w], x = s[threadIdx.x];
            s[threadIdx.x] = NAN_MAX ? nanmax(x, y) : ((y > x || y != y) ? y : x);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) *out = s[0];
}
constexpr int MP_BLOCKS = 8192;   // the fused reduction passes' workgroups (one partial each)

// k_mac_centres over the whole grid on MP_BLOCKS x RED_T threads, also folding max(u_c^2 +
// v_c^2) (NaN-propagating, k_reduce_p1<3>'s rule: a max is exact in any order) into one
// partial per block -- reduce_maxsq2_nan's pass over u_c, v_c saved
// WRITE: also the centre planes (off: the advection samples the faces itself, k_sim_sl_t<1>)
template <bool WRITE>
__global__ void __launch_bounds__(RED_T) k_mac_centres_m2(const double *__restrict__ u,
                                                          const double *__restrict__ v, int N,
                                                          double *__restrict__ uc,
                                                          double *__restrict__ vc, int *bad,
                                                          double *__restrict__ part) {
    __shared__ double s[RED_T];
    double acc = -INFINITY;
    bool fin = true;
    const long n = (long)N * N;
    constexpr int CM_U = 2;   // cells per trip, loads first (the max is exact in any order)
    const long S = (long)gridDim.x * RED_T;
    for (long c0 = blockIdx.x * (long)RED_T + threadIdx.x; c0 < n; c0 += CM_U * S) {
        double ul[CM_U], ur[CM_U], vd[CM_U], vu[CM_U];
#pragma unroll
        for (int m = 0; m < CM_U; ++m) {
            const long c = c0 + m * S;
            ul[m] = ur[m] = vd[m] = vu[m] = 0.0;
            if (c < n) {
                const int j = dv32(c, N), i = (int)(c - (long)j * N);
                ul[m] = u[(long)j * (N + 1) + i]; ur[m] = u[(long)j * (N + 1) + i + 1];
                vd[m] = v[c]; vu[m] = v[c + N];
            }
        }
#pragma unroll
        for (int m = 0; m < CM_U; ++m) {
            const long c = c0 + m * S;
            if (c >= n) break;
            const double a = 0.5 * (ul[m] + ur[m]);
            const double b = 0.5 * (vd[m] + vu[m]);
            if (WRITE) { uc[c] = a; vc[c] = b; }
            fin = fin && isfinite(a) && isfinite(b);
            const double x = a * a + b * b;
            acc = (x > acc || x != x) ? x : acc;
        }
    }
    if (!fin) atomicOr(bad, 1);
    s[threadIdx.x] = acc;
    __syncthreads();
    for (int w = RED_T / 2; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) {
            const double y = s[threadIdx.x + w];
            s[threadIdx.x] = (y > s[threadIdx.x] || y != y) ? y : s[threadIdx.x];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = s[0];
}

__global__ void k_mac_phi(const double *__restrict__ X1n, const double *__restrict__ X2n, long n,
                          double x0, double y0, double R, double *__restrict__ X1,
                          double *__restrict__ X2, double *__restrict__ phi, int *big = nullptr) {
    const long c = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (c >= n) return;
    const double a = X1n[c], b = X2n[c];
    X1[c] = a; X2[c] = b;
    const double ph = disc_phi(a, b, x0, y0, R);
    phi[c] = ph;
    if (big && !(fabs(ph) < 0x1p928)) atomicOr(big, 1);
}

// The support box of a disc's map: cells where X1 or X2 is not +-0 (NaN included), as
// {min row, max row, min col, max col} (box[0..3]; empty: {INT_MAX, -1, INT_MAX, -1}).
// Each block (256 cells of one row) leaves its column extent in bres[block] (x = INT_MAX:
// none), from its waves' ballots; k_box_reduce folds them (no contended atomics).
__device__ __forceinline__ void box_fold(bool nz, int i, int2 *bres) {
    __shared__ int smin[4], smax[4];
    const unsigned long long m = __ballot(nz);
    const int w = threadIdx.x >> 6, l0 = i - (int)(threadIdx.x & 63);   // lane 0's column
    if ((threadIdx.x & 63) == 0) {
        smin[w] = m ? l0 + __builtin_ctzll(m) : INT_MAX;
        smax[w] = m ? l0 + 63 - __builtin_clzll(m) : -1;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int a = INT_MAX, b = -1;
        for (int k = 0; k < (int)(blockDim.x >> 6); ++k) { a = min(a, smin[k]); b = max(b, smax[k]); }
        bres[(long)blockIdx.y * gridDim.x + blockIdx.x] = make_int2(a, b);
    }
}
// one workgroup: the box of nrows x nbx block extents (row r of them is grid row j0 + r)
__global__ void __launch_bounds__(1024) k_box_reduce(const int2 *__restrict__ bres, int nbx,
                                                     int nrows, int j0, int *box) {
    __shared__ int s[4][1024];
    int jmin = INT_MAX, jmax = -1, imin = INT_MAX, imax = -1;
    for (long e = threadIdx.x; e < (long)nbx * nrows; e += 1024) {
        const int2 v = bres[e];
        if (v.y >= 0) {
            const int j = j0 + (int)(e / nbx);
            jmin = min(jmin, j); jmax = max(jmax, j);
            imin = min(imin, v.x); imax = max(imax, v.y);
        }
    }
    s[0][threadIdx.x] = jmin; s[1][threadIdx.x] = jmax; s[2][threadIdx.x] = imin; s[3][threadIdx.x] = imax;
    __syncthreads();
    for (int h = 512; h > 0; h >>= 1) {
        if ((int)threadIdx.x < h) {
            s[0][threadIdx.x] = min(s[0][threadIdx.x], s[0][threadIdx.x + h]);
            s[1][threadIdx.x] = max(s[1][threadIdx.x], s[1][threadIdx.x + h]);
            s[2][threadIdx.x] = min(s[2][threadIdx.x], s[2][threadIdx.x + h]);
            s[3][threadIdx.x] = max(s[3][threadIdx.x], s[3][threadIdx.x + h]);
        }
        __syncthreads();
    }
    if (threadIdx.x < 4) box[threadIdx.x] = s[threadIdx.x][0];
}
// phi = disc_phi(X1, X2) over the grid and the support box (rmt_mac_sim_step's start in the
// box mode: phi then holds disc_phi(0, 0) wherever the map is zero, as every later step keeps)
__global__ void __launch_bounds__(256) k_mac_box_phi(const double *__restrict__ X1,
                                                     const double *__restrict__ X2, int N,
                                                     double x0, double y0, double R,
                                                     double *__restrict__ phi, int2 *bres) {
    const int j = blockIdx.y, i = blockIdx.x * 256 + threadIdx.x;
    bool nz = false;
    if (i < N) {
        const long c = (long)j * N + i;
        const double a = X1[c], b = X2[c];
        phi[c] = disc_phi(a, b, x0, y0, R);
        nz = !(a == 0.0 && b == 0.0);
    }
    box_fold(nz, i, bres);
}
// k_mac_phi on the cells [j0, j1) x [i0, i1) only, and the new map's support box
__global__ void __launch_bounds__(256) k_mac_phi_box(const double *__restrict__ X1n,
                                                     const double *__restrict__ X2n, int N, int j0,
                                                     int i0, int i1, double x0, double y0,
                                                     double R, double *__restrict__ X1,
                                                     double *__restrict__ X2,
                                                     double *__restrict__ phi, int *big,
                                                     int2 *bres) {
    const int j = j0 + blockIdx.y, i = i0 + blockIdx.x * 256 + threadIdx.x;
    bool nz = false;
    if (i < i1) {
        const long c = (long)j * N + i;
        const double a = X1n[c], b = X2n[c];
        X1[c] = a; X2[c] = b;
        const double ph = disc_phi(a, b, x0, y0, R);
        phi[c] = ph;
        if (!(fabs(ph) < 0x1p928)) atomicOr(big, 1);
        nz = !(a == 0.0 && b == 0.0);
    }
    box_fold(nz, i, bres);
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
                                                       double *__restrict__ part, int jb, int je,
                                                       int jr0, int jr1, bool skip_ok,
                                                       const int *__restrict__ phi_big = nullptr,
                                                       bool box_launch = false) {
    const bool phi_ok = phi_big && *phi_big == 0;
    // S on rows [jb, je); the J range over rows [jr0, jr1).  box_launch (box mode with
    // contact set): block row y covers disc y's box grown by 6 cells -- every cell the
    // predictor reads S at (see below); overlapping boxes compute a cell twice, the same
    // values.  Partials: one (min J, max J) pair per block.
    __shared__ double smin[MS_TPB], smax[MS_TPB];
    double jmin = 1.0, jmax = 1.0;
    int r0 = jb, c0 = 0, w = N;
    long area = (long)(je - jb) * N;
    if (box_launch) {
        const int *b = D.bx.b[blockIdx.y];
        r0 = max(jb, b[0] - 6); c0 = max(0, b[2] - 6);
        w = max(0, min(N, b[3] + 6) - c0);
        area = (long)max(0, min(je, b[1] + 6) - r0) * w;
    }
    for (long t = blockIdx.x * (long)MS_TPB + threadIdx.x; t < area;
         t += (long)gridDim.x * MS_TPB) {
        const int tj = dv32(t, w);
        const int j = r0 + tj, i = c0 + (int)(t - (long)tj * w);
        const long c = (long)j * N + i;
        const bool own = j >= jr0 && j < jr1;
        // The sums start at +0.0 and only add, so they are never -0.0: adding a +-0.0 term
        // leaves them bit for bit unchanged.  Two kinds of term are exactly +-0.0 and skipped:
        //  * a disc's stress outside its solid (solid_stress_cell: sigma = 0) with a finite
        //    phi there (omh finite: omh * 0 = +-0; a NaN phi takes the product, NaN);
        //  * a contact pair where either phi >= eps or is NaN (fc = min(fa, fb) = +0.0, s =
        //    -0.0) and both gradient numerators are finite and below 2^930: then |gx|, |gy| <
        //    2^930 / (2 h) (host: 2 h >= 2^-30), nx, ny are finite (|n| <= 1 or mag = inf),
        //    and txx, txy, tyy = -0.0 * finite = +-0.0.  With phi_big clear (k_mac_phi: every
        //    phi finite and below 2^928) every numerator is, and the test is skipped.
        // S is +0.0 away from every box and k_mac_predict reads it only within 3 cells of a
        // face within 3 cells of a box: cells farther than 6 from every box are not written
        if (D.bx.n && D.bx.contact && !D.bx.near(j, i, 6)) continue;
        double axx = 0.0, axy = 0.0, ayy = 0.0;
        const bool inner = j >= 1 && j < N - 1 && i >= 1 && i < N - 1;
        for (int k = 0; k < D.K; ++k) {
            if (D.bx.n && !D.bx.in(k, j, i)) continue;   // phi_k = disc_phi(0, 0) > 0: no term
            Stress s{0.0, 0.0, 0.0, 1.0};
            const bool st = inner && solid_stress_cell(D.X1[k], D.X2[k], D.phi[k], c, N, dx, dy,
                                                       mu_s, 0.0, 0.0, 0.0, false, s);
            const double ph = D.phi[k][c];
            if (st || ph != ph) {
                const double omh = 1 - heaviside(ph, w_t);
                axx = axx + omh * s.sxx; axy = axy + omh * s.sxy; ayy = ayy + omh * s.syy;
            }
            if (own) { jmin = fmin(jmin, s.J); jmax = fmax(jmax, s.J); }
        }
        if (eta > 0)
            for (int a = 0; a < D.K; ++a)
                for (int b = a + 1; b < D.K; ++b) {
                    const double *pa = D.phi[a], *pb = D.phi[b];
                    // outside a box with contact set, that disc's phi is >= eps (fc = +0.0)
                    if (skip_ok && phi_ok && D.bx.n && D.bx.contact &&
                        !(D.bx.in(a, j, i) && D.bx.in(b, j, i)))
                        continue;
                    if (skip_ok && !(pa[c] < eps && pb[c] < eps)) {
                        if (phi_ok) continue;
                        const double gxn = i >= 1 && i < N - 1
                                               ? (pa[c + 1] - pb[c + 1]) - (pa[c - 1] - pb[c - 1])
                                               : 0.0;
                        const double gyn = j >= 1 && j < N - 1
                                               ? (pa[c + N] - pb[c + N]) - (pa[c - N] - pb[c - N])
                                               : 0.0;
                        if (fabs(gxn) < 0x1p930 && fabs(gyn) < 0x1p930) continue;
                    }
                    double txx, txy, tyy;
                    contact_cell(pa, pb, c, j, i, N, eta, 2 * mu_s, eps, dx, dy, txx, txy, tyy);
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
    if (threadIdx.x == 0) {
        const long pb = (long)blockIdx.y * gridDim.x + blockIdx.x;
        part[2 * pb] = smin[0]; part[2 * pb + 1] = smax[0];
    }
}

// k_mac_stress's zero-term skip needs 2 h >= 2^-30 and finite contact constants (see there)
static bool stress_skip_ok(const rmt_mac_params &P) {
    return 2.0 * P.dx >= 0x1p-30 && std::isfinite(P.eta) && std::isfinite(2.0 * P.mu_s);
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
// Faces: u rows [F.u0, F.u1) (stride N + 1) then v rows [F.v0, F.v1) (stride N), one thread
// each.
struct FaceRows {
    int u0, u1, v0, v1;
};
__host__ __device__ inline long face_count(const FaceRows &F, int N) {
    return (long)(F.u1 - F.u0) * (N + 1) + (long)(F.v1 - F.v0) * N;
}
__global__ void k_mac_predict(const double *__restrict__ u, const double *__restrict__ v,
                              const double *__restrict__ Sxx, const double *__restrict__ Sxy,
                              const double *__restrict__ Syy, const double *__restrict__ fu,
                              const double *__restrict__ fv, int N, double nu, double dx,
                              double dy, double dx2, double dy2, double dt, double U, double rho,
                              double *__restrict__ us, double *__restrict__ vs, FaceRows F,
                              SBox bx = SBox{}) {
    // dx2, dy2: the reference's dx**2 on a Python float (libm pow), computed on the host
    const long t = blockIdx.x * (long)blockDim.x + threadIdx.x;
    const int W = N + 1;
    const long nuf = (long)(F.u1 - F.u0) * W, q = (long)F.u0 * W + t;
    if (t < nuf) {   // u face (j, i), row stride N + 1
        const int j = dv32(q, W), i = (int)(q - (long)j * W);
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
        // (where S is +0.0 on the whole stencil the divergences are +0.0: the same sum)
        if (Sxx && !bx.near(j, i, 3)) r = r + 0.5 * (0.0 + 0.0) / rho;
        else if (Sxx) r = r + 0.5 * (divx_at(Sxx, Sxy, j, i, N, dx, dy) + divx_at(Sxx, Sxy, j, i - 1, N, dx, dy)) / rho;
        else if (fu) r = r + fu[q] / rho;
        us[q] = uc + dt * r;
    } else if (t < nuf + (long)(F.v1 - F.v0) * N) {   // v face (j, i), row stride N
        const long p = (long)F.v0 * N + (t - nuf);
        const int j = dv32(p, N), i = (int)(p - (long)j * N);
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
        if (Sxx && !bx.near(j, i, 3)) r = r + 0.5 * (0.0 + 0.0) / rho;
        else if (Sxx) r = r + 0.5 * (divy_at(Sxy, Syy, j, i, N, dx, dy) + divy_at(Sxy, Syy, j - 1, i, N, dx, dy)) / rho;
        else if (fv) r = r + fv[p] / rho;
        vs[p] = vc + dt * r;
    }
}

// rhs = (rho / dt) * div(u*, v*)  (mac.py:81-84, 133-134)
__global__ void k_mac_rhs(const double *__restrict__ u, const double *__restrict__ v, int N,
                          double dx, double dy, double coef, double *__restrict__ rhs, int jb,
                          int je) {
    const long c = (long)jb * N + blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (c >= (long)je * N) return;
    const int j = dv32(c, N), i = (int)(c - (long)j * N);
    const long cu = (long)j * (N + 1) + i;
    const double d = (u[cu + 1] - u[cu]) / dx + (v[c + N] - v[c]) / dy;
    rhs[c] = coef * d;
}

// k_mac_rhs with its row sums: one block per row (N rows), each thread the columns t,
// t + 256, ... -- rhs written as k_mac_rhs writes it, and summed in k_rowsum's order (the
// strided partials, then the halving tree), so the row-tree root is the one rowtree_root
// would form from the written plane
__global__ void __launch_bounds__(256) k_mac_rhs_rows(const double *__restrict__ u,
                                                      const double *__restrict__ v, int N,
                                                      double dx, double dy, double coef,
                                                      double *__restrict__ rhs,
                                                      double *__restrict__ rs) {
    __shared__ double s[256];
    const int j = blockIdx.x;
    double acc = 0.0;
    for (int i = threadIdx.x; i < N; i += 256) {
        const long c = (long)j * N + i, cu = (long)j * (N + 1) + i;
        const double d = (u[cu + 1] - u[cu]) / dx + (v[c + N] - v[c]) / dy;
        const double r = coef * d;
        rhs[c] = r;
        acc += r;
    }
    s[threadIdx.x] = acc;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w) s[threadIdx.x] = s[threadIdx.x] + s[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) rs[j] = s[0];
}

// u = u* - (dt/rho) grad_p_u(phi), v likewise (mac.py:87-101, 137-138)
__global__ void k_mac_correct(const double *__restrict__ us, const double *__restrict__ vs,
                              const double *__restrict__ phi, int N, double dx, double dy,
                              double c0, double *__restrict__ u, double *__restrict__ v,
                              FaceRows F) {
    const long t = blockIdx.x * (long)blockDim.x + threadIdx.x;
    const long nuf = (long)(F.u1 - F.u0) * (N + 1), q = (long)F.u0 * (N + 1) + t;
    if (t < nuf) {
        const int j = dv32(q, N + 1), i = (int)(q - (long)j * (N + 1));
        const double g = (i == 0 || i == N) ? 0.0 : (phi[(long)j * N + i] - phi[(long)j * N + i - 1]) / dx;
        u[q] = us[q] - c0 * g;
    } else if (t < nuf + (long)(F.v1 - F.v0) * N) {
        const long p = (long)F.v0 * N + (t - nuf);
        const int j = dv32(p, N);
        const double g = (j == 0 || j == N) ? 0.0 : (phi[p] - phi[p - N]) / dy;
        v[p] = vs[p] - c0 * g;
    }
}

// k_mac_correct over the whole grid on MP_BLOCKS x RED_T threads (u faces, then v faces),
// also folding max |u| over the u faces (nanmax: exact in any order) into one partial per
// block -- k_mac_diag's pass over u saved (it is then launched with u = nullptr)
__global__ void __launch_bounds__(RED_T) k_mac_correct_um(const double *__restrict__ us,
                                                          const double *__restrict__ vs,
                                                          const double *__restrict__ phi, int N,
                                                          double dx, double dy, double c0,
                                                          double *__restrict__ u,
                                                          double *__restrict__ v,
                                                          double *__restrict__ part,
                                                          double *__restrict__ partv = nullptr) {
    // partv (nullable): the same NaN-propagating max |v| partials (k_m2_bound)
    __shared__ double s[RED_T];
    double acc = 0.0, accv = 0.0;
    const long nuf = (long)N * (N + 1), tot = 2 * nuf;
    // CU_U faces per trip: their loads issued together, then written in face order (the max
    // is exact in any order)
    constexpr int CU_U = 2;
    const long S = (long)gridDim.x * RED_T;
    for (long t0 = blockIdx.x * (long)RED_T + threadIdx.x; t0 < tot; t0 += CU_U * S) {
        double a[CU_U], p1[CU_U], p0[CU_U];
#pragma unroll
        for (int m = 0; m < CU_U; ++m) {
            const long t = t0 + m * S;
            a[m] = 0.0; p1[m] = 0.0; p0[m] = 0.0;
            if (t < nuf) {
                const int j = dv32(t, N + 1), i = (int)(t - (long)j * (N + 1));
                a[m] = us[t];
                if (!(i == 0 || i == N)) { p1[m] = phi[(long)j * N + i]; p0[m] = phi[(long)j * N + i - 1]; }
            } else if (t < tot) {
                const long q = t - nuf;
                const int j = dv32(q, N);
                a[m] = vs[q];
                if (!(j == 0 || j == N)) { p1[m] = phi[q]; p0[m] = phi[q - N]; }
            }
        }
#pragma unroll
        for (int m = 0; m < CU_U; ++m) {
            const long t = t0 + m * S;
            if (t < nuf) {
                const int j = dv32(t, N + 1), i = (int)(t - (long)j * (N + 1));
                const double g = (i == 0 || i == N) ? 0.0 : (p1[m] - p0[m]) / dx;
                const double x = a[m] - c0 * g;
                u[t] = x;
                acc = nanmax(acc, fabs(x));
            } else if (t < tot) {
                const long q = t - nuf;
                const int j = dv32(q, N);
                const double g = (j == 0 || j == N) ? 0.0 : (p1[m] - p0[m]) / dy;
                const double y = a[m] - c0 * g;
                v[q] = y;
                accv = nanmax(accv, fabs(y));
            }
        }
    }
    s[threadIdx.x] = acc;
    __syncthreads();
    for (int w = RED_T / 2; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) s[threadIdx.x] = nanmax(s[threadIdx.x], s[threadIdx.x + w]);
        __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = s[0];
    if (!partv) return;
    __syncthreads();
    s[threadIdx.x] = accv;
    __syncthreads();
    for (int w = RED_T / 2; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) s[threadIdx.x] = nanmax(s[threadIdx.x], s[threadIdx.x + w]);
        __syncthreads();
    }
    if (threadIdx.x == 0) partv[blockIdx.x] = s[0];
}
// The next step's SL bound from the correction's face maxima (u, v unchanged since): a cell
// centre value is the mean of two faces, so |u_c| <= max |u|, |v_c| <= max |v| and
// m2 = max|u|^2 + max|v|^2 bounds max(u_c^2 + v_c^2) -- the block-skip certificate only needs
// a bound, and a looser one only skips fewer tiles (the same values either way).  The
// non-finite flag: a face NaN / inf makes the max NaN / inf (a centre value is then
// non-finite as well; two finite faces whose sum overflows are the one case not flagged).
__global__ void __launch_bounds__(1024) k_m2_bound(const double *__restrict__ pu,
                                                   const double *__restrict__ pv, int G,
                                                   int *__restrict__ bad, double *__restrict__ out) {
    __shared__ double s[2][1024];
    double a = 0.0, b = 0.0;
    for (int k = threadIdx.x; k < G; k += 1024) { a = nanmax(a, pu[k]); b = nanmax(b, pv[k]); }
    s[0][threadIdx.x] = a; s[1][threadIdx.x] = b;
    __syncthreads();
    for (int w = 512; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) {
            s[0][threadIdx.x] = nanmax(s[0][threadIdx.x], s[0][threadIdx.x + w]);
            s[1][threadIdx.x] = nanmax(s[1][threadIdx.x], s[1][threadIdx.x + w]);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const double mu = s[0][0], mv = s[1][0];
        // a face above DBL_MAX / 2 may give an overflowing centre velocity (the sum of two
        // faces): flagged as k_mac_centres flagged a non-finite centre
        const double half_max = 0x1.fffffffffffffp1022;
        if (!(isfinite(mu) && isfinite(mv)) || mu > half_max || mv > half_max) atomicOr(bad, 1);
        *out = mu * mu + mv * mv;
    }
}

// per-disc centroid sums over phi <= 0 (x, y, count) and max|u| partials (u nullable: the
// max comes from k_mac_correct_um)
constexpr int MD_VALS = 3 * MAC_MAXD + 1;
// (rows [jb, je): cells and u faces).  Without u, only the items of rows [r0, r1) are
// visited, the rows holding every box (outside its box phi_k > 0 adds nothing): each thread
// still takes its items in increasing order, so the sums are those of the whole range.
__global__ void __launch_bounds__(MS_TPB) k_mac_diag(DiscSet D, const double *__restrict__ u,
                                                     int N, double dx, double *__restrict__ part,
                                                     int jb, int je, int r0, int r1) {
    __shared__ double s[MS_TPB];
    double acc[MD_VALS];
    for (int k = 0; k < MD_VALS; ++k) acc[k] = 0.0;
    const long n = (long)(je - jb) * N, nf = (long)(je - jb) * (N + 1);
    // MD_U grid-stride items per trip: their loads are issued together, then accumulated in
    // item order (the same sums as one item per trip)
    constexpr int MD_U = 4;
    const long S = (long)MS_BLOCKS * MS_TPB;
    long tfirst = blockIdx.x * (long)MS_TPB + threadIdx.x, tend = nf;
    if (!u) {
        const long tlo = (long)(max(r0, jb) - jb) * N;
        tend = min(n, (long)(max(r1, jb) - jb) * N);
        if (tlo > tfirst) tfirst += (tlo - tfirst) / S * S;   // (the last item of this thread below tlo)
    }
    for (long t0 = tfirst; t0 < tend; t0 += MD_U * S) {
        double ua[MD_U];
        unsigned in[MD_U];   // bit k: phi_k <= 0 at the item's cell
#pragma unroll
        for (int m = 0; m < MD_U; ++m) {
            const long t = t0 + m * S;
            ua[m] = t < nf && u ? u[(long)jb * (N + 1) + t] : 0.0;
            in[m] = 0;
            if (t < n && t < tend) {
                const long c = (long)jb * N + t;
                const int j = dv32(c, N), i = (int)(c - (long)j * N);
#pragma unroll
                for (int k = 0; k < MAC_MAXD; ++k)   // (outside its box phi_k > 0)
                    if (k < D.K && (!D.bx.n || D.bx.in(k, j, i)) && D.phi[k][c] <= 0.0)
                        in[m] |= 1u << k;
            }
        }
#pragma unroll
        for (int m = 0; m < MD_U; ++m) {
            const long t = t0 + m * S;
            if (t >= tend) break;
            acc[3 * MAC_MAXD] = nanmax(acc[3 * MAC_MAXD], fabs(ua[m]));
            if (t < n) {
                const long c = (long)jb * N + t;
                const int j = dv32(c, N), i = (int)(c - (long)j * N);
                const double xc = (i + 0.5) * dx, yc = (j + 0.5) * dx;
                for (int k = 0; k < D.K; ++k)
                    if ((in[m] >> k) & 1) { acc[3 * k] += xc; acc[3 * k + 1] += yc; acc[3 * k + 2] += 1.0; }
            }
        }
    }
    for (int k = 0; k < MD_VALS; ++k) {
        s[threadIdx.x] = acc[k];
        __syncthreads();
        for (int w = MS_TPB / 2; w > 0; w >>= 1) {
            if (threadIdx.x < w)
                s[threadIdx.x] = k == 3 * MAC_MAXD ? nanmax(s[threadIdx.x], s[threadIdx.x + w])
                                                   : s[threadIdx.x] + s[threadIdx.x + w];
            __syncthreads();
        }
        if (threadIdx.x == 0) part[(long)blockIdx.x * MD_VALS + k] = s[0];
        __syncthreads();
    }
}

static int mac_project_impl(rmt_ctx *ctx, const double *us, const double *vs, double dx,
                            double dy, double dt, double rho, double *u, double *v, double *phi,
                            double *rhs, bool plan = true, double *umax_part = nullptr,
                            double *vmax_part = nullptr) {
    const int N = ctx->nx;
    const long nf = (long)N * (N + 1);
    if (plan) RMT_TRY(dct2_plan(ctx, N, N, dx, dy));
    // rhs - rhs.mean() (mac.py:135): the row sums with the rhs, the row-tree root, and the
    // subtraction on the DCT's first load (the values sub_mean_rows would leave in rhs;
    // nothing else reads them)
    double *root = ctx->red + RED_BLOCKS + 16;
    RMT_CHECK(N <= ctx->rsum_len, RMT_EINVAL, "mac projection: rows out of range");
    k_mac_rhs_rows<<<N, 256, 0, ctx->stream>>>(us, vs, N, dx, dy, rho / dt, rhs, ctx->rsum);
    RMT_LAUNCHED();
    RMT_TRY(rowtree_sums(ctx, N, root));
    RMT_TRY(dct2_solve(ctx, rhs, phi, root, (double)N * N));
    if (umax_part)
        k_mac_correct_um<<<MP_BLOCKS, RED_T, 0, ctx->stream>>>(us, vs, phi, N, dx, dy, dt / rho,
                                                                u, v, umax_part, vmax_part);
    else
        k_mac_correct<<<grid1d(2 * nf, 256), 256, 0, ctx->stream>>>(us, vs, phi, N, dx, dy,
                                                                    dt / rho, u, v,
                                                                    FaceRows{0, N, 0, N + 1});
    RMT_LAUNCHED();
    return RMT_OK;
}

}  // namespace rmt

// ------------------------------------------------------------------ fused MAC sim --
struct rmt_mac_sim {
    rmt_ctx *ctx = nullptr;
    rmt_mac_params P{};
    void *block = nullptr;
    int *cand = nullptr;   // the no-op test's candidate list (CAND_CAP cells + counter)
    double *u, *v, *p, *us, *vs, *uc, *vc, *X1n, *X2n, *phi_pre, *Sxx, *Sxy, *Syy;
    double *X1[RMT_MAC_MAXD], *X2[RMT_MAC_MAXD], *phi[RMT_MAC_MAXD];
    double *xs, *ys, *part, *out;
    unsigned long long *kbits;   // the advection's known plane (phi_pre < 0), 64-cell words
    int *flags;
    int2 *bres;                  // per-block column extents of the box passes (box_fold)
    double *mpart;               // per-block maxima of the fused reduction passes
    double *mpartv;              // (the correction's max |v| partials: k_m2_bound)
    int *dbox;                   // [K][4] device support boxes (k_box_reduce), host copy:
    int hbox[RMT_MAC_MAXD][4];
    double t = 0;
    bool diverged = false;
    std::vector<rmt_mac_diag> diag;
};

using namespace rmt;

extern "C" {

int rmt_mac_divergence(rmt_ctx *ctx, const double *u, const double *v, double dx, double dy,
                       double *out) {
    RMT_CHECK(ctx && u && v && out && ctx->nx == ctx->ny, RMT_EINVAL, "bad argument");
    const long n = (long)ctx->nx * ctx->nx;
    k_mac_rhs<<<grid1d(n, 256), 256, 0, ctx->stream>>>(u, v, ctx->nx, dx, dy, 1.0, out, 0,
                                                       ctx->nx);
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
                                                                dx, dy, -1.0, gu, gv,
                                                                FaceRows{0, N, 0, N + 1});
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
        std::pow(dy, 2.0), dt, U_lid, rho, us, vs, FaceRows{0, N, 0, N + 1});
    RMT_LAUNCHED();
    return RMT_OK;
}

int rmt_mac_contact_stress(rmt_ctx *ctx, const double *phi_a, const double *phi_b, double eta,
                           double Gsum, double eps, double dx, double dy, double *txx,
                           double *txy, double *tyy);

// candidate capacity of the no-op test's list: 32 cells per grid row (a disc's rim holds
// about 4 per row it spans; beyond the capacity k_ex_none_list walks the rows instead)
static int mac_cand_cap(int N) { return 32 * N; }

int rmt_mac_sim_create(rmt_ctx *ctx, const rmt_mac_params *prm, rmt_mac_sim **out) {
    RMT_CHECK(ctx && prm && out, RMT_EINVAL, "null argument");
    RMT_CHECK(prm->n_discs >= 1 && prm->n_discs <= RMT_MAC_MAXD, RMT_EINVAL, "1..8 discs");
    RMT_CHECK(prm->N >= 4 && prm->N <= 32768, RMT_EINVAL, "N in 4..32768 (32-bit face indices)");
    RMT_CHECK(ctx->nx == prm->N && ctx->ny == prm->N, RMT_EINVAL, "ctx grid != N x N");
    const int N = prm->N;
    RMT_TRY(dct2_plan(ctx, N, N, prm->dx, prm->dx));
    rmt_mac_sim *S = new rmt_mac_sim;
    S->ctx = ctx; S->P = *prm;
    const long n = (long)N * N, nf = (long)N * (N + 1);
    const int K = prm->n_discs;
    const size_t dbl = 5 * nf + (9 + 3 * K) * n + 2 * N + (2 + MD_VALS) * MS_BLOCKS + 64 + 32 +
                       2 * MP_BLOCKS;
    RMT_HIP(hipMalloc(&S->block, dbl * 8 + 64));
    RMT_HIP(hipMemsetAsync(S->block, 0, dbl * 8 + 64, ctx->stream));
    double *q = (double *)S->block;
    double **faces[] = {&S->u, &S->v, &S->us, &S->vs};
    for (auto pp : faces) { *pp = q; q += nf; }
    // the spare face plane: the known-plane words (ceil(N / 64) per row), then the box
    // pass's per-block extents ((N / 256 + 1) x N) -- together far below nf doubles
    S->kbits = (unsigned long long *)q;
    S->bres = (int2 *)(q + (long)N * ((N + 63) / 64));

    q += nf;
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
    S->mpart = q; q += MP_BLOCKS;
    S->mpartv = q; q += MP_BLOCKS;
    S->dbox = (int *)q; q += 4 * RMT_MAC_MAXD / 2;
    S->flags = (int *)q;
    // index-grid coordinates (mac_multi_disc_lid.py:41): Xg = arange(N) * dx
    std::vector<double> g(N);
    for (int i = 0; i < N; ++i) g[i] = i * prm->dx;
    RMT_HIP(hipMemcpyAsync(S->xs, g.data(), N * 8, hipMemcpyHostToDevice, ctx->stream));
    RMT_HIP(hipMemcpyAsync(S->ys, g.data(), N * 8, hipMemcpyHostToDevice, ctx->stream));
    RMT_TRY(ensure_bytes(ctx, extrap_workspace(N, N, prm->layers)));
    RMT_HIP(hipMalloc(&S->cand, (mac_cand_cap(N) + 1) * sizeof(int)));
    RMT_HIP(hipStreamSynchronize(ctx->stream));
    *out = S;
    return RMT_OK;
}

int rmt_mac_sim_destroy(rmt_mac_sim *S) {
    if (!S) return RMT_OK;
    (void)hipFree(S->block);
    (void)hipFree(S->cand);
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
    // Box mode: a disc's advection, extrapolation and phi run only on its map's support box
    // grown by G cells.  Exact when the origin lies outside every reference disc (disc_phi(0,
    // 0) > 0): then a zero map cell is not known and its SL mask is 0, so the advected map is
    // zero outside the old support, the extrapolation's targets lie within `layers` cells of
    // known cells and it reads values within 4 more (9 x 9 windows), and phi = disc_phi(0, 0)
    // wherever the map stays zero.  The box comes back with each step's diagnostics (no
    // extra host round trip); a call starts with one full pass per disc (phi, box).
    const int G = P.layers + 6;
    bool box_mode = ctx->opt.mac_boxes != 0 && P.layers > 0;
    D.bx.contact = 1;
    for (int k = 0; k < K; ++k) {
        const double p0 = std::sqrt(P.cx[k] * P.cx[k] + P.cy[k] * P.cy[k]) - P.R[k];
        box_mode = box_mode && p0 > 0.0;
        D.bx.contact = D.bx.contact && p0 >= eps;   // (a contact term needs both phi < eps)
    }
    D.bx.n = 0;   // set per step once the boxes are known
    const size_t kb_bytes = (size_t)N * ((N + 63) / 64) * sizeof(unsigned long long);
    if (box_mode && nsteps > 0 && S->t < t_end && !S->diverged) {
        for (int k = 0; k < K; ++k) {
            k_mac_box_phi<<<dim3((N + 255) / 256, N), 256, 0, st>>>(
                S->X1[k], S->X2[k], N, P.cx[k], P.cy[k], P.R[k], S->phi[k], S->bres);
            k_box_reduce<<<1, 1024, 0, st>>>(S->bres, (N + 255) / 256, N, 0, S->dbox + 4 * k);
            RMT_LAUNCHED();
        }
        RMT_HIP(hipMemcpyAsync(S->hbox, S->dbox, 4 * K * sizeof(int), hipMemcpyDeviceToHost, st));
        RMT_HIP(hipStreamSynchronize(st));
    }
    for (int it = 0; it < nsteps; ++it) {
        if (!(S->t < t_end) || S->diverged) break;
        double dt = P.dt;
        if (S->t + dt > t_end) dt = t_end - S->t;
        RMT_HIP(hipMemsetAsync(S->flags, 0, 5 * sizeof(int), st));   // [4]: k_mac_phi's big
        // with max |u_c|^2, which bounds every velocity sample of the backtraces (the SL
        // block skip)
        const bool face_sl = ctx->opt.mac_face_sl != 0;
        // within a call the previous step's correction has the face maxima (m2_bound)
        const bool m2b = face_sl && it > 0 && ctx->opt.mac_m2_bound != 0;
        if (m2b)
            k_m2_bound<<<1, 1024, 0, st>>>(S->mpart, S->mpartv, MP_BLOCKS, S->flags, S->out + 8);
        else if (face_sl)
            k_mac_centres_m2<false><<<MP_BLOCKS, RED_T, 0, st>>>(S->u, S->v, N, S->uc, S->vc,
                                                                 S->flags, S->mpart);
        else
            k_mac_centres_m2<true><<<MP_BLOCKS, RED_T, 0, st>>>(S->u, S->v, N, S->uc, S->vc,
                                                                S->flags, S->mpart);
        if (!m2b)
            k_max_partials<false><<<1, 1024, 0, st>>>(S->mpart, MP_BLOCKS, -INFINITY, S->out + 8);
        RMT_LAUNCHED();
        for (int k = 0; k < K; ++k) {
            int cb[4] = {0, N, 0, N};   // the cells this disc's passes cover
            if (box_mode) {
                D.bx.n = K;
                const int *b = S->hbox[k];
                if (b[1] < b[0]) { cb[1] = 0; cb[3] = 0; }   // empty map
                else {
                    cb[0] = std::max(0, b[0] - G); cb[1] = std::min(N, b[1] + 1 + G);
                    cb[2] = std::max(0, b[2] - G); cb[3] = std::min(N, b[3] + 1 + G);
                    // whole SL tiles: the phi pass covers exactly the cells they advected
                    cb[0] -= cb[0] % 4; cb[1] = std::min(N, (cb[1] + 3) / 4 * 4);
                    cb[2] -= cb[2] % 64; cb[3] = std::min(N, (cb[3] + 63) / 64 * 64);
                }
                RMT_HIP(hipMemsetAsync(S->kbits, 0, kb_bytes, st));
            }
            for (int q = 0; q < 4; ++q) D.bx.b[k][q] = cb[q];   // (the stress / diag passes)
            // phi from the current map (already S->phi[k]), advect with the pre-advection mask
            RMT_TRY(sl_disc_map(ctx, S->X1[k], S->X2[k], face_sl ? S->u : S->uc,
                                face_sl ? S->v : S->vc, S->xs, S->ys, dt, dx, dx, P.cx[k],
                                P.cy[k], P.R[k], S->X1n, S->X2n, S->phi_pre, S->flags + 1,
                                S->out + 8, S->kbits, box_mode ? cb : nullptr, face_sl));
            // the known plane from the advection pass (its k_ex_bits pass over phi_pre saved);
            // the no-op test over every row at once (a disc with nothing to fit scans them all)
            ctx->ex_none_wide = true;
            // box mode: the known cells lie in rows [cb0, cb1) (kbits cleared elsewhere), so a
            // candidate -- an unknown 8-neighbour of a known cell -- in [cb0 - 1, cb1 + 1)
            if (box_mode) {
                ctx->ex_none_rows[0] = std::max(0, cb[0] - 1);
                ctx->ex_none_rows[1] = cb[1] > cb[0] ? std::min(N, cb[1] + 1) : 1;
                if (cb[1] <= cb[0]) ctx->ex_none_rows[0] = 0;   // (empty map: one row, no candidate)
                // likewise the columns [cb2 - 1, cb3 + 1): their 64-column words
                ctx->ex_none_cols[0] = std::max(0, cb[2] - 1) >> 6;
                ctx->ex_none_cols[1] = cb[3] > cb[2] ? (std::min(N - 1, cb[3]) >> 6) + 1 : 1;
            }
            ctx->ex_cand = S->cand; ctx->ex_cand_cap = mac_cand_cap(N);
            ctx->ex_none_host = ctx->opt.mac_noop_host != 0;
            const int es = extrapolate(ctx, S->X1n, S->X2n, S->phi_pre, dx, dx, P.layers, S->X1n,
                                       S->X2n, S->flags + 2, S->kbits);
            ctx->ex_none_wide = false;
            ctx->ex_none_rows[0] = ctx->ex_none_rows[1] = 0;
            ctx->ex_none_cols[0] = ctx->ex_none_cols[1] = 0;
            ctx->ex_cand = nullptr; ctx->ex_cand_cap = 0;
            ctx->ex_none_host = false;
            RMT_TRY(es);
            if (!box_mode)
                k_mac_phi<<<grid1d(n, 256), 256, 0, st>>>(S->X1n, S->X2n, n, P.cx[k], P.cy[k],
                                                          P.R[k], S->X1[k], S->X2[k], S->phi[k],
                                                          S->flags + 4);
            else if (cb[1] > cb[0] && cb[3] > cb[2]) {
                const int nbx = (cb[3] - cb[2] + 255) / 256;
                k_mac_phi_box<<<dim3(nbx, cb[1] - cb[0]), 256, 0, st>>>(
                    S->X1n, S->X2n, N, cb[0], cb[2], cb[3], P.cx[k], P.cy[k], P.R[k], S->X1[k],
                    S->X2[k], S->phi[k], S->flags + 4, S->bres);
                k_box_reduce<<<1, 1024, 0, st>>>(S->bres, nbx, cb[1] - cb[0], cb[0],
                                                  S->dbox + 4 * k);
            } else {
                k_box_reduce<<<1, 1024, 0, st>>>(S->bres, 0, 0, 0, S->dbox + 4 * k);   // empty
            }
            RMT_LAUNCHED();
        }
        // box mode with contact: only the discs' boxes grown by 6 (MS_BLOCKS / K blocks each,
        // one J partial per block); otherwise the whole grid
        const bool sbox = D.bx.n > 0 && D.bx.contact;
        const dim3 sg = sbox ? dim3(MS_BLOCKS / K, K) : dim3(MS_BLOCKS);
        k_mac_stress<<<sg, MS_TPB, 0, st>>>(D, N, dx, dx, P.mu_s, w_t, P.eta, eps, S->Sxx,
                                            S->Sxy, S->Syy, S->part, 0, N, 0, N,
                                            stress_skip_ok(P), S->flags + 4, sbox);
        RMT_LAUNCHED();
        const int npart = (int)(sg.x * sg.y);
        double jr[2 * MS_BLOCKS];
        RMT_HIP(hipMemcpyAsync(jr, S->part, 2 * npart * sizeof(double), hipMemcpyDeviceToHost, st));
        k_mac_predict<<<grid1d(2 * nf, 256), 256, 0, st>>>(S->u, S->v, S->Sxx, S->Sxy, S->Syy,
                                                            nullptr, nullptr, N, nu, dx, dx, dx2,
                                                            dx2, dt, P.U_lid, P.rho, S->us, S->vs,
                                                            FaceRows{0, N, 0, N + 1}, D.bx);
        RMT_LAUNCHED();
        // max |u| from the correction's pass, folded on the device into out[9]
        RMT_TRY(mac_project_impl(ctx, S->us, S->vs, dx, dx, dt, P.rho, S->u, S->v, S->p,
                                 S->X1n, true, S->mpart, S->mpartv));
        k_max_partials<true><<<1, 1024, 0, st>>>(S->mpart, MP_BLOCKS, 0.0, S->out + 9);
        int dr0 = 0, dr1 = N;   // the rows holding every box
        if (D.bx.n) {
            dr0 = N; dr1 = 0;
            for (int k = 0; k < K; ++k)
                if (D.bx.b[k][1] > D.bx.b[k][0]) {
                    dr0 = std::min(dr0, D.bx.b[k][0]); dr1 = std::max(dr1, D.bx.b[k][1]);
                }
        }
        k_mac_diag<<<MS_BLOCKS, MS_TPB, 0, st>>>(D, nullptr, N, dx, S->part + 2 * MS_BLOCKS, 0, N,
                                                 dr0, dr1);
        RMT_LAUNCHED();
        std::vector<double> dp((size_t)MS_BLOCKS * MD_VALS);
        RMT_HIP(hipMemcpyAsync(dp.data(), S->part + 2 * MS_BLOCKS, dp.size() * 8,
                               hipMemcpyDeviceToHost, st));
        double um = 0.0;
        RMT_HIP(hipMemcpyAsync(&um, S->out + 9, sizeof(double), hipMemcpyDeviceToHost, st));
        int fl[4];
        RMT_HIP(hipMemcpyAsync(fl, S->flags, sizeof(fl), hipMemcpyDeviceToHost, st));
        if (box_mode)   // the next step's boxes, with the diagnostics
            RMT_HIP(hipMemcpyAsync(S->hbox, S->dbox, 4 * K * sizeof(int), hipMemcpyDeviceToHost, st));
        RMT_HIP(hipStreamSynchronize(st));
        RMT_CHECK(!fl[0] && !fl[1], RMT_ENONFINITE,
                  "advect_reference_map: non-finite velocity (the simulation diverged)");
        RMT_CHECK(!fl[3], RMT_EDEVICE, extrap_abort_detail(fl[3]));
        S->t += dt;
        rmt_mac_diag r{};
        r.t = S->t; r.dt = dt; r.n_discs = K;
        r.minJ = 1.0; r.maxJ = 1.0;
        for (int b = 0; b < npart; ++b) {
            r.minJ = std::fmin(r.minJ, jr[2 * b]); r.maxJ = std::fmax(r.maxJ, jr[2 * b + 1]);
        }
        double acc[MD_VALS] = {0};
        for (int b = 0; b < MS_BLOCKS; ++b)
            for (int k = 0; k < MD_VALS; ++k) {
                const double x = dp[(size_t)b * MD_VALS + k];
                acc[k] = k == 3 * MAC_MAXD ? nanmax(acc[k], x) : acc[k] + x;
            }
        for (int k = 0; k < K; ++k) {
            r.cx[k] = acc[3 * k + 2] > 0 ? acc[3 * k] / acc[3 * k + 2] : NAN;
            r.cy[k] = acc[3 * k + 2] > 0 ? acc[3 * k + 1] / acc[3 * k + 2] : NAN;
        }
        acc[3 * MAC_MAXD] = nanmax(acc[3 * MAC_MAXD], um);
        r.umax = acc[3 * MAC_MAXD];
        // mac_multi_disc_lid.py:100-103: the driver stops on a non-finite u, a folded (J < 0)
        // or over-stretched (J > 20) map, or a disc with no phi <= 0 cell left
        bool lost = false;
        for (int k = 0; k < K; ++k) lost |= !(acc[3 * k + 2] > 0);
        r.diverged = !std::isfinite(r.umax) || r.minJ < 0.0 || r.maxJ > 20.0 || lost;
        S->diag.push_back(r);
        if (r.diverged) { S->diverged = true; break; }
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

// ------------------------------------------------------------ MAC slabs (config 5) --
// rmt_mac_sim's step decomposed into row slabs, as rmt_slab (slab.hip) decomposes the
// cell-centred step.  Slab `rank` owns cell rows [r0, r1), u face rows [r0, r1) and v face
// rows [r0, r1] (the face row r1 is computed by both neighbours, from the same inputs), and
// keeps RMT_SLAB_HALO rows on either side resident.  Planes are addressed with GLOBAL
// indices (pointer - lo * row length) so every kernel above runs unchanged on a row range.
// Phases (collectives between them: pyrmt_amd/distributed.py, MacDistributedSim):
//   halo(u, v, X1_k, X2_k)
//   advect        centres on the resident rows; per disc SL-RK4 on rows r0-3 .. r1+3 and
//                 the known bits of the owned rows
//   allgather(bits_k); rim_pack (all discs); allgather(scalars); allgather(rim_k)
//   extrapolate   per disc: dense replica, exact extrapolation, rim write-back, phi rebuilt
//   predict       stress on rows r0-2 .. r1+2 (J range of the owned rows), predictor,
//                 rhs of the owned rows and its row-tree root
//   allgather(roots); project_rows (mean removed, DCT-II along x, column blocks packed)
//   all_to_all; project_cols (DCT-II solve along y of the column block); all_to_all
//   project_unrows (inverse DCT-II along x into p)
//   halo(p, 1 row); correct (+ diagnostics partials -> scalar block); allgather(scalars)
// With every slab holding 2^m rows at a multiple of 2^m the fields are bit-identical to
// rmt_mac_sim's (the row-tree mean); the centroid sums differ in summation order only.
namespace rmt {
constexpr int MSL_MAXG = 64;
enum { MS_FLAGS = 0, MS_JMIN = 1, MS_JMAX = 2, MS_UMAX = 3, MS_CEN = 4,
       MS_COUNT = MS_CEN + 3 * MAC_MAXD, MS_ROOT = MS_COUNT + MAC_MAXD, MS_FIT = MS_ROOT + 1,
       MS_ANY = MS_FIT + 1, MS_N = MS_ANY + MAC_MAXD + 2 };
static_assert(MS_N == RMT_MAC_SLAB_SCALARS, "rmt.h scalar block size");

// J range and diagnostics partials -> the scalar block; flags folded in
__global__ void __launch_bounds__(256) k_mac_slab_scal(const double *__restrict__ part,
                                                       const int *__restrict__ flags, int K,
                                                       double *__restrict__ scal) {
    __shared__ double s[256];
    const int t = threadIdx.x;
    const double *dp = part + 2 * MS_BLOCKS;
    for (int v = 0; v < 2 + 3 * K + 1; ++v) {
        // v: 0 J min, 1 J max, 2 .. 2+3K centroid sums, last max|u|
        const int kind = v == 0 ? 0 : (v == 1 || v == 2 + 3 * K) ? 1 : 2;
        double a = kind == 2 ? 0.0 : (kind == 0 ? 1.0 : (v == 1 ? 1.0 : 0.0));
        for (int b = t; b < MS_BLOCKS; b += 256) {
            const double x = v == 0 ? part[2 * b] : v == 1 ? part[2 * b + 1]
                           : v == 2 + 3 * K ? dp[(long)b * MD_VALS + 3 * MAC_MAXD]
                                            : dp[(long)b * MD_VALS + (v - 2)];
            a = kind == 0 ? fmin(a, x) : kind == 1 ? (v == 1 ? fmax(a, x) : nanmax(a, x)) : a + x;
        }
        s[t] = a;
        __syncthreads();
        for (int w = 128; w > 0; w >>= 1) {
            if (t < w) {
                const double x = s[t + w];
                s[t] = kind == 0 ? fmin(s[t], x)
                     : kind == 1 ? (v == 1 ? fmax(s[t], x) : nanmax(s[t], x)) : s[t] + x;
            }
            __syncthreads();
        }
        if (t == 0) {
            const int o = v == 0 ? MS_JMIN : v == 1 ? MS_JMAX : v == 2 + 3 * K ? MS_UMAX
                                                                               : MS_CEN + v - 2;
            scal[o] = s[0];
        }
        __syncthreads();
    }
    if (t == 0) {
        int fl = flags[0], fit = 0;
        for (int k = 0; k < K; ++k) { fit += flags[4 + 2 * k]; fl |= flags[5 + 2 * k] ? 4 : 0; }
        scal[MS_FLAGS] = (double)fl;
        scal[MS_FIT] = (double)fit;
    }
}
// per disc: did the no-op test on the owned rows find an acceptable target?
__global__ void k_mac_slab_any(const int *__restrict__ nctl, int K, double *__restrict__ scal) {
    const int k = threadIdx.x;
    if (k < K) scal[MS_ANY + k] = (double)nctl[k * EXC_WORDS + EXC_ANY];
}
}  // namespace rmt

struct rmt_mac_slab {
    rmt_ctx *ctx = nullptr;
    rmt_mac_params P{};
    int G = 1, rank = 0, N = 0, W = 0, r0 = 0, r1 = 0, lo = 0, hi = 0, c0 = 0, c1 = 0;
    int rs[rmt::MSL_MAXG + 1], cs[rmt::MSL_MAXG + 1];
    void *block = nullptr;
    double *u, *us;            // (hi - lo) x (N + 1)
    double *v, *vs;            // (hi - lo + 1) x N: face rows lo .. hi
    double *p, *uc, *vc, *Sxx, *Sxy, *Syy;
    double *X1[RMT_MAC_MAXD], *X2[RMT_MAC_MAXD], *phi[RMT_MAC_MAXD];
    double *X1n[RMT_MAC_MAXD], *X2n[RMT_MAC_MAXD], *phi_pre[RMT_MAC_MAXD];
    double *X1d, *X2d;         // dense N x N extrapolation replica (shared by the discs)
    u64 *bits[RMT_MAC_MAXD];   // N x W known planes
    u64 *rimw;
    int *rowcnt;
    double *rim[RMT_MAC_MAXD]; // 3 doubles per owned cell
    double *rhs, *A, *Y, *B, *T, *xs, *scal, *part;
    int *flags;                // [0] flags, [4 + 2k, 5 + 2k] disc k {fitted, aborted}
    int *nctl;                 // K x EXC_WORDS: k_ex_none control words of each disc
    double *gc(double *q) const { return q - (long)lo * N; }         // cells, v faces
    double *gu(double *q) const { return q - (long)lo * (N + 1); }   // u faces
    rmt::DiscSet discs() const {
        rmt::DiscSet D{};
        D.K = P.n_discs;
        for (int k = 0; k < D.K; ++k) {
            D.X1[k] = X1[k] - (long)lo * N; D.X2[k] = X2[k] - (long)lo * N;
            D.phi[k] = phi[k] - (long)lo * N;
        }
        return D;
    }
};

extern "C" {

int rmt_mac_slab_create(rmt_ctx *ctx, const rmt_mac_params *prm, int G, int rank,
                        const int *row_splits, const int *col_splits, rmt_mac_slab **out) {
    RMT_CHECK(ctx && prm && row_splits && col_splits && out, RMT_EINVAL, "null argument");
    RMT_CHECK(G >= 1 && G <= MSL_MAXG && rank >= 0 && rank < G, RMT_EINVAL, "slab: bad G/rank");
    RMT_CHECK(prm->n_discs >= 1 && prm->n_discs <= RMT_MAC_MAXD, RMT_EINVAL, "1..8 discs");
    RMT_CHECK(prm->N >= 4 && prm->N <= 32768, RMT_EINVAL, "N in 4..32768 (32-bit face indices)");
    const int N = prm->N;
    RMT_CHECK(ctx->nx == N && ctx->ny == N, RMT_EINVAL, "slab: ctx must be the global N x N");
    RMT_CHECK(N <= 8192, RMT_ENOTSUP, "MAC slab step: N <= 8192");
    for (int k = 0; k < G; ++k) {
        RMT_CHECK(row_splits[k + 1] - row_splits[k] >= RMT_SLAB_HALO + 1 && !(row_splits[k] & 1),
                  RMT_EINVAL, "slab: row splits must be even, > RMT_SLAB_HALO rows each");
        RMT_CHECK(col_splits[k + 1] - col_splits[k] >= 2 && !(col_splits[k] & 1), RMT_EINVAL,
                  "slab: column splits must be even, >= 2 columns each");
    }
    RMT_CHECK(row_splits[0] == 0 && row_splits[G] == N && col_splits[0] == 0 &&
                  col_splits[G] == N, RMT_EINVAL, "slab: splits must cover 0 .. N");
    RMT_TRY(dct2_plan(ctx, N, N, prm->dx, prm->dx));
    rmt_mac_slab *S = new rmt_mac_slab;
    S->ctx = ctx; S->P = *prm; S->G = G; S->rank = rank; S->N = N; S->W = (N + 63) / 64;
    for (int k = 0; k <= G; ++k) { S->rs[k] = row_splits[k]; S->cs[k] = col_splits[k]; }
    S->r0 = row_splits[rank]; S->r1 = row_splits[rank + 1];
    S->c0 = col_splits[rank]; S->c1 = col_splits[rank + 1];
    S->lo = std::max(0, S->r0 - RMT_SLAB_HALO); S->hi = std::min(N, S->r1 + RMT_SLAB_HALO);
    const int K = prm->n_discs, rows = S->r1 - S->r0;
    const long nl = (long)(S->hi - S->lo) * N, nu = (long)(S->hi - S->lo) * (N + 1);
    const long nv = (long)(S->hi - S->lo + 1) * N, no = (long)rows * N, nd = (long)N * N;
    const long nc = S->c1 - S->c0, W = S->W;
    const size_t dbl = 2 * nu + 2 * nv + 6 * nl + 6 * K * nl + 2 * nd + 3 * K * no + 3 * no +
                       2 * nc * N + N + MS_N + (2 + MD_VALS) * MS_BLOCKS + 16;
    const size_t bytes = dbl * 8 + (size_t)(K * N + rows) * W * 8 + (rows + 64) * 4 +
                         (size_t)K * EXC_WORDS * 4 + 256;
    RMT_HIP(hipMalloc(&S->block, bytes));
    RMT_HIP(hipMemsetAsync(S->block, 0, bytes, ctx->stream));
    double *q = (double *)S->block;
    S->u = q; q += nu; S->us = q; q += nu;
    S->v = q; q += nv; S->vs = q; q += nv;
    double **pl[] = {&S->p, &S->uc, &S->vc, &S->Sxx, &S->Sxy, &S->Syy};
    for (auto pp : pl) { *pp = q; q += nl; }
    for (int k = 0; k < K; ++k) {
        double **dk[] = {&S->X1[k], &S->X2[k], &S->phi[k], &S->X1n[k], &S->X2n[k],
                         &S->phi_pre[k]};
        for (auto pp : dk) { *pp = q; q += nl; }
    }
    S->X1d = q; q += nd;
    S->X2d = q; q += nd;
    for (int k = 0; k < K; ++k) { S->rim[k] = q; q += 3 * no; }
    S->rhs = q; q += no;
    S->A = q; q += no;
    S->Y = q; q += no;
    S->B = q; q += nc * N;
    S->T = q; q += nc * N;
    S->xs = q; q += N;
    S->scal = q; q += MS_N;
    S->part = q; q += (2 + MD_VALS) * MS_BLOCKS + 16;
    u64 *b = (u64 *)q;
    for (int k = 0; k < K; ++k) { S->bits[k] = b; b += (long)N * W; }
    S->rimw = b; b += (long)rows * W;
    S->rowcnt = (int *)b;
    S->flags = S->rowcnt + rows + 32;
    S->nctl = S->flags + 32;
    std::vector<double> g(N);
    for (int i = 0; i < N; ++i) g[i] = i * prm->dx;   // mac_multi_disc_lid.py:41
    RMT_HIP(hipMemcpyAsync(S->xs, g.data(), N * 8, hipMemcpyHostToDevice, ctx->stream));
    RMT_TRY(ensure_bytes(ctx, extrap_workspace(N, N, prm->layers)));
    RMT_HIP(hipStreamSynchronize(ctx->stream));
    *out = S;
    return RMT_OK;
}

int rmt_mac_slab_destroy(rmt_mac_slab *S) {
    if (!S) return RMT_OK;
    (void)hipFree(S->block);
    delete S;
    return RMT_OK;
}

int rmt_mac_slab_info(rmt_mac_slab *S, int *ints8) {
    RMT_CHECK(S && ints8, RMT_EINVAL, "null argument");
    const int v[8] = {S->r0, S->r1, S->lo, S->hi, S->c0, S->c1, S->W, RMT_SLAB_HALO};
    for (int k = 0; k < 8; ++k) ints8[k] = v[k];
    return RMT_OK;
}

int rmt_mac_slab_buffer(rmt_mac_slab *S, int id, int disc, void **ptr) {
    RMT_CHECK(S && ptr, RMT_EINVAL, "null argument");
    const bool per_disc = id == 3 || id == 4 || id == 5 || id == 6 || id == 7;
    RMT_CHECK(id >= 0 && id <= 10 && (!per_disc || (disc >= 0 && disc < S->P.n_discs)),
              RMT_EINVAL, "unknown buffer id / disc");
    void *b[] = {S->u, S->v, S->p, per_disc ? S->X1[disc] : nullptr,
                 per_disc ? S->X2[disc] : nullptr, per_disc ? S->phi[disc] : nullptr,
                 per_disc ? (void *)S->bits[disc] : nullptr, per_disc ? S->rim[disc] : nullptr,
                 S->A, S->B, S->scal};
    *ptr = b[id];
    return RMT_OK;
}

int rmt_mac_slab_advect(rmt_mac_slab *S, double dt) {
    RMT_CHECK(S, RMT_EINVAL, "null slab");
    rmt_ctx *ctx = S->ctx;
    const rmt_mac_params &P = S->P;
    const int N = S->N;
    RMT_HIP(hipMemsetAsync(S->flags, 0, (32 + P.n_discs * EXC_WORDS) * sizeof(int), ctx->stream));
    k_mac_centres<<<grid1d((long)(S->hi - S->lo) * N, 256), 256, 0, ctx->stream>>>(
        S->gu(S->u), S->gc(S->v), N, S->gc(S->uc), S->gc(S->vc), S->flags, S->lo, S->hi);
    RMT_LAUNCHED();
    const int jb = std::max(0, S->r0 - 3), je = std::min(N, S->r1 + 3);
    RMT_TRY(reduce_maxsq2_nan(ctx, S->uc, S->vc, (long)(S->hi - S->lo) * N, S->scal + MS_N - 1));
    for (int k = 0; k < P.n_discs; ++k) {
        RMT_TRY(slab_sl(ctx, S->gc(S->X1[k]), S->gc(S->X2[k]), S->gc(S->uc), S->gc(S->vc), S->xs,
                        S->xs, N, N, dt, P.dx, P.dx, P.cx[k], P.cy[k], P.R[k], S->gc(S->X1n[k]),
                        S->gc(S->X2n[k]), S->gc(S->phi_pre[k]), S->flags, jb, je, S->lo, S->hi,
                        S->scal + MS_N - 1));
        RMT_TRY(slab_bits(ctx, S->gc(S->phi_pre[k]), N, S->W, S->bits[k], S->r0, S->r1));
    }
    return RMT_OK;
}

int rmt_mac_slab_rim_pack(rmt_mac_slab *S) {
    RMT_CHECK(S, RMT_EINVAL, "null slab");
    const int K = S->P.n_discs;
    for (int k = 0; k < K; ++k) {
        RMT_TRY(slab_rim_pack(S->ctx, S->bits[k], S->N, S->N, S->W, S->r0, S->r1, S->rimw,
                              S->rowcnt, S->gc(S->X1n[k]), S->gc(S->X2n[k]), S->rim[k],
                              S->scal + MS_COUNT + k));
        // k_ex_none's exact no-op test, candidates split by rows: if no slab finds an
        // acceptable first-layer target the extrapolation of disc k is the identity
        RMT_TRY(extrap_none_rows(S->ctx, S->bits[k], S->N, S->N, S->P.dx, S->P.dx, S->r0, S->r1,
                                 S->nctl + k * EXC_WORDS));
    }
    k_mac_slab_any<<<1, 64, 0, S->ctx->stream>>>(S->nctl, K, S->scal);
    RMT_LAUNCHED();
    return RMT_OK;
}

// disc k proven a no-op on every slab (scalar MS_ANY + k zero everywhere): keep the
// advected map, rebuild phi -- what rmt_mac_slab_extrapolate computes then, without the
// rim allgather and the dense replica
int rmt_mac_slab_extrapolate_identity(rmt_mac_slab *S, int disc) {
    RMT_CHECK(S && disc >= 0 && disc < S->P.n_discs, RMT_EINVAL, "bad argument");
    const rmt_mac_params &P = S->P;
    const int N = S->N, k = disc;
    const int jb = std::max(0, S->r0 - 3), je = std::min(N, S->r1 + 3);
    const long o = (long)jb * N, n = (long)(je - jb) * N;
    k_mac_phi<<<grid1d(n, 256), 256, 0, S->ctx->stream>>>(
        S->gc(S->X1n[k]) + o, S->gc(S->X2n[k]) + o, n, P.cx[k], P.cy[k], P.R[k],
        S->gc(S->X1[k]) + o, S->gc(S->X2[k]) + o, S->gc(S->phi[k]) + o);
    RMT_LAUNCHED();
    return RMT_OK;
}

int rmt_mac_slab_extrapolate(rmt_mac_slab *S, int disc, const double *gathered,
                             const long long *counts, long long cap) {
    RMT_CHECK(S && counts && (gathered || cap == 0) && disc >= 0 && disc < S->P.n_discs,
              RMT_EINVAL, "bad argument");
    rmt_ctx *ctx = S->ctx;
    const rmt_mac_params &P = S->P;
    const int N = S->N, k = disc;
    RMT_TRY(slab_rim_extrapolate(ctx, gathered, counts, S->G, cap, S->X1d, S->X2d, S->bits[k],
                                 P.dx, P.dx, P.layers, S->flags + 4 + 2 * k, S->gc(S->X1n[k]),
                                 S->gc(S->X2n[k]), (long)S->lo * N, (long)S->hi * N));
    const int jb = std::max(0, S->r0 - 3), je = std::min(N, S->r1 + 3);
    const long o = (long)jb * N, n = (long)(je - jb) * N;
    k_mac_phi<<<grid1d(n, 256), 256, 0, ctx->stream>>>(
        S->gc(S->X1n[k]) + o, S->gc(S->X2n[k]) + o, n, P.cx[k], P.cy[k], P.R[k],
        S->gc(S->X1[k]) + o, S->gc(S->X2[k]) + o, S->gc(S->phi[k]) + o);
    RMT_LAUNCHED();
    return RMT_OK;
}

int rmt_mac_slab_predict(rmt_mac_slab *S, double dt) {
    RMT_CHECK(S, RMT_EINVAL, "null slab");
    rmt_ctx *ctx = S->ctx;
    const rmt_mac_params &P = S->P;
    const int N = S->N, rows = S->r1 - S->r0;
    const double dx = P.dx, w_t = 2.0 * dx, eps = 3.0 * dx, nu = P.mu_f / P.rho;
    const double dx2 = std::pow(dx, 2.0);
    const DiscSet D = S->discs();
    k_mac_stress<<<MS_BLOCKS, MS_TPB, 0, ctx->stream>>>(
        D, N, dx, dx, P.mu_s, w_t, P.eta, eps, S->gc(S->Sxx), S->gc(S->Sxy), S->gc(S->Syy),
        S->part, std::max(0, S->r0 - 2), std::min(N, S->r1 + 2), S->r0, S->r1,
        stress_skip_ok(P));
    RMT_LAUNCHED();
    const FaceRows F{S->r0, S->r1, S->r0, std::min(S->r1 + 1, N + 1)};
    k_mac_predict<<<grid1d(face_count(F, N), 256), 256, 0, ctx->stream>>>(
        S->gu(S->u), S->gc(S->v), S->gc(S->Sxx), S->gc(S->Sxy), S->gc(S->Syy), nullptr, nullptr,
        N, nu, dx, dx, dx2, dx2, dt, P.U_lid, P.rho, S->gu(S->us), S->gc(S->vs), F);
    RMT_LAUNCHED();
    double *rhs_g = S->rhs - (long)S->r0 * N;
    k_mac_rhs<<<grid1d((long)rows * N, 256), 256, 0, ctx->stream>>>(
        S->gu(S->us), S->gc(S->vs), N, dx, dx, P.rho / dt, rhs_g, S->r0, S->r1);
    RMT_LAUNCHED();
    return rowtree_root(ctx, S->rhs, rows, N, S->scal + MS_ROOT);
}

int rmt_mac_slab_project_rows(rmt_mac_slab *S, const double *roots) {
    RMT_CHECK(S && roots, RMT_EINVAL, "null argument");
    rmt_ctx *ctx = S->ctx;
    const int N = S->N, rows = S->r1 - S->r0;
    RMT_TRY(sub_tree_mean(ctx, S->rhs, (long)rows * N, roots, S->G, (double)N * N));
    RMT_TRY(dct2_plan(ctx, N, N, S->P.dx, S->P.dx));
    RMT_TRY(dct2_pass(ctx, 0, 0, S->rhs, S->Y, rows, 0));
    return slab_cols(ctx, true, S->Y, rows, N, S->cs, S->G, S->A);
}

int rmt_mac_slab_project_cols(rmt_mac_slab *S) {
    RMT_CHECK(S, RMT_EINVAL, "null slab");
    rmt_ctx *ctx = S->ctx;
    const int nc = S->c1 - S->c0;
    transpose(ctx, ctx->stream, S->B, S->N, nc, S->T);
    RMT_TRY(dct2_pass(ctx, 1, 1, S->T, S->T, nc, S->c0));
    transpose(ctx, ctx->stream, S->T, nc, S->N, S->B);
    RMT_LAUNCHED();
    return RMT_OK;
}

int rmt_mac_slab_project_unrows(rmt_mac_slab *S) {
    RMT_CHECK(S, RMT_EINVAL, "null slab");
    rmt_ctx *ctx = S->ctx;
    const int N = S->N, rows = S->r1 - S->r0;
    RMT_TRY(slab_cols(ctx, false, S->Y, rows, N, S->cs, S->G, S->A));
    return dct2_pass(ctx, 2, 0, S->Y, S->gc(S->p) + (long)S->r0 * N, rows, 0);
}

int rmt_mac_slab_correct(rmt_mac_slab *S, double dt) {
    RMT_CHECK(S, RMT_EINVAL, "null slab");
    rmt_ctx *ctx = S->ctx;
    const rmt_mac_params &P = S->P;
    const int N = S->N;
    const FaceRows F{S->r0, S->r1, S->r0, std::min(S->r1 + 1, N + 1)};
    k_mac_correct<<<grid1d(face_count(F, N), 256), 256, 0, ctx->stream>>>(
        S->gu(S->us), S->gc(S->vs), S->gc(S->p), N, P.dx, P.dx, dt / P.rho, S->gu(S->u),
        S->gc(S->v), F);
    RMT_LAUNCHED();
    k_mac_diag<<<MS_BLOCKS, MS_TPB, 0, ctx->stream>>>(S->discs(), S->gu(S->u), N, P.dx,
                                                     S->part + 2 * MS_BLOCKS, S->r0, S->r1, S->r0, S->r1);
    RMT_LAUNCHED();
    k_mac_slab_scal<<<1, 256, 0, ctx->stream>>>(S->part, S->flags, P.n_discs, S->scal);
    RMT_LAUNCHED();
    return RMT_OK;
}

}  // extern "C"
