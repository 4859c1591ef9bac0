// rmt_internal.hpp -- shared state and per-cell device arithmetic of librmt.
//
// Every __device__ formula below keeps the reference's floating-point operation order
// (Python evaluates left to right; `c * x * y` is `(c*x)*y`) and is compiled with
// -ffp-contract=off, so kernels built from them reproduce the CPU reference bit for bit
// wherever no transcendental function or FFT is involved.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <rocfft/rocfft.h>
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <string>
#include "../../include/rmt.h"
#include "divk.hpp"

namespace rmt {

// Workgroups of a launch over a device-side tile list (count on the device): kernels loop
// b = blockIdx.x, b + gridDim.x, ... < *count; a fix-up list is a few hundred tiles, and a
// launch of max_tiles mostly-empty workgroups costs its dispatch.
constexpr int LIST_BLOCKS = 1024;
extern int g_list_blocks;   // RMT_LIST_BLOCKS (A/B of the list launches' grid; ops.hip)
inline unsigned list_grid(long max_tiles) {
    return (unsigned)std::max(1L, std::min<long>(max_tiles, g_list_blocks));
}

// NaN-propagating max (a NaN operand wins; fmax would drop it)
__host__ __device__ __forceinline__ double nanmax(double a, double b) {
    return (a != a || b != b) ? (a + b) : (a > b ? a : b);
}


// ---------------------------------------------------------------- error plumbing --
void set_error(const std::string &msg);
#define RMT_HIP(call)                                                                   \
    do {                                                                                \
        hipError_t e_ = (call);                                                         \
        if (e_ != hipSuccess) {                                                         \
            ::rmt::set_error(std::string(#call) + ": " + hipGetErrorString(e_));        \
            return RMT_EDEVICE;                                                         \
        }                                                                               \
    } while (0)
// after a launch: report the failing host line (file:line names the kernel launched above)
#define RMT_LAUNCHED()                                                                  \
    do {                                                                                \
        hipError_t e_ = hipGetLastError();                                              \
        if (e_ != hipSuccess) {                                                         \
            ::rmt::set_error(std::string(__FILE__) + ":" + std::to_string(__LINE__) +   \
                             " launch: " + hipGetErrorString(e_));                      \
            return RMT_EDEVICE;                                                         \
        }                                                                               \
    } while (0)
#define RMT_CHECK(cond, code, msg)                                                      \
    do {                                                                                \
        if (!(cond)) { ::rmt::set_error(msg); return (code); }                          \
    } while (0)
// Host -> device upload of a table that kernels on any of the context's streams read: a
// plain hipMemcpy from pageable memory may return once the data is staged, before its DMA
// lands, and kernels on non-blocking streams are not ordered after it -- so drain the device.
#define RMT_UPLOAD(dst, src, bytes)                                                     \
    do {                                                                                \
        RMT_HIP(hipMemcpy((dst), (src), (bytes), hipMemcpyHostToDevice));               \
        RMT_HIP(hipDeviceSynchronize());                                                \
    } while (0)
#define RMT_TRY(expr)                                                                   \
    do { int s_ = (expr); if (s_ != RMT_OK) return s_; } while (0)

struct DctPlan;   // poisson.hip (DCT-I, collocated grid)
struct Dct2Plan;  // poisson.hip (DCT-II, MAC grid)
struct PerPlan;   // periodic.hip (reduced-grid 2D FFT)

}  // namespace rmt

// Per-context implementation switches: bit-identical alternatives of the schedule and the
// kernels (A/B measurements, regression tests).  Every field starts from its environment
// variable at rmt_ctx_create (defaults below when unset) and can be changed per context with
// rmt_ctx_set_option(ctx, name, value) (ops.hip: the name table).
struct rmt_opts {
    int ext_events = 1;       // RMT_EXT_EVENTS: cross-stream events complete with their kernel
    int ex_arena_bump = 0;    // RMT_EX_ARENA=bump: record arena by bump allocation
    int ex_profile = 0;       // RMT_EX_PROFILE: the chain's per-phase clocks (diagnostic)
    int fix_all = 0;          // RMT_FIX_ALL: the fix-up lists every tile (regression switch)
    int dct_rocfft = 0;       // RMT_DCT_ROCFFT: rocFFT for every DCT length
    int transpose2 = 1;       // RMT_TRANSPOSE2: 16-byte transposes
    int sim_hiprio = 1;       // RMT_SIM_HIPRIO: the step's internal stream at the highest priority
    int sim_sync = 0;         // RMT_SIM_SYNC: the synchronous step path
    int early_geometry = 1;   // RMT_EARLY_GEOMETRY
    int early_transpose = 1;  // RMT_EARLY_TRANSPOSE
    int fused_fluid = 1;      // RMT_FUSED_FLUID
    int no_overlap = 0;       // RMT_NO_OVERLAP: no second stream
    int side_tail = 1;        // RMT_SIDE_TAIL
    int par_overlap = 1;      // RMT_PAR_OVERLAP
    int fused_fixprep = 1;    // RMT_FUSED_FIXPREP
    int merged_join = 1;      // RMT_MERGED_JOIN
    int test_delay_side = 0;  // RMT_TEST_DELAY_SIDE: sleep units on the second stream (tests)
    int test_delay_main = 0;  // RMT_TEST_DELAY_MAIN: ... on the main stream (tests)
    int test_delay_geo = 0;   // RMT_TEST_DELAY_GEO: ... ahead of a slab's early geometry (tests)
    int test_nowait_drop = 0; // RMT_TEST_NOWAIT_DROP: a dropped slab geometry is not waited for
                              // (the pre-fix behaviour, to show the hazard the wait removes)
    int ch_cols = 2;          // RMT_CH_PARTS: chain workgroups per layer group (column ranges)
    int ch_lgroups = 0;       // RMT_CH_LAYERS: chain layer groups (0: one per layer)
    int edge_slots = 64;      // RMT_EDGE_SLOTS_USED: edge-tile lists kept (1..64; fewer evict)
    int edge_stream = 1;      // RMT_EDGE_STREAM: a full stage's edge tiles beside its interior
    int sl_phi = 1;           // RMT_SL_PHI: the side stream's SL pass also writes phi + fluid bits
    int mac_boxes = 1;        // RMT_MAC_BOXES: config 5's per-disc passes on the map's support box
    int skip_marked_rows = 1; // RMT_SKIP_MARKED_ROWS: the speculative row DCT leaves out the rows
                              // the fix-up transforms again
    int tail_stream = 1;      // RMT_TAIL_STREAM: the pressure update beside the SL and prep
    int diag_first = 0;       // RMT_DIAG_FIRST: the step's diagnostics ahead of the next geometry
    int mac_noop_host = 1;    // RMT_MAC_NOOP_HOST: MAC extrapolation's no-op verdict read on the host
    int mac_face_sl = 1;      // RMT_MAC_FACE_SL: MAC advection samples the face planes (no centre planes)
    int mac_m2_bound = 1;     // RMT_MAC_M2_BOUND: MAC SL bound from the last correction's face maxima
    int diag_seg = 1;         // RMT_DIAG_SEG: the step's diagnostics read only the segments that
                              // can hold a solid cell or J != 1 (k_diag_seg)
    int dct_desc = 1;         // RMT_DCT_DESC: n = 4096 DCT-I plan 13, 9, 7, 5 (fft_4095d;
                              // 0: 5, 7, 9, 13, fft_4095)
    int sl_zero_flags = 1;    // RMT_SL_ZERO_FLAGS: the side SL pass skips the loads and stores of
                              // tiles whose map stays +0.0 (zero-tile flags, k_sim_sl_t)
};

#define RMT_EDGE_PRIOS 2   // edge-tile streams kept, one per priority (momentum.hip edge_stream)
#ifndef RMT_EDGE_SLOTS
#define RMT_EDGE_SLOTS 64   // >= every (window, grid) key of a step: 8 slabs x 4 stages + the fused 4
#endif
struct rmt_ctx {
    int ny = 0, nx = 0, device = 0;
    hipStream_t stream = nullptr;
    // scratch (grown on demand, owned)
    double *scratch = nullptr;
    size_t scratch_bytes = 0;
    double *red = nullptr;      // reduction partials (host-visible results copied out)
    double *rsum = nullptr;     // per-row sums of the row-tree reductions
    int rsum_len = 0;
    unsigned char *bytes = nullptr;
    size_t bytes_len = 0;
    unsigned long bytes_gen = 0;   // bumped by every ensure_bytes (a user of the workspace)
    rmt::DctPlan *dct = nullptr;
    rmt::Dct2Plan *dct2 = nullptr;
    rmt::PerPlan *per = nullptr;
    // optional kernel timers (rmt_sim profiling): [0,1] around the four RK4 stage kernels,
    // [2,3] around the extrapolation sweep kernel
    bool prof = false;
    int ex_layers = 0;          // last extrapolation call (rmt_extrap_last_path)
    bool ex_chain = false;
    bool ex_par = false;        // the last geometry laid out the parallel mode (extrap_par.hip)
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    // optional (sim.hip overlap): recorded on the stream right before the extrapolation's
    // serial chain kernel starts (or after the call when no chain kernel runs)
    hipEvent_t ev_chain = nullptr;
    // optional (sim.hip overlap): extrap_finish leaves the fallback sweep (an early exit unless
    // a chain capacity limit tripped) to the caller, who runs extrap_sweep on another stream
    // after ev_chain, beside the chain instead of ahead of it
    bool ex_sweep_defer = false;
    // optional (sim.hip overlap, with ex_sweep_defer): ev_chain tracks the completion of the
    // values pass right before the chain (launch_done) instead of a record of its own
    bool ev_chain_vals = false;
    // optional (mac.hip: the extrapolation on the critical stream, where the no-op test finds
    // nothing to fit as often as not): k_ex_none on a wave per row instead of 64 workgroups
    bool ex_none_wide = false;
    // optional (mac.hip box mode): the rows [ex_none_rows[0], ex_none_rows[1]) hold every
    // candidate target (the known plane is zero outside them); je <= jb: every row
    int ex_none_rows[2] = {0, 0};
    int ex_none_cols[2] = {0, 0};   // (and the 64-column words [c0, c1) of those rows)
    // optional (mac.hip): a candidate list of ex_cand_cap cells + its counter, for the
    // no-op test's fit-per-wave form (k_ex_cand / k_ex_none_list) under ex_none_wide
    int *ex_cand = nullptr;
    int ex_cand_cap = 0;
    // optional (mac.hip): read the no-op test's verdict back on the host, and when no target
    // can be accepted skip the rest of the call's launches (the identity: ex_noop_skip)
    bool ex_none_host = false, ex_noop_skip = false;
    // momentum.hip: the stage tiles a full launch's interior kernel skips, per row window
    struct EdgeTiles { int *list = nullptr; int n = 0; long key[6] = {}; };
    EdgeTiles edge[RMT_EDGE_SLOTS];
    int edge_next = 0;
    // momentum.hip (opt.edge_stream): the stream the edge-tile launches of the full-grid stages
    // run on, beside the interior launch, at the priority of the stream it serves; events:
    // [0] the stage inputs ready, [1 + s] interior stage s done, [5 + s] edge stage s done
    hipStream_t edge_sts[RMT_EDGE_PRIOS] = {};   // one per stream priority served
    int edge_prios[RMT_EDGE_PRIOS] = {};
    hipEvent_t edge_ev[9] = {};
    void *imex[2] = {nullptr, nullptr};   // imex.hip: the DST preconditioner plans (u, v)
    rmt_opts opt;   // implementation switches (above)
};
static_assert(sizeof(((rmt_ctx *)nullptr)->edge) / sizeof(rmt_ctx::EdgeTiles) == RMT_EDGE_SLOTS, "edge slots");

namespace rmt {

int ensure_scratch(rmt_ctx *ctx, size_t bytes);    // >= bytes of double scratch
int ensure_bytes(rmt_ctx *ctx, size_t bytes);      // >= bytes of byte scratch
inline unsigned grid1d(long n, int block) { return (unsigned)((n + block - 1) / block); }

// A launch whose completion also completes `done` (hipExtLaunchKernel's stop event tracks the
// kernel itself: no marker packet between it and the stream's next launch -- an event record
// there costs the in-order stream ~6-8 us of command-processor time).  RMT_EXT_EVENTS=0: the
// launch, then a plain record.  done null: a plain launch.
template <typename... Formals, typename... Actuals>
inline hipError_t launch_done(const rmt_ctx *ctx, void (*k)(Formals...), dim3 g, dim3 b,
                              uint32_t lds, hipStream_t s, hipEvent_t done, Actuals... a) {
    if (done && ctx->opt.ext_events) {
        hipExtLaunchKernelGGL(k, g, b, lds, s, nullptr, done, 0, a...);
        return hipGetLastError();
    }
    hipExtLaunchKernelGGL(k, g, b, lds, s, nullptr, nullptr, 0, a...);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess && done) e = hipEventRecord(done, s);
    return e;
}

// ------------------------------------------------------------- device arithmetic --
// utils.py:4-25: second-order gradient along a line of length n (stride s) at index k;
// f points at element k itself (works on global rows/columns and on LDS tiles).
__device__ __forceinline__ double grad2(const double *f, long s, int k, int n, double h2) {
    if (k == 0) return (-3 * f[0] + 4 * f[s] - f[2 * s]) / h2;
    if (k == n - 1) return (3 * f[0] - 4 * f[-s] + f[-2 * s]) / h2;
    return (f[s] - f[-s]) / h2;
}

// utils.py:61-114 diff_upwind_3rd along a line; f points at element k.
__device__ __forceinline__ double upwind3(const double *f, long s, int k, int n, double vel,
                                          double h) {
    if (k >= 2 && k < n - 2) {
        if (vel > 0) return (2 * f[s] + 3 * f[0] - 6 * f[-s] + f[-2 * s]) / (6 * h);
        return (-f[2 * s] + 6 * f[s] - 3 * f[0] - 2 * f[-s]) / (6 * h);
    }
    if (vel > 0 && k > 0) return (f[0] - f[-s]) / h;
    if (vel <= 0 && k < n - 1) return (f[s] - f[0]) / h;
    if (k > 0) return (f[0] - f[-s]) / h;
    if (k < n - 1) return (f[s] - f[0]) / h;
    return 0.0;
}

// The same two stencils with every division by a precomputed divisor (divk.hpp: correctly
// rounded, so bit-identical): K2 = 2h, K6 = 6h, K1 = h
__device__ __forceinline__ double grad2k(const double *f, long s, int k, int n, const DivK &K2) {
    if (k == 0) return divk(-3 * f[0] + 4 * f[s] - f[2 * s], K2);
    if (k == n - 1) return divk(3 * f[0] - 4 * f[-s] + f[-2 * s], K2);
    return divk(f[s] - f[-s], K2);
}
__device__ __forceinline__ double upwind3k(const double *f, long s, int k, int n, double vel,
                                           const DivK &K6, const DivK &K1) {
    if (k >= 2 && k < n - 2) {
        if (vel > 0) return divk(2 * f[s] + 3 * f[0] - 6 * f[-s] + f[-2 * s], K6);
        return divk(-f[2 * s] + 6 * f[s] - 3 * f[0] - 2 * f[-s], K6);
    }
    if (vel > 0 && k > 0) return divk(f[0] - f[-s], K1);
    if (vel <= 0 && k < n - 1) return divk(f[s] - f[0], K1);
    if (k > 0) return divk(f[0] - f[-s], K1);
    if (k < n - 1) return divk(f[s] - f[0], K1);
    return 0.0;
}

// interpolators.py:4-61 bilinear_interpolate at one query point.  CHK (slab-decomposed
// step): the two rows read must be resident, rows [lo, hi); otherwise *oob is set and the
// result is NaN (a departure point farther than the halo: never at CFL <= 1).
template <bool CHK>
__device__ __forceinline__ double bilinear_t(const double *__restrict__ u, double xq, double yq,
                                             const DivK &Kx, const DivK &Ky, int nx, int ny,
                                             int lo, int hi, bool *oob) {
    double x = divk(xq, Kx), y = divk(yq, Ky);
    if (!(isfinite(x) && isfinite(y))) return __builtin_nan("");
    if (x < 0.0) x = 0.0; else if (x > nx - 1.0) x = nx - 1.0;
    if (y < 0.0) y = 0.0; else if (y > ny - 1.0) y = ny - 1.0;
    int ix = (int)floor(x), iy = (int)floor(y);
    if (ix >= nx - 1) ix = nx - 2;
    if (iy >= ny - 1) iy = ny - 2;
    if (CHK && (iy < lo || iy + 1 >= hi)) { *oob = true; return __builtin_nan(""); }
    double fx = x - ix, fy = y - iy;
    const double *r0 = u + (long)iy * nx, *r1 = r0 + nx;
    return (1 - fx) * (1 - fy) * r0[ix] + fx * (1 - fy) * r0[ix + 1] +
           (1 - fx) * fy * r1[ix] + fx * fy * r1[ix + 1];
}
// dx, dy entry (the standalone operators): the divisors made per call
__device__ __forceinline__ double bilinear(const double *__restrict__ u, double xq, double yq,
                                           double dx, double dy, int nx, int ny) {
    return bilinear_t<false>(u, xq, yq, divk_make(dx), divk_make(dy), nx, ny, 0, ny, nullptr);
}

// functions.py:194-227: RK4 backtrace of one point; returns the foot (xb, yb).
template <bool CHK>
__device__ __forceinline__ void sl_backtrace_t(const double *__restrict__ a,
                                               const double *__restrict__ b, double x, double y,
                                               double dt, const DivK &Kx, const DivK &Ky, int nx,
                                               int ny, int lo, int hi, bool *oob, double &xb,
                                               double &yb) {
#define BL_(f, X, Y) bilinear_t<CHK>(f, X, Y, Kx, Ky, nx, ny, lo, hi, oob)
    const double hdt = 0.5 * dt, dt6 = dt / 6.0;
    double k1x = BL_(a, x, y), k1y = BL_(b, x, y);
    double x2 = x - hdt * k1x, y2 = y - hdt * k1y;
    double k2x = BL_(a, x2, y2), k2y = BL_(b, x2, y2);
    double x3 = x - hdt * k2x, y3 = y - hdt * k2y;
    double k3x = BL_(a, x3, y3), k3y = BL_(b, x3, y3);
    double x4 = x - dt * k3x, y4 = y - dt * k3y;
    double k4x = BL_(a, x4, y4), k4y = BL_(b, x4, y4);
#undef BL_
    xb = x - dt6 * (k1x + 2 * k2x + 2 * k3x + k4x);
    yb = y - dt6 * (k1y + 2 * k2y + 2 * k3y + k4y);
}
__device__ __forceinline__ void sl_backtrace(const double *__restrict__ a,
                                             const double *__restrict__ b, double x, double y,
                                             double dt, double dx, double dy, int nx, int ny,
                                             double &xb, double &yb) {
    sl_backtrace_t<false>(a, b, x, y, dt, divk_make(dx), divk_make(dy), nx, ny, 0, ny, nullptr,
                          xb, yb);
}

// Semi-Lagrangian block skip.  With every velocity sample bounded by sqrt(m2) and
// dt * sqrt(m2) <= 0.9 h, every RK4 stage point and the foot of cell (i, j) lie within 0.9
// cells of it, so all its bilinear stencils read rows j-1 .. j+2 and columns i-1 .. i+2.  A
// block of cells [i0, i0 + w) of row j whose map is +0.0 on that whole neighbourhood therefore
// advects to exactly +0.0 (non-negative weights times +0.0, summed) -- the map is zero away
// from the solid, so most blocks skip the backtrace.  Rows outside [lo, hi) are not
// resident: such a block is not certified.  Call with every thread of the block.
// m2 from reduce_maxsq2_nan: finite only if every velocity is, so a skipped block needs no
// finiteness check of its own
__device__ __forceinline__ bool sl_skip_ok(const double *m2, double dt, double h) {
    return m2 && dt * sqrt(*m2) <= 0.9 * h;
}
__device__ __forceinline__ bool sl_zero_block(const double *__restrict__ X1,
                                              const double *__restrict__ X2, int ny, int nx,
                                              int j, int i0, int w, int lo, int hi) {
    const int ja = max(0, j - 1), jb = min(ny - 1, j + 2);
    const int ia = max(0, i0 - 1), ib = min(nx - 1, i0 + w + 1), cw = ib - ia + 1;
    const int nq = (jb - ja + 1) * cw;
    unsigned long long bits = (ja < lo || jb >= hi) ? 1 : 0;
    if (!bits) {
        // all loads issued before any test (no early exit: one memory round trip)
#pragma unroll 4
        for (int q = threadIdx.x; q < nq; q += blockDim.x) {
            const long c = (long)(ja + q / cw) * nx + ia + q % cw;
            bits |= (unsigned long long)__double_as_longlong(X1[c]) |
                    (unsigned long long)__double_as_longlong(X2[c]);
        }
    }
    return !__syncthreads_or(bits != 0);
}

// interpolators.py:144-156 cubic_convolution (Catmull-Rom); Numba's x**3 = x * (x * x)
__device__ __forceinline__ double cubic_conv(double v0, double v1, double v2, double v3, double x) {
    const double a0 = -0.5 * v0 + 1.5 * v1 - 1.5 * v2 + 0.5 * v3;
    const double a1 = v0 - 2.5 * v1 + 2.0 * v2 - 0.5 * v3;
    const double a2 = -0.5 * v0 + 0.5 * v2;
    const double x2 = x * x, x3 = x * x2;
    return a0 * x3 + a1 * x2 + a2 * x + v1;
}
// interpolators.py:64-142 bicubic_interpolate at one query point: clamped 4x4 stencil,
// Catmull-Rom in x then y, result clamped to the stencil's min / max
__device__ __forceinline__ double bicubic(const double *__restrict__ u, double xq, double yq,
                                          double dx, double dy, int nx, int ny) {
    double x = xq / dx, y = yq / dy;
    if (!(isfinite(x) && isfinite(y))) return __builtin_nan("");
    if (x < 0.0) x = 0.0; else if (x > nx - 1.0) x = nx - 1.0;
    if (y < 0.0) y = 0.0; else if (y > ny - 1.0) y = ny - 1.0;
    const int ix = (int)floor(x), iy = (int)floor(y);
    const double fx = x - ix, fy = y - iy;
    double rv[4], lo = 1e18, hi = -1e18;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        const int yg = min(max(iy - 1 + m, 0), ny - 1);
        double cv[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const double v = u[(long)yg * nx + min(max(ix - 1 + q, 0), nx - 1)];
            cv[q] = v;
            if (v < lo) lo = v;
            if (v > hi) hi = v;
        }
        rv[m] = cubic_conv(cv[0], cv[1], cv[2], cv[3], fx);
    }
    double r = cubic_conv(rv[0], rv[1], rv[2], rv[3], fy);
    if (r < lo) r = lo;
    if (r > hi) r = hi;
    return r;
}
// functions.py:228-251 RK4 backtrace with the bicubic interpolant
__device__ __forceinline__ void sl_backtrace_cubic(const double *__restrict__ a,
                                                   const double *__restrict__ b, double x,
                                                   double y, double dt, double dx, double dy,
                                                   int nx, int ny, double &xb, double &yb) {
    const double hdt = 0.5 * dt, dt6 = dt / 6.0;
    double k1x = bicubic(a, x, y, dx, dy, nx, ny), k1y = bicubic(b, x, y, dx, dy, nx, ny);
    double x2 = x - hdt * k1x, y2 = y - hdt * k1y;
    double k2x = bicubic(a, x2, y2, dx, dy, nx, ny), k2y = bicubic(b, x2, y2, dx, dy, nx, ny);
    double x3 = x - hdt * k2x, y3 = y - hdt * k2y;
    double k3x = bicubic(a, x3, y3, dx, dy, nx, ny), k3y = bicubic(b, x3, y3, dx, dy, nx, ny);
    double x4 = x - dt * k3x, y4 = y - dt * k3y;
    double k4x = bicubic(a, x4, y4, dx, dy, nx, ny), k4y = bicubic(b, x4, y4, dx, dy, nx, ny);
    xb = x - dt6 * (k1x + 2 * k2x + 2 * k3x + k4x);
    yb = y - dt6 * (k1y + 2 * k2y + 2 * k3y + k4y);
}

// benchmarks/common.py:55-57 disc signed distance, numpy order: sqrt(dx*dx + dy*dy) - R.
__device__ __forceinline__ double disc_phi(double X1, double X2, double x0, double y0,
                                           double R) {
    double a = X1 - x0, b = X2 - y0;
    return sqrt(a * a + b * b) - R;
}

// functions.py:660-671 smoothed_heaviside.
// The two constant branches are taken before the sine (the values the reference's np.where
// keeps; a NaN v fails both tests and takes the formula, as there): most cells of a grid lie
// outside the band, and an f64 sine is ~100 instructions.
__device__ __forceinline__ double heaviside(double v, double w_t) {
    if (v > w_t) return 1.0;
    if (v < -w_t) return 0.0;
    const double inv_wt = 1.0 / w_t, inv_pi = 1.0 / M_PI;
    return 0.5 * (1.0 + v * inv_wt + inv_pi * sin(M_PI * v * inv_wt));
}

// output.py:41-134 strain-energy density at one cell (4-cell edge-padded central grads).
__device__ __forceinline__ double se_density(const double *__restrict__ X1,
                                             const double *__restrict__ X2, long c, int j, int i,
                                             int ny, int nx, double dx, double dy, double mu_s,
                                             double kappa) {
    long cl = i > 0 ? c - 1 : c, cr = i < nx - 1 ? c + 1 : c;
    long cd = j > 0 ? c - nx : c, cu = j < ny - 1 ? c + nx : c;
    double G11 = (X1[cr] - X1[cl]) / (2 * dx), G12 = (X1[cu] - X1[cd]) / (2 * dy);
    double G21 = (X2[cr] - X2[cl]) / (2 * dx), G22 = (X2[cu] - X2[cd]) / (2 * dy);
    double detG = G11 * G22 - G12 * G21;
    if (!(fabs(detG) > 1e-10)) return 0.0;
    double F11 = G22 / detG, F12 = -G12 / detG, F21 = -G21 / detG, F22 = G11 / detG;
    double I1 = (F11 * F11 + F21 * F21) + (F12 * F12 + F22 * F22);
    double Jv = 1.0 / detG, jm = Jv - 1.0;
    return 0.5 * mu_s * (I1 - 2.0) + 0.5 * kappa * (jm * jm);
}

struct Stress { double sxx, sxy, syy, J; };
// The cell arithmetic of functions.py:545-658 on accessors: X1(o), X2(o), PH(o) give the
// value at the neighbour o of the cell (o: 0 = c, 1 = left, 2 = right, 3 = down, 4 = up), so
// that a kernel can take phi from LDS and the map from any plane -- one arithmetic for all.
template <class F1, class F2, class FP>
__device__ __forceinline__ bool solid_stress_acc(F1 X1, F2 X2, FP PH, double dx, double dy,
                                                 double mu_s, double kappa, double w_cut,
                                                 double clamp, bool iso, Stress &out) {
    out = {0.0, 0.0, 0.0, 1.0};
    double pc = PH(0);
    bool in_band = w_cut > 0.0 ? (pc < w_cut) : (pc <= 0.0);
    if (!in_band) return false;
    const double inv_2dx = 1.0 / (2.0 * dx), inv_2dy = 1.0 / (2.0 * dy);
    double g11, g21, g12, g22;
    if (w_cut > 0.0) {
        g11 = (X1(2) - X1(1)) * inv_2dx; g21 = (X2(2) - X2(1)) * inv_2dx;
        g12 = (X1(4) - X1(3)) * inv_2dy; g22 = (X2(4) - X2(3)) * inv_2dy;
    } else {
        bool lf = PH(1) > 0.0, rf = PH(2) > 0.0;
        if (lf && !rf) { g11 = (X1(2) - X1(0)) / dx; g21 = (X2(2) - X2(0)) / dx; }
        else if (rf && !lf) { g11 = (X1(0) - X1(1)) / dx; g21 = (X2(0) - X2(1)) / dx; }
        else { g11 = (X1(2) - X1(1)) * inv_2dx; g21 = (X2(2) - X2(1)) * inv_2dx; }
        bool bf = PH(3) > 0.0, tf = PH(4) > 0.0;
        if (bf && !tf) { g12 = (X1(4) - X1(0)) / dy; g22 = (X2(4) - X2(0)) / dy; }
        else if (tf && !bf) { g12 = (X1(0) - X1(3)) / dy; g22 = (X2(0) - X2(3)) / dy; }
        else { g12 = (X1(4) - X1(3)) * inv_2dy; g22 = (X2(4) - X2(3)) * inv_2dy; }
    }
    double detG = g11 * g22 - g12 * g21;
    if (fabs(detG) < 1e-10) return false;
    if (clamp > 0.0) {
        double lo = 1.0 / clamp;
        if (detG < lo) detG = lo; else if (detG > clamp) detG = clamp;
    }
    double f11 = g22 / detG, f12 = -g12 / detG, f21 = -g21 / detG, f22 = g11 / detG;
    double b11 = f11 * f11 + f12 * f12, b12 = f11 * f21 + f12 * f22, b22 = f21 * f21 + f22 * f22;
    double jv = 1.0 / detG;
    double vol = kappa * (jv - 1.0);
    if (iso) {
        double trh = 0.5 * (b11 + b22), jm2 = 1.0 / (jv * jv);
        out = {mu_s * jm2 * (b11 - trh) + vol, mu_s * jm2 * b12, mu_s * jm2 * (b22 - trh) + vol, jv};
    } else {
        out = {mu_s * b11 + vol, mu_s * b12, mu_s * b22 + vol, jv};
    }
    return true;
}
// functions.py:545-658 solid_cauchy_stress at interior cell c of the planes (offsets 1, nx)
__device__ __forceinline__ bool solid_stress_cell(const double *__restrict__ X1,
                                                  const double *__restrict__ X2,
                                                  const double *__restrict__ phi, long c,
                                                  long nx, double dx, double dy, double mu_s,
                                                  double kappa, double w_cut, double clamp,
                                                  bool iso, Stress &out) {
    const long off[5] = {c, c - 1, c + 1, c - nx, c + nx};
    return solid_stress_acc([&](int o) { return X1[off[o]]; }, [&](int o) { return X2[off[o]]; },
                            [&](int o) { return phi[off[o]]; }, dx, dy, mu_s, kappa, w_cut,
                            clamp, iso, out);
}

// functions.py:256-318 WENO5 reconstructions (Jiang-Shu, eps 1e-6; x**2 as x*x like Numba).
__device__ __forceinline__ double weno5_combine(double r0, double r1, double r2, double s0,
                                                double t0, double s1, double t1, double s2,
                                                double t2) {
    const double eps = 1.0e-6;
    double b0 = (13.0 / 12.0) * (s0 * s0) + (1.0 / 4.0) * (t0 * t0);
    double b1 = (13.0 / 12.0) * (s1 * s1) + (1.0 / 4.0) * (t1 * t1);
    double b2 = (13.0 / 12.0) * (s2 * s2) + (1.0 / 4.0) * (t2 * t2);
    double e0 = eps + b0, e1 = eps + b1, e2 = eps + b2;
    double a0 = 0.1 / (e0 * e0), a1 = 0.6 / (e1 * e1), a2 = 0.3 / (e2 * e2);
    double as = a0 + a1 + a2;
    return (a0 / as) * r0 + (a1 / as) * r1 + (a2 / as) * r2;
}
__device__ __forceinline__ double weno5_left(double vm2, double vm1, double v0, double vp1,
                                             double vp2) {
    return weno5_combine((2.0 * vm2 - 7.0 * vm1 + 11.0 * v0) / 6.0,
                         (-vm1 + 5.0 * v0 + 2.0 * vp1) / 6.0,
                         (2.0 * v0 + 5.0 * vp1 - vp2) / 6.0,
                         vm2 - 2.0 * vm1 + v0, vm2 - 4.0 * vm1 + 3.0 * v0,
                         vm1 - 2.0 * v0 + vp1, vm1 - vp1,
                         v0 - 2.0 * vp1 + vp2, 3.0 * v0 - 4.0 * vp1 + vp2);
}
__device__ __forceinline__ double weno5_right(double vm1, double v0, double vp1, double vp2,
                                              double vp3) {
    return weno5_combine((2.0 * vp3 - 7.0 * vp2 + 11.0 * vp1) / 6.0,
                         (-vp2 + 5.0 * vp1 + 2.0 * v0) / 6.0,
                         (2.0 * vp1 + 5.0 * v0 - vm1) / 6.0,
                         vp3 - 2.0 * vp2 + vp1, 3.0 * vp1 - 4.0 * vp2 + vp3,
                         vp2 - 2.0 * vp1 + v0, vp2 - v0,
                         vp1 - 2.0 * v0 + vm1, vp1 - 4.0 * v0 + 3.0 * vm1);
}
// functions.py:347-389: (q_{k+1/2} - q_{k-1/2}) along a line with domain-edge fallbacks;
// f points at element k.
__device__ __forceinline__ double weno5_diff(const double *f, long s, int k, int n, double vel) {
#define F_(o) f[(long)(o) * s]
    double qp, qm;
    if (vel >= 0.0) {
        qp = weno5_left(F_(-2), F_(-1), F_(0), F_(1), F_(2));
        qm = k >= 3 ? weno5_left(F_(-3), F_(-2), F_(-1), F_(0), F_(1))
                    : weno5_left(F_(-2), F_(-1), F_(0), F_(1), F_(2));
    } else {
        qp = k + 3 < n ? weno5_right(F_(-1), F_(0), F_(1), F_(2), F_(3))
                       : weno5_left(F_(-2), F_(-1), F_(0), F_(1), F_(2));
        qm = weno5_right(F_(-1), F_(0), F_(1), F_(2), k + 3 < n ? F_(3) : F_(n - 1 - k));
    }
#undef F_
    return qp - qm;
}

// benchmarks/common.py:27-50 as data: for boundary kind `kind`, the BC'd value of each
// velocity component at (j, i) is either a constant or the raw (pre-BC) value of one
// source cell.  Callers read the raw value themselves (no device lambdas).
// functions.py:1073-1089 (_compute_pressure_gradient) at one cell
// of p - m (m: a mean not yet subtracted from p; x - 0.0 == x, so m = 0 is the plain field)
__device__ __forceinline__ void pgrad_cell(const double *__restrict__ p, long c, int j, int i,
                                           int ny, int nx, double dx, double dy, double &gx,
                                           double &gy, double m = 0.0) {
    const double *row = p + (c - i), *col = p + i;
    gx = 0.0; gy = 0.0;
    if (j >= 1 && j < ny - 1 && i >= 1 && i < nx - 1) {
        gx = ((p[c + 1] - m) - (p[c - 1] - m)) / (2 * dx);
        gy = ((p[c + nx] - m) - (p[c - nx] - m)) / (2 * dy);
    }
    if (i == 0) gx = (-3.0 * (row[0] - m) + 4.0 * (row[1] - m) - (row[2] - m)) / (2.0 * dx);
    if (i == nx - 1)
        gx = (3.0 * (row[nx - 1] - m) - 4.0 * (row[nx - 2] - m) + (row[nx - 3] - m)) / (2.0 * dx);
    if (j == 0) gy = (-3.0 * (col[0] - m) + 4.0 * (col[nx] - m) - (col[2L * nx] - m)) / (2.0 * dy);
    if (j == ny - 1)
        gy = (3.0 * (col[(long)(ny - 1) * nx] - m) - 4.0 * (col[(long)(ny - 2) * nx] - m) +
              (col[(long)(ny - 3) * nx] - m)) / (2.0 * dy);
}
// pgrad_cell with the divisions by 2dx, 2dy precomputed (divk.hpp, bit-identical)
__device__ __forceinline__ void pgrad_cellk(const double *__restrict__ p, long c, int j, int i,
                                            int ny, int nx, const DivK &Kx2, const DivK &Ky2,
                                            double &gx, double &gy, double m = 0.0) {
    const double *row = p + (c - i), *col = p + i;
    gx = 0.0; gy = 0.0;
    if (j >= 1 && j < ny - 1 && i >= 1 && i < nx - 1) {
        gx = divk((p[c + 1] - m) - (p[c - 1] - m), Kx2);
        gy = divk((p[c + nx] - m) - (p[c - nx] - m), Ky2);
    }
    if (i == 0) gx = divk(-3.0 * (row[0] - m) + 4.0 * (row[1] - m) - (row[2] - m), Kx2);
    if (i == nx - 1)
        gx = divk(3.0 * (row[nx - 1] - m) - 4.0 * (row[nx - 2] - m) + (row[nx - 3] - m), Kx2);
    if (j == 0) gy = divk(-3.0 * (col[0] - m) + 4.0 * (col[nx] - m) - (col[2L * nx] - m), Ky2);
    if (j == ny - 1)
        gy = divk(3.0 * (col[(long)(ny - 1) * nx] - m) - 4.0 * (col[(long)(ny - 2) * nx] - m) +
                  (col[(long)(ny - 3) * nx] - m), Ky2);
}
struct BCSrc {
    bool u_const, v_const;
    double u_val, v_val;
    long u_src, v_src;
};
__device__ __forceinline__ BCSrc bc_source(int kind, double lid, int j, int i, int ny, int nx) {
    const long c = (long)j * nx + i;
    BCSrc s{false, false, 0.0, 0.0, c, c};
    if (kind == RMT_BC_NOSLIP_LID) {
        if (i == 0 || i == nx - 1 || j == 0 || j == ny - 1) {
            s.u_const = s.v_const = true;
            s.u_val = (j == ny - 1 && i != 0 && i != nx - 1) ? lid : 0.0;
        }
    } else if (kind == RMT_BC_PERIODIC) {
        // test_poisson.py _periodic_bc: last column <- column 0, then last row <- row 0
        s.u_src = s.v_src = (long)(j == ny - 1 ? 0 : j) * nx + (i == nx - 1 ? 0 : i);
    } else if (kind == RMT_BC_FREESLIP_BOX) {
        if (i == 0 || i == nx - 1) s.u_const = true;
        else if (j == 0) s.u_src = c + nx;
        else if (j == ny - 1) s.u_src = c - nx;
        if (j == 0 || j == ny - 1) s.v_const = true;
        else if (i == 0) s.v_src = c + 1;
        else if (i == nx - 1) s.v_src = c - 1;
    }
    return s;
}

// ------------------------------------------------------------------- reductions --
constexpr int RED_BLOCKS = 1024, RED_T = 256;   // ctx->red holds RED_BLOCKS + 64 doubles
int reduce_sum(rmt_ctx *ctx, const double *x, long n, double *dev_out);     // device scalar
int reduce_max(rmt_ctx *ctx, const double *x, long n, double *dev_out);
int reduce_maxsq2(rmt_ctx *ctx, const double *a, const double *b, long n, double *dev_out);
// the same with NaN propagating (a non-finite velocity makes the bound NaN: no SL block skip)
int reduce_maxsq2_nan(rmt_ctx *ctx, const double *a, const double *b, long n, double *dev_out);
int reduce_max_partials_nan(rmt_ctx *ctx, double *o);   // (RED_BLOCKS partials in ctx->red)
int reduce_mean(rmt_ctx *ctx, const double *x, long n, double *dev_out);
int read_scalar(rmt_ctx *ctx, const double *dev, double *host);
// row-tree sums (ops.hip): root of rows [0, nrows) of x (row length nx) into *dev_root;
// x -= tree(G roots) / count; and both for a whole (ny, nx) plane
int rowtree_root(rmt_ctx *ctx, const double *x, int nrows, int nx, double *dev_root);
// the tree over row sums already in ctx->rsum (dct_pass's rs)
int rowtree_sums(rmt_ctx *ctx, int nrows, double *dev_root);
int sub_tree_mean(rmt_ctx *ctx, double *x, long n, const double *dev_roots, int G, double count);
// functions.py:1255-1364 (constant density, Neumann DCT-I) for the fused step: dt read from
// the device (dtp), and the max of u^2 + v^2 over the corrected velocity per 256-cell block
// into m2part (the next step's compute_timestep input), ceil(nx / 256) * ny entries
// the same projection split around the extrapolation chain: rows part (Rhie-Chow rhs + row
// DCT-I into ctx->scratch; rowmark: only the marked rows, else all), then the rest (dtp null:
// the scalar dt)
int projection_rows(rmt_ctx *ctx, const double *a_star, const double *b_star, double dx,
                    double dy, const double *dtp, double dt, double rho, const double *p_prev,
                    const unsigned char *rowmark, const int *tiles = nullptr,
                    const int *tcount = nullptr, int max_tiles = 0,
                    const unsigned char *dct_skip = nullptr);
int projection_finish(rmt_ctx *ctx, const double *a_star, const double *b_star, double dx,
                      double dy, const double *dtp, double dt, double rho, int bc_kind,
                      double lid, const double *p_prev, double *a, double *b, double *p,
                      double *m2part, bool sub_mean = true,
                      const unsigned char *early_marks = nullptr, hipEvent_t done = nullptr);
int projection_dev(rmt_ctx *ctx, const double *a_star, const double *b_star, double dx,
                   double dy, const double *dtp, double rho, int bc_kind, double lid,
                   const double *p_prev, double *a, double *b, double *p, double *m2part);
int sub_mean_rows(rmt_ctx *ctx, double *x, int ny, int nx);
// p = p + (pc - *pc_root / (ny nx)) then p -= mean(p): projection_finish(sub_mean = false)'s
// deferred pressure update and mean removal in one pass
int sub_mean_rows_upd(rmt_ctx *ctx, double *p, const double *pc, const double *pc_root, int ny,
                      int nx);

// Row window of a slab-decomposed call (slab.hip): planes are addressed with GLOBAL cell
// indices j*nx + i (the caller offsets its pointers by -lo*nx), rows [lo, hi) are resident,
// rows [jb, je) are computed, and ny stays the global row count, so every boundary test
// of the reference sees the true domain edge.  A single-domain call is {0, ny, 0, ny}.
struct RowWin { int jb, je, lo, hi; };

// rho > 0: divU = (rho * div) / dt, the projection's rhs (dt = *dtp when dtp is given)
int divergence_rc_rows(rmt_ctx *ctx, const double *a, const double *b, const double *p,
                       double d_f, double dx, double dy, double *divU, int jb, int je,
                       double rho = 0.0, double dt = 1.0, const double *dtp = nullptr);
// dtp (nullable): dt_rho = *dtp / rho on the device
int project_correct_rows(rmt_ctx *ctx, const double *a_s, const double *b_s, const double *pc,
                         const double *p_prev, double dx, double dy, double dt_rho, int bc,
                         double lid, double *a, double *b, double *p, int jb, int je,
                         const double *dtp = nullptr, double rho = 1.0);

// sim.hip: the fused step's diagnostic partials (centroid sums, J range, energies) over rows
// [jb, je); part holds DIAG_PART doubles, out receives 10
constexpr int DIAG_PART = 512 * 10;
int diag_rows(rmt_ctx *ctx, const double *phi, const double *J, const double *xs,
              const double *ys, const double *u, const double *v, const double *X1,
              const double *X2, const rmt_sim_params &P, int jb, int je, double *part,
              double *out);

// dev_m2 (optional, device): a bound on a^2 + b^2 over the grid (enables the block skip);
// kbits (optional): the known plane (phi_pre < 0) as 64-cell words instead of phi_pre;
// cbox (optional, host {j0, j1, i0, i1}): only the 64 x 4 tiles meeting those cells
int sl_disc_map(rmt_ctx *ctx, const double *X1, const double *X2, const double *a,
                const double *b, const double *xs, const double *ys, double dt, double dx,
                double dy, double x0, double y0, double R, double *X1n, double *X2n,
                double *phi_pre, int *bad, const double *dev_m2 = nullptr,
                unsigned long long *kbits = nullptr, const int *cbox = nullptr,
                bool faces = false);

// --------------------------------------------------------------------- momentum --
// every stage keeps its own k plane (k1, k2, k3; the last stage forms (k1 + 2 k2) + 2 k3
// itself), so a tile-list re-run of any stage (momentum_fixup) finds its inputs.  accu/accv
// serve the unfused mode only; acc2u holds the stage kernels' pure-fluid tile-row flags
constexpr int MOM_WORK_PLANES = 17;
struct MomWork {                 // MOM_WORK_PLANES planes + solid byte plane + flag
    double *H, *rho, *k1u, *k1v, *k2u, *k2v, *accu, *accv, *us, *vs, *gxx, *gxy, *gyy;
    double *k3u, *k3v, *acc2u, *acc2v;
    unsigned char *solid;
    int *any_solid;
    const double *dtp;           // device dt (the fused step's k_dt output), or null: P->dt
    // the pure-fluid row flags (k_fluid_rows' output, at fluid_rows_buf) were already written
    // by the producer of phi (the fused step's k_phi_rebuild): momentum_rk4 skips that pass
    bool fluid_rows_ready = false;
    // or k_sim_sl_t left per-(row, tile) bits there (its phi output; k_fluid_rows_bits)
    const unsigned char *fluid_bits = nullptr;
    // (nullable) an event the stages wait for before they read p (sim.hip's tail_stream)
    hipEvent_t wait_p = nullptr;
    // per 64-column row segment (nx % 64 == 0), persistent across steps: the last write of the
    // prep planes there was a pure-fluid segment's constants, so k_mom_prep may skip it while
    // it stays pure fluid (null: prep every cell)
    unsigned char *prep_const = nullptr;
};
inline MomWork mom_work(double *w, long n, unsigned char *solid, int *flag) {
    return MomWork{w,          w + n,      w + 2 * n,  w + 3 * n,  w + 4 * n,  w + 5 * n,
                   w + 6 * n,  w + 7 * n,  w + 8 * n,  w + 9 * n,  w + 10 * n, w + 11 * n,
                   w + 12 * n, w + 13 * n, w + 14 * n, w + 15 * n, w + 16 * n, solid, flag,
                   nullptr, false, nullptr, nullptr};
}
// where momentum_rk4 keeps the per-(row, 64-column tile) pure-fluid flags of rows [lo, ...)
inline unsigned char *fluid_rows_buf(const MomWork &W, int lo, int nx) {
    return (unsigned char *)(W.acc2u + (long)lo * nx);
}
// where k_sim_sl_t leaves its per-(row, 64-column tile) fluid bits (the fused step: whole grid)
inline unsigned char *fluid_bits_buf(const MomWork &W) { return (unsigned char *)W.acc2v; }
// the flags' threshold: a stage tile is pure fluid where every phi > max(w_t, w_cut, 0)
inline double fluid_threshold(const rmt_momentum_params *P) {
    const double w_cut = P->stress_band ? P->w_t : 0.0;
    return std::max({P->w_t, w_cut, 0.0});
}
int momentum_rk4(rmt_ctx *ctx, const rmt_momentum_params *P, const double *u, const double *v,
                 const double *p, const double *X1, const double *X2, const double *phi,
                 double *u_new, double *v_new, double *sxx, double *sxy, double *syy, double *J,
                 const MomWork &W, const RowWin *win = nullptr);
// re-run prep + the 4 stages on the 64 x 16 tiles listed in tiles[0 .. *count) (device) after
// a speculative momentum_rk4 whose inputs changed only inside them (sim.hip overlap)
constexpr int MOM_TX = 64, MOM_TY = 16;
int momentum_mode();   // rmt_momentum_set_mode / RMT_MOM_MODE
// the context's edge-tile stream at ctx->stream's priority (nullptr: opt.edge_stream off or no
// stream of the context's own)
int edge_stream(rmt_ctx *ctx, hipStream_t *out);
// skip_prep: the caller ran fixup_phi_prep on the same tiles
int momentum_fixup(rmt_ctx *ctx, const rmt_momentum_params *P, const double *u, const double *v,
                   const double *p, const double *X1, const double *X2, const double *phi,
                   double *u_new, double *v_new, double *sxx, double *sxy, double *syy, double *J,
                   const MomWork &W, const int *tiles, const int *count, int max_tiles,
                   const RowWin *win = nullptr, bool skip_prep = false);
// the fused step's level-set rebuild on the fix-up tiles and momentum_fixup's prep in one
// kernel (k_phi_prep_tiles; single domain, nx % 64 == 0): X1, X2 <- X1n, X2n, phi =
// disc_phi(X1n, X2n), the next step's known-plane words (nbits, nullable), then the prep planes
int fixup_phi_prep(rmt_ctx *ctx, const rmt_momentum_params *P, const MomWork &W,
                   const double *X1n, const double *X2n, double x0, double y0, double R,
                   double *X1, double *X2, double *phi, unsigned long long *nbits, double *sxx,
                   double *sxy, double *syy, double *J, const int *tiles, const int *count,
                   int max_tiles, const int *st_src = nullptr, int *st_dst = nullptr,
                   hipEvent_t done = nullptr);

// ---------------------------------------------------------------------- poisson --
// dev_root: nullptr -> p = solve - mean (functions.py:1119); else p = the raw solve and
// *dev_root = its row-tree sum (mean = *dev_root / (ny nx), the caller subtracts it as it
// reads p), or 0 when the mean was subtracted already (rocFFT path)
int dct_solve(rmt_ctx *ctx, const double *rhs, double dx, double dy, double *p,
              double *dev_root = nullptr);
int dct_plan(rmt_ctx *ctx, double dx, double dy);
bool dct_lds_ready(rmt_ctx *ctx);
// rs (nullable): per-row sums of the output, in k_rowsum's order (rowtree_sums finishes them);
// rowmark (nullable): transform only the rows r with rowmark[r] != 0 (unmarked: only the
// others)
int dct_pass(rmt_ctx *ctx, bool solve, int axis, const double *src, double *dst, int nrows,
             int row0, double scale, double *rs = nullptr,
             const unsigned char *rowmark = nullptr, bool unmarked = false);
// the LDS solve after its forward row pass (pc holds DCT_x of the rhs): columns, inverse rows,
// the row-tree sum of the result into *dev_root (mean not subtracted)
int dct_solve_after_rows(rmt_ctx *ctx, double *pc, double *dev_root,
                         const unsigned char *early_marks = nullptr);
// the row blocks of pc without a marked row, transposed into the plan's column buffer ahead
// of dct_solve_after_rows(..., rowmark) (which then transposes only the others)
int dct_transpose_unmarked(rmt_ctx *ctx, const double *pc, const unsigned char *rowmark);
void transpose(const rmt_ctx *ctx, hipStream_t st, const double *in, int R, int C, double *out,
               const unsigned char *rowmark = nullptr, int mode = 0);
// MAC grid (mac.py:104-123): DCT-II Neumann solve on a (ny, nx) cell grid, (0,0) -> 0
int dct2_plan(rmt_ctx *ctx, int ny, int nx, double dx, double dy);
// mroot (nullable): rhs's row-tree root; the solve then takes rhs - root / mcount
int dct2_solve(rmt_ctx *ctx, const double *rhs, double *p, const double *mroot = nullptr,
               double mcount = 1.0);
int dct2_set_lambda(rmt_ctx *ctx, const double *lamx, const double *lamy);
// one DCT-II pass over nrows rows (mode 0 forward, 1 column solve with row0 = global
// x-frequency of local row 0, 2 inverse; axis 0: length nx, 1: length ny)
int dct2_pass(rmt_ctx *ctx, int mode, int axis, const double *src, double *dst, int nrows,
              int row0, const double *mroot = nullptr, double mcount = 1.0);
void dct2_destroy(Dct2Plan *P);
void per_destroy(PerPlan *P);
void dct_destroy(DctPlan *);

// ------------------------------------------------------------------ extrapolate --
// dev_status (optional, device): receives {cells fitted, aborted} after the sweep
// kin (optional): the known plane (phi < 0) as 64-cell words, ny x ceil(nx/64); phi unused then
int extrapolate(rmt_ctx *ctx, const double *X1, const double *X2, const double *phi, double dx,
                double dy, int max_layers, double *X1o, double *X2o, int *dev_status = nullptr,
                const unsigned long long *kin = nullptr);
// extrapolate() in two halves: the geometry (reads no map value when kin is given and the
// call is in place) and the values + chain (max_layers > 0; same ctx, nothing else may use
// ctx->bytes in between)
int extrap_geometry(rmt_ctx *ctx, const double *X1, const double *X2, const double *phi,
                    double dx, double dy, int max_layers, double *X1o, double *X2o,
                    const unsigned long long *kin);
// the extrapolation's device status words {fitted, aborted} (valid until the next geometry)
const int *extrap_status(rmt_ctx *ctx, int max_layers);
// the error message for a nonzero abort word (status[1]; extrap.hpp EXA_*): what timed out,
// in which chain part, waiting for which producer
std::string extrap_abort_detail(int code);
int extrap_finish(rmt_ctx *ctx, double dx, double dy, int max_layers, double *X1o, double *X2o,
                  int *dev_status);
// the fallback sweep of the last extrap_finish on stream s (ctx->ex_sweep_defer), ordered after
// that call's ev_chain; the map and the status words are final once it completes
int extrap_sweep(rmt_ctx *ctx, double dx, double dy, int max_layers, double *X1o, double *X2o,
                 hipStream_t s);
size_t extrap_workspace(int ny, int nx, int max_layers, bool px = false);   // ctx->bytes used
void imex_destroy(rmt_ctx *ctx);   // imex.hip: the context's DST plans
// the parallel extrapolation mode (extrap_par.hip; rmt_extrap_set_parallel or the environment
// variable RMT_EXTRAP_PARALLEL=1): the fits solved as one sparse triangular system by
// segments instead of the exact raster-order chain -- not bit-exact, see extrap_par.hip
bool extrap_par_enabled();
// generation of the extrapolation's configuration (mode, parallel switch): bumped on a change
unsigned long extrap_config_gen();
void extrap_config_changed();
// the exact no-op test of extrapolate() (k_ex_none) on rows [jb, je) of a whole known plane:
// ctl[EXC_ANY] (extrap.hpp; zeroed by the caller) set iff a first-layer target there fits
int extrap_none_rows(rmt_ctx *ctx, const unsigned long long *kbits, int ny, int nx, double dx,
                     double dy, int jb, int je, int *ctl);
// after extrapolate(): the MOM_TX x MOM_TY tiles within `margin` cells of a possible target
// (device list + count); the momentum of every other cell ignores the extrapolated values
int extrap_fix_tiles(rmt_ctx *ctx, int max_layers, int margin, int *list, int *count);

// --------------------------------------------------------- slab phases (slab.hip) --
// shared by the cell-centred slabs (rmt_slab) and the MAC slabs (rmt_mac_slab, mac.hip);
// plane pointers are global-index views (pointer - lo * nx)
int slab_sl(rmt_ctx *ctx, const double *X1, const double *X2, const double *a, const double *b,
            const double *xs, const double *ys, int ny, int nx, double dt, double dx, double dy,
            double x0, double y0, double R, double *X1n, double *X2n, double *phi_pre,
            int *flags, int jb, int je, int lo, int hi, const double *dev_m2 = nullptr);
int slab_bits(rmt_ctx *ctx, const double *phi, int nx, int W, unsigned long long *bits, int r0,
              int r1);
// cells whose 15x15 box holds a known and an unknown cell (the values the extrapolation can
// read or write), as bit words of the whole grid; rowcnt: ny + 1 ints of scratch
int rim_words(rmt_ctx *ctx, const unsigned long long *bits, int ny, int nx, int W,
              unsigned long long *rimw, int *rowcnt);
int slab_rim_pack(rmt_ctx *ctx, const unsigned long long *bits, int ny, int nx, int W, int r0,
                  int r1, unsigned long long *rimw, int *rowcnt, const double *X1n,
                  const double *X2n, double *rim, double *count);
int slab_rim_extrapolate(rmt_ctx *ctx, const double *gathered, const long long *counts, int G,
                         long long cap, double *X1d, double *X2d, const unsigned long long *bits,
                         double dx, double dy, int layers, int *exflags, double *X1n,
                         double *X2n, long c_lo, long c_hi,
                         const double *gs = nullptr, hipEvent_t geo = nullptr);
int slab_cols(rmt_ctx *ctx, bool pack, double *Y, int rows, int nx, const int *csplits, int G,
              double *A);

}  // namespace rmt
