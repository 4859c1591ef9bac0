// divk.hpp -- correctly rounded division by a divisor known in advance (bit-identical to
// IEEE x / d), for the stencil divisions of the reference: (f[i+1] - f[i-1]) / (2h),
// (...) / (6h), xq / dx, (...) / (rho + 1e-12) with constant rho (utils.py:4-114,
// interpolators.py:21, functions.py:941).  The reference divides; a compiled f64 division is
// 11 VALU instructions on gfx950 (v_div_scale x2, v_rcp, 5 fma, mul, v_div_fmas,
// v_div_fixup); this is 3 fma-class instructions plus an integer range test.
//
// Precomputed on the host: yh = RN(1/d), yl = RN(1/d - yh).  For x:
//     q0 = RN(x*yh + RN(x*yl))        (fma)
//     t  = RN(q0*d - x)               (fma; exact, see below)
//     q1 = RN(q0 - t*yh)              (fma)
// Claim: q1 = RN(x/d) for every x with 2^-900 <= |x| < 2^1000, and for x = +-0 (|q1| = 0;
// the sign is copied from x, as x/d has it for d > 0), provided d > 0 is normal and its
// significand D = d / 2^e_d satisfies D < 2 - 2^-50 (checked on the host; D = 1 is exact)
// and its exponent e_d lies in [-20, 60] (DIVK_ED_MIN .. DIVK_ED_MAX): then for every
// certified x the quotient x/d stays normal and finite (|x/d| < 2^1000 / 2^-20 = 2^1020 and
// > 2^-900 / 2^61 = 2^-961) and x*yl (~ 2^-54 x/d >= 2^-1015) does not underflow, which the
// sketch below assumes.  Other divisors take IEEE division (rspan = 0).
// Proof sketch (z = x/d, z in [2^f, 2^(f+1)), u = ulp(z) = 2^(f-52)):
//   * |x*(yh+yl) - z| <= 2^-106 z and |RN(x*yl) - x*yl| <= 2^-106 z, so q0 = RN(z(1+eta))
//     with |eta| <= 2^-105(1+2^-50): |q0 - z| <= u/2 + 2^-52 u < u, so q0 is a faithful
//     quotient and the remainder x - q0*d is exactly representable (no underflow: the
//     remainder's grain 2^(e_q0 + e_d - 104) >= 2^-1074 for |x| >= 2^-900), i.e. t is exact.
//   * q0 - t*yh = q0 + (z - q0) d yh = z - (z - q0) eps with eps = 1 - d*yh,
//     |eps| <= d * ulp(1/d)/2 = D 2^-54.  So q1 = RN(z') with |z' - z| <= (1/2 + 2^-52) u D 2^-54.
//   * No midpoint m = (odd) 2^(f-53) lies that close to z: x is a multiple of 2^(f+e_d-52),
//     m*d = odd * Dint * 2^(f+e_d-105) (Dint = D 2^52), so x - m*d is a nonzero multiple of
//     2^(f+e_d-105) (a binary quotient is never a midpoint) and |z - m| >= 2^-53 u / D.
//   * (1/2 + 2^-52) D 2^-54 < 2^-53 / D  <=>  D^2 (1 + 2^-51) < 4, true for D < 2 - 2^-50:
//     z' and z lie strictly between the same two midpoints (the binade edges below z have a
//     finer grid and lie farther away), so RN(z') = RN(z).
// Outside the certified range (NaN, inf, |x| < 2^-900 nonzero, |x| >= 2^1000) the kernel
// takes IEEE division.  tools/divk_check.hip tests the claim against IEEE division on the
// hardest cases (x/d within 2^-105 relative of a midpoint, built from Dint^-1 mod 2^54) and
// on random operands; tests/test_divk.py runs it, and the GPU suite checks the device code.
#pragma once
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdint>
#include <cstring>

namespace rmt {

struct DivK {
    double d, yh, yl;
    unsigned rspan;   // certified |x| high words [DIVK_HI_LO, DIVK_HI_LO + rspan); 0: IEEE only
};

// 2^-900 and 2^1000 as high words of |x| (exponent field in bits 20..30)
constexpr unsigned DIVK_HI_LO = (unsigned)(1023 - 900) << 20;
constexpr unsigned DIVK_HI_HI = (unsigned)(1023 + 1000) << 20;
constexpr int DIVK_ED_MIN = -20, DIVK_ED_MAX = 60;   // certified divisor exponents

__host__ __device__ inline DivK divk_make(double d) {
    DivK k{d, 0.0, 0.0, 0u};
    if (!(d > 0.0) || !std::isfinite(d) || !std::isnormal(d)) return k;   // IEEE only
    int e;
    const double D = 2.0 * std::frexp(d, &e);            // significand in [1, 2)
    if (!(D < 2.0 - 0x1p-50)) return k;
    if (e - 1 < DIVK_ED_MIN || e - 1 > DIVK_ED_MAX) return k;   // quotients may leave the normal range
    k.yh = 1.0 / d;
    const double r = std::fma(-d, k.yh, 1.0);             // 1 - d*yh, exact
    k.yl = r / d;                                         // RN(r / d) = RN(1/d - yh)
    k.rspan = DIVK_HI_HI - DIVK_HI_LO;
    return k;
}

__host__ __device__ __forceinline__ unsigned divk_hiword(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return (unsigned)__double2hiint(x);
#else
    uint64_t b;
    std::memcpy(&b, &x, 8);
    return (unsigned)(b >> 32);
#endif
}
__host__ __device__ __forceinline__ unsigned divk_loword(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return (unsigned)__double2loint(x);
#else
    uint64_t b;
    std::memcpy(&b, &x, 8);
    return (unsigned)b;
#endif
}

// x / K.d, correctly rounded
__host__ __device__ __forceinline__ double divk(double x, const DivK &K) {
    const double q0 = std::fma(x, K.yh, x * K.yl);
    const double t = std::fma(q0, K.d, -x);
    double q = std::fma(-t, K.yh, q0);
    const unsigned hi = divk_hiword(x) & 0x7fffffffu, lo = divk_loword(x);
    const bool ok = (hi - DIVK_HI_LO) < K.rspan || (hi | lo) == 0u;
    if (__builtin_expect(!ok, 0)) q = x / K.d;
    return std::copysign(q, x);   // x = -0 with yl < 0: RN(x*yl) = +0 makes q0 = +0
}

// ---- unchecked form, certified per batch (the stencil kernels' interior paths) ----------
// divk_nc(x, K) is divk without its per-call range test: equal to x / K.d whenever x is in the
// certified range (or +-0) and K.rspan != 0.  A kernel certifies its numerators in bulk, not
// one by one, with the grain argument:
//   every double y with 2^-800 <= |y| is a multiple of 2^-852 (its ulp is), and so is 0.  A
//   sum, difference or small-integer multiple of such values is exact or rounds onto a grid
//   of spacing >= 2^-852 (results below 2^-800 are exact: they fit in 53 bits of 2^-852),
//   so it is again a multiple of 2^-852: zero, or at least 2^-852 > 2^-900 in magnitude.
//   With |y| < 2^990 and at most 16 such terms, |sum| < 2^994 < 2^1000.
// So a numerator formed by additions / small-integer scalings (exact factors 2, 3, 4, 6) of
// stored values that all passed DivNote (|y| in [2^-800, 2^990) or 0, finite) lies in the
// certified range; a numerator of any other form (a sum of quotients, ...) is noted itself.
// A failed note sends the work item (tile phase, cell) to the checked divk: bit-identical
// either way, the note only picks which one runs.
__host__ __device__ __forceinline__ double divk_nc(double x, const DivK &K) {
    const double q0 = std::fma(x, K.yh, x * K.yl);
    const double t = std::fma(q0, K.d, -x);
    return std::copysign(std::fma(-t, K.yh, q0), x);
}

__host__ __device__ __forceinline__ int divk_frexp_exp(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_frexp_exp(x);   // 0 for +-0 (and for inf / NaN: the lt test below)
#else
    int e = 0;
    if (std::isfinite(x)) (void)std::frexp(x, &e);
    return e;
#endif
}

// running certificate of the values noted: |y| in [2^-800, 2^990) or y = +-0, none NaN / inf
struct DivNote {
    int emin = 0;      // min frexp exponent (|y| >= 2^-800 <=> e >= -799; 0 for y = 0)
    bool lt = true;    // every |y| < 2^990 (false for inf, NaN)
    __host__ __device__ __forceinline__ void note(double y) {
        emin = std::min(emin, divk_frexp_exp(y));
        lt = lt && std::fabs(y) < 0x1p990;
    }
    __host__ __device__ __forceinline__ bool ok() const { return emin >= -799 && lt; }
};

}  // namespace rmt
