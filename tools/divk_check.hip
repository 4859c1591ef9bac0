// divk_check.hip -- host check of divk (pyrmt_amd/csrc/divk.hpp) against IEEE division.
//
//   divk_check [d ...]     (default: the stencil divisors of the configs' grids)
//
// For each divisor d: (1) the hardest operands -- x with x/d within ~2^-105 relative of a
// rounding midpoint, built by solving M*Dint = k (mod 2^s) for small k (M odd: the midpoint
// M 2^-53 or 2^-54 of a binade, Dint = d's 53-bit integer significand), scaled over the
// certified exponent range; (2) random operands of every exponent, both signs; (3) the
// special and out-of-range operands (zeros, subnormals, tiny/huge normals, inf, NaN).  The
// same hard cases also run through the single-reciprocal Markstein form
// (q0 = RN(x*yh) instead of the two-term product), which is NOT correct for every x: the
// count of its failures, and of the plain product x * RN(1/d), shows that the generator
// reaches operands next to a midpoint.
// Prints one line per divisor; exit status 1 if divk ever differs from x / d (bitwise).
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <cstdint>
#include <random>
#include <vector>
#include "../pyrmt_amd/csrc/divk.hpp"

using rmt::DivK;
typedef unsigned __int128 u128;

static uint64_t bits(double x) { uint64_t b; memcpy(&b, &x, 8); return b; }

static double naive(double x, const DivK &K) {   // Markstein with q0 = RN(x*yh)
    const double q0 = x * K.yh;
    const double t = std::fma(q0, K.d, -x);
    return std::fma(-t, K.yh, q0);
}

// inverse of an odd a modulo 2^64 (Newton)
static uint64_t inv64(uint64_t a) {
    uint64_t x = a;
    for (int i = 0; i < 6; ++i) x *= 2 - a * x;
    return x;
}

int main(int argc, char **argv) {
    std::vector<double> ds;
    for (int a = 1; a < argc; ++a) ds.push_back(strtod(argv[a], nullptr));
    if (ds.empty()) {
        const int Ns[] = {65, 129, 256, 512, 1024, 4096, 8192};
        for (int N : Ns) {
            const double dx = 1.0 / (N - 1);             // np.linspace spacing of [0, 1]
            ds.push_back(dx); ds.push_back(2 * dx); ds.push_back(6 * dx);
            ds.push_back(1.0 / N); ds.push_back(2.0 / N);   // MAC grid
        }
        ds.push_back(1.0 + 1e-12);                           // rho + 1e-12 at rho = 1
        ds.push_back(0.3); ds.push_back(0.7); ds.push_back(1.9999999999999); ds.push_back(3.0);
        // outside the certified divisor exponents (IEEE division): a tiny and a huge divisor
        ds.push_back(3.0e-9); ds.push_back(7.0e30); ds.push_back(0x1p-20); ds.push_back(0x1.8p60);
    }
    std::mt19937_64 rng(12345);
    long total_bad = 0;
    for (double d : ds) {
        const DivK K = rmt::divk_make(d);
        long n = 0, bad = 0, nbad = 0, nhard = 0, nmul = 0;
        auto check = [&](double x, bool hard) {
            const double q = rmt::divk(x, K), r = x / d;
            ++n;
            if (bits(q) != bits(r) && !(q != q && r != r)) {
                if (bad < 5) printf("  MISMATCH d=%a x=%a divk=%a ieee=%a\n", d, x, q, r);
                ++bad;
            }
            if (hard) {
                ++nhard;
                const double s = naive(x, K);
                if (bits(s) != bits(r)) ++nbad;
                if (bits(x * K.yh) != bits(r)) ++nmul;   // x * RN(1/d): wrong near midpoints
            }
        };
        int e;
        const double D = 2.0 * std::frexp(d, &e);
        const uint64_t Dint = (uint64_t)std::ldexp(D, 52);
        const int tz = __builtin_ctzll(Dint);
        const uint64_t Dodd = Dint >> tz, Dinv = inv64(Dodd);
        // (1) hard cases: M * Dint = X * 2^s + k with M odd in (2^53, 2^54), X in [2^52, 2^53)
        for (int s = 53; s <= 54; ++s) {
            for (long ko = -20001; ko <= 20001; ko += 2) {    // M odd: k / 2^tz odd
                const long k = ko * (1L << tz);
                const int sm = s - tz;                       // M * Dodd = ko (mod 2^sm)
                const uint64_t mask = (1ull << sm) - 1;
                const uint64_t M0 = ((uint64_t)ko * Dinv) & mask;
                if (sm < 40) continue;                       // D = 1 and nearby: exact
                for (u128 M = M0; M < ((u128)1 << 54); M += (u128)1 << sm) {
                    if (M <= ((u128)1 << 53)) {              // first M of the range
                        M += (((((u128)1 << 53) - M) >> sm) << sm);
                        if (M <= ((u128)1 << 53)) continue;
                    }
                    if (!(M & 1)) continue;
                    const u128 P = M * (u128)Dint;
                    const __int128 Xs = (__int128)P - k;
                    if (Xs % ((__int128)1 << s)) continue;
                    const __int128 X = Xs >> s;
                    if (X < ((__int128)1 << 52) || X >= ((__int128)1 << 53)) continue;
                    const double x = std::ldexp((double)(uint64_t)X, s - 105);
                    for (int rep = 0; rep < 3; ++rep) {
                        const int sc = (int)(rng() % 1800) - 850;       // 2^-850 .. 2^950
                        const double xs = std::ldexp(x, sc);
                        check(xs, true);
                        check(-xs, true);
                    }
                }
            }
        }
        // (2) random operands over the whole certified range and beyond
        for (int i = 0; i < 400000; ++i) {
            const uint64_t m = rng() & ((1ull << 52) - 1);
            const int ex = (int)(rng() % 2046) + 1;                   // every normal exponent
            uint64_t b = ((uint64_t)ex << 52) | m | ((rng() & 1) ? (1ull << 63) : 0);
            double x;
            memcpy(&x, &b, 8);
            check(x, false);
        }
        // (3) specials
        const double sp[] = {0.0, -0.0, 0x1p-1074, -0x1p-1074, 0x1p-1022, 0x1.8p-950, 0x1p-900,
                             0x1.fffffffffffffp-901, 0x1p1000, 0x1.fffffffffffffp999, 1e308,
                             INFINITY, -INFINITY, NAN, 1.0, d, -d, 3 * d, d / 3};
        for (double x : sp) check(x, false);
        // (4) divk_nc on numerators the kernels certify in bulk (divk.hpp, DivNote): sums and
        // small-integer combinations of noted values, including cancelling pairs near 2^-800
        long nnc = 0;
        auto stored = [&]() {
            const int r = (int)(rng() % 8);
            if (r == 0) return (rng() & 1) ? 0.0 : -0.0;
            int ex = r == 1 ? -799 + (int)(rng() % 4) : r == 2 ? 986 + (int)(rng() % 4)
                                                           : (int)(rng() % 1789) - 799;
            const double m = 0.5 + (double)(rng() >> 12) * 0x1p-53;   // [0.5, 1)
            return std::ldexp((rng() & 1) ? -m : m, ex);
        };
        for (int i = 0; i < 300000 && K.rspan; ++i) {   // rspan 0: divk_nc is never used
            double a = stored(), b = stored(), c = stored(), e4 = stored();
            if (i & 1) b = std::nextafter(a, (rng() & 1) ? INFINITY : -INFINITY);   // cancel
            rmt::DivNote nt;
            nt.note(a); nt.note(b); nt.note(c); nt.note(e4);
            if (!nt.ok()) continue;
            const double nums[3] = {a - b, 2 * a + 3 * b - 6 * c + e4, -a + 6 * b - 3 * c - 2 * e4};
            for (double x : nums) {
                const double q = rmt::divk_nc(x, K), r = x / d;
                ++nnc;
                if (bits(q) != bits(r)) {
                    if (bad < 5) printf("  NC MISMATCH d=%a x=%a nc=%a ieee=%a\n", d, x, q, r);
                    ++bad;
                }
            }
        }
        {   // the notes reject what they must
            rmt::DivNote t1, t2, t3, t4, t5;
            t1.note(0x1p-801); t2.note(0x1p990); t3.note(NAN); t4.note(-INFINITY); t5.note(0x1p-1074);
            if (t1.ok() || t2.ok() || t3.ok() || t4.ok() || t5.ok()) { printf("  DivNote accepts out of range\n"); ++bad; }
            rmt::DivNote t6;
            t6.note(0.0); t6.note(-0.0); t6.note(0x1p-800); t6.note(-0x1.fffffffffffffp989);
            if (!t6.ok()) { printf("  DivNote rejects the range's edges\n"); ++bad; }
        }
        printf("d=%.17g (%a) D=%.17g fast=%d: %ld operands, %ld mismatches; hard cases %ld, "
               "single-reciprocal Markstein wrong on %ld, x*RN(1/d) on %ld of them; %ld certified "
               "numerators unchecked\n", d, d, D, K.rspan != 0, n, bad, nhard, nbad, nmul, nnc);
        total_bad += bad;
    }
    printf("%s\n", total_bad ? "FAIL" : "OK: divk == IEEE division on every operand");
    return total_bad ? 1 : 0;
}
