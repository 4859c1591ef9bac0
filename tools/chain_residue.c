/* chain_residue.c -- feasibility probe for a constant-latency fold after the chain's last source.
 *
 * A fit's 6 sums (functions.py:128-138) are sequential: s <- fl(s + t) over the window in
 * raster order.  Once the last-arriving source c is folded in (a = fl(S_pre + p_c)), the rest
 * is F(a) = fl(..fl(fl(a + t1) + t2).. + tn) with every t known beforehand.  If the partial
 * sums of F(a) and F(a') stay in the same binades and a - a' is a multiple of 2G (G = the
 * largest ulp on the path), rounding commutes with the shift: F(a) = F(a') + (a - a').  So
 * with a predicted start a^ (S_pre + cf * X^, X^ = the input map at c) the fold can run BEFORE
 * c arrives, once per residue r of a mod 2G (2^(m+1) residues, m = binade growth), and the
 * arrival only picks the residue and adds the shift -- if the slack checks pass.
 *
 * This probe runs the serial sweep on a deformed disc map, emulates that scheme for every fit
 * (critical source = the dynamic source latest in chain order (j + 5L, L, i)), checks that
 * the shortcut reproduces the sequential fold bit for bit whenever its checks pass, and
 * prints the pass rate and the lanes (sum over the 6 sums of 2^(m+1)) it needs.
 *   gcc -O2 -o /tmp/chain_residue tools/chain_residue.c -lm && /tmp/chain_residue 4096 3
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static int ex_of(double v) { int e; frexp(v, &e); return e; }   /* v in [2^(e-1), 2^e) */

typedef struct { double F, lo, hi; } Res;

/* fold t[0..n) from s, tracking the slack of every partial sum inside its binade */
static Res fold(double s, const double *t, int n) {
    Res r = {0, INFINITY, INFINITY};
    for (int k = 0; k < n; ++k) {
        s = s + t[k];
        if (!(s > 0)) { r.lo = -1; r.hi = -1; }
        const int e = ex_of(s);
        const double b = ldexp(1.0, e - 1), g = ldexp(1.0, e - 53);
        r.lo = fmin(r.lo, s - b - g);
        r.hi = fmin(r.hi, 2 * b - g - s);
    }
    r.F = s;
    return r;
}


/* the k_ex_chain fast fold's acceptance (VAR 35): residues mod 8 ulp, near test on the top 14
 * mantissa bits, max binade <= e0 + 2, |d| <= 2^(Emin - 15); returns 1 and *out on success */
static unsigned hiw(double v) { unsigned long long b; memcpy(&b, &v, 8); return (unsigned)(b >> 32); }
static unsigned low(double v) { unsigned long long b; memcpy(&b, &v, 8); return (unsigned)b; }
static double mk(unsigned h, unsigned l) { unsigned long long b = ((unsigned long long)h << 32) | l; double v; memcpy(&v, &b, 8); return v; }
static int kernel_fast(double ah, double a, const double *t, int nt, double *out) {
    unsigned hA = hiw(ah), lA = low(ah), hB = hiw(a), lB = low(a);
    unsigned rr = lB & 7u;
    double f = mk(hA, (lA & ~7u) | rr);
    unsigned mx = hA, mn = hA; int nr = 0;
    for (int j = 0; j < nt; ++j) {
        f += t[j];
        unsigned h = hiw(f);
        if (h > mx) mx = h; if (h < mn) mn = h;
        nr = nr || ((h + 0x40u) & 0xFFF80u) == 0u;
    }
    unsigned e0 = hA & 0x7FF00000u, emn = (mn >> 20) & 0x7FFu;
    int same = (hB & 0xFFF00000u) == (hA & 0xFFF00000u) && (hA >> 31) == 0u && e0 >= (0x100u << 20) && e0 <= (0x700u << 20);
    int okb = !nr && (mx >> 31) == 0u && (mx & 0x7FF00000u) <= e0 + (2u << 20) && emn > 64u;
    double del = mk(hB, lB & ~7u) - mk(hA, lA & ~7u);
    double lim = mk((emn - 15u) << 20, 0u);
    if (!(same && okb && fabs(del) <= lim)) return 0;
    *out = f + del;
    return 1;
}

int main(int argc, char **argv) {
    int N = argc > 1 ? atoi(argv[1]) : 4096, ML = argc > 2 ? atoi(argv[2]) : 3;
    int ny = N, nx = N;
    double dx = 1.0 / (nx - 1), dy = 1.0 / (ny - 1);
    size_t n = (size_t)ny * nx;
    double *X1 = malloc(n * 8), *X2 = malloc(n * 8), *P1 = malloc(n * 8), *P2 = malloc(n * 8);
    unsigned char *known = calloc(n, 1), *target = calloc(n, 1);
    int *lay = malloc(n * sizeof(int));
    for (int j = 0; j < ny; ++j)
        for (int i = 0; i < nx; ++i) {
            double x = dx * i, y = dy * j;
            double a = x + 0.05 * sin(2 * M_PI * y) * cos(M_PI * x), b = y + 0.03 * sin(2 * M_PI * x);
            double phi = sqrt((a - 0.6) * (a - 0.6) + (b - 0.5) * (b - 0.5)) - 0.2;
            size_t c = (size_t)j * nx + i;
            known[c] = phi < 0; X1[c] = known[c] ? a : 0; X2[c] = known[c] ? b : 0;
            P1[c] = a; P2[c] = b;          /* predictor: the smooth map itself */
            lay[c] = -1;
        }
    double r = 4 * sqrt(dx * dx + dy * dy), r2 = r * r;
    long nfit = 0, nstatic = 0, npass = 0, nlane_ok = 0, nbad = 0, hist[9] = {0};
    long sum_fail_exp = 0, sum_fail_slack = 0, sum_fail_neg = 0, kfits = 0, kok = 0, kbad = 0;
    for (int L = 0; L < ML; ++L) {
        memset(target, 0, n);
        for (int j = 1; j < ny - 1; ++j)
            for (int i = 1; i < nx - 1; ++i) {
                size_t c = (size_t)j * nx + i;
                if (known[c]) continue;
                for (int dj = -1; dj <= 1 && !target[c]; ++dj)
                    for (int di = -1; di <= 1; ++di)
                        if (known[c + (long)dj * nx + di]) { target[c] = 1; break; }
            }
        for (int j = 1; j < ny - 1; ++j)
            for (int i = 1; i < nx - 1; ++i) {
                size_t c = (size_t)j * nx + i;
                if (!target[c]) continue;
                double x0 = dx * i, y0 = dy * j;
                double cf[81][3], b1[81], b2[81], p1[81], p2[81];
                int cnt = 0, crit = -1;
                long ckey = -1;
                double A[6] = {0};
                for (int jj = j - 4; jj <= j + 4; ++jj)
                    for (int ii = i - 4; ii <= i + 4; ++ii) {
                        if (jj < 0 || jj >= ny || ii < 0 || ii >= nx) continue;
                        size_t cc = (size_t)jj * nx + ii;
                        if (!known[cc]) continue;
                        double xi = dx * ii, yi = dy * jj;
                        double d2 = (xi - x0) * (xi - x0) + (yi - y0) * (yi - y0);
                        if (d2 > r2) continue;
                        double w = exp(-d2 / r2);
                        cf[cnt][0] = w * 1.0; cf[cnt][1] = w * xi; cf[cnt][2] = w * yi;
                        b1[cnt] = X1[cc]; b2[cnt] = X2[cc]; p1[cnt] = P1[cc]; p2[cnt] = P2[cc];
                        A[0] += w * 1.0 * 1.0; A[1] += w * 1.0 * xi; A[2] += w * 1.0 * yi;
                        A[3] += w * xi * xi; A[4] += w * xi * yi; A[5] += w * yi * yi;
                        if (lay[cc] >= 0) {
                            long key = ((long)(jj + 5 * lay[cc]) * 16 + lay[cc]) * nx + ii;
                            if (key > ckey) { ckey = key; crit = cnt; }
                        }
                        ++cnt;
                    }
                if (cnt < 3) continue;
                double M0 = A[0], M1 = A[1], M2 = A[2], M4 = A[3], M5 = A[4], M8 = A[5];
                double det = M0 * (M4 * M8 - M5 * M5) - M1 * (M1 * M8 - M5 * M2) + M2 * (M1 * M5 - M4 * M2);
                if (!(fabs(det) > 1e-10)) continue;
                ++nfit;
                /* the 6 sums: the shortcut against the sequential fold */
                if (crit < 0) { ++nstatic; }
                else {
                    int lanes = 0, ok = 1, kall = 1;
                    for (int k = 0; k < 6; ++k) {
                        const double *bb = k < 3 ? b1 : b2, *pp = k < 3 ? p1 : p2;
                        double s = 0.0, t[81];
                        for (int q = 0; q < crit; ++q) s += cf[q][k % 3] * bb[q];
                        const double a = s + cf[crit][k % 3] * bb[crit];
                        const double ah = s + cf[crit][k % 3] * pp[crit];
                        int nt = 0;
                        double up = ah;
                        for (int q = crit + 1; q < cnt; ++q) {
                            t[nt] = cf[q][k % 3] * bb[q];
                            if (t[nt] > 0) up += t[nt];
                            ++nt;
                        }
                        double seq = a;
                        for (int q = 0; q < nt; ++q) seq += t[q];
                        { double kr; if (kernel_fast(ah, a, t, nt, &kr)) { if (memcmp(&kr, &seq, 8)) ++kbad; } else kall = 0; }
                        if (!(ah > 0) || !(a > 0)) { ok = 0; ++sum_fail_neg; continue; }
                        up *= 1 + 1e-12;
                        const int e0 = ex_of(ah), em = ex_of(up), m = em - e0;
                        const double g0 = ldexp(1.0, e0 - 53), G2 = ldexp(1.0, em - 52);
                        lanes += 2 << m;
                        if (ex_of(a) != e0) { ok = 0; ++sum_fail_exp; continue; }
                        const double ahi = floor(ah / G2) * G2, ahi_true = floor(a / G2) * G2;
                        const long rr = (long)((a - ahi_true) / g0);
                        const double ar = ahi + rr * g0;
                        Res R = fold(ar, t, nt);
                        const double d = ahi_true - ahi;
                        if (!(R.lo >= 0 && -R.lo <= d && d <= R.hi)) { ok = 0; ++sum_fail_slack; continue; }
                        const double fast = R.F + d;
                        if (memcmp(&fast, &seq, 8) != 0) {
                            ++nbad;
                            if (nbad < 5) fprintf(stderr, "MISMATCH j=%d i=%d k=%d %.17g %.17g\n", j, i, k, fast, seq);
                        }
                    }
                    int lb = 0;
                    while ((8 << lb) < lanes && lb < 8) ++lb;
                    hist[lb]++;
                    if (lanes <= 64) ++nlane_ok;
                    if (ok) ++npass;
                    ++kfits; if (kall) ++kok;
                }
                /* the fit itself (serial semantics) */
                double B1[3] = {0}, B2[3] = {0};
                for (int q = 0; q < cnt; ++q)
                    for (int k = 0; k < 3; ++k) { B1[k] += cf[q][k] * b1[q]; B2[k] += cf[q][k] * b2[q]; }
                double Aw[3][3] = {{M0, M1, M2}, {M1, M4, M5}, {M2, M5, M8}};
                double o[2];
                for (int h = 0; h < 2; ++h) {
                    const double *b = h ? B2 : B1;
                    double id = 1.0 / det;
                    double xs = (b[0] * (Aw[1][1] * Aw[2][2] - Aw[1][2] * Aw[2][1]) - Aw[0][1] * (b[1] * Aw[2][2] - Aw[1][2] * b[2]) + Aw[0][2] * (b[1] * Aw[2][1] - Aw[1][1] * b[2])) * id;
                    double ys = (Aw[0][0] * (b[1] * Aw[2][2] - Aw[1][2] * b[2]) - b[0] * (Aw[1][0] * Aw[2][2] - Aw[1][2] * Aw[2][0]) + Aw[0][2] * (Aw[1][0] * b[2] - b[1] * Aw[2][0])) * id;
                    double zs = (Aw[0][0] * (Aw[1][1] * b[2] - b[1] * Aw[2][1]) - Aw[0][1] * (Aw[1][0] * b[2] - b[1] * Aw[2][0]) + b[0] * (Aw[1][0] * Aw[2][1] - Aw[1][1] * Aw[2][0])) * id;
                    o[h] = xs + ys * x0 + zs * y0;
                }
                X1[c] = o[0]; X2[c] = o[1]; known[c] = 1; lay[c] = L;
            }
    }
    printf("N=%d fits %ld (no dynamic source %ld); shortcut passes %ld (%.1f%% of dynamic), "
           "lanes<=64 %ld; mismatches %ld\n", N, nfit, nstatic, npass,
           100.0 * npass / (nfit - nstatic), nlane_ok, nbad);
    printf("kernel fast fold: %ld of %ld fits (%.1f%%), wrong results %ld\n", kok, kfits, 100.0 * kok / kfits, kbad);
    printf("per-sum failures: binade of a %ld, slack %ld, non-positive %ld\n", sum_fail_exp,
           sum_fail_slack, sum_fail_neg);
    printf("lanes histogram (<=8, 16, 32, 64, 128, 256, ...):");
    for (int b = 0; b < 9; ++b) printf(" %ld", hist[b]);
    printf("\n");
    return 0;
}
