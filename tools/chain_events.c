/* chain_events.c -- CPU model of the chain's event fold (tools only; not the product).
 *
 * The chain folds every fit's six weighted sums in the reference's window order
 * (functions.py:128-138).  The event fold replaces that sequential fold by a walk over a
 * few "events", using a PREDICTED partial-sum path s^_m built before the chain from the
 * exact static products and predicted values of the fit's dynamic sources:
 *
 *   before the first dynamic term the actual and predicted sums are equal (the static prefix P);
 *   at a dynamic term m (or a static "event" step m) the actual sum is formed for real:
 *       s = RN((s^_{m-1} + d) + t_m),  d' = s - s^_m       (s, s^_m in one binade: exact)
 *   between events every static step satisfies RN(x^ + d) = RN(x^) + d -- the shift by d,
 *   a multiple of ulp(E) with E the binade at the last event, commutes with the rounding --
 *   provided s^_m stays in a binade <= E, is not a rounding tie, and |d| <= dist(s^_m, the
 *   binade's edges) - ulp(s^_m) (the block margin M);
 *   the fold's result is s^_n + d.
 *
 * This model runs the reference's serial extrapolation (rmto_extrapolate's loop), and for
 * every accepted fit builds the path from the previous map's values (sim.hip's ex_pred),
 * walks the events with the actual values, and compares the six sums with the exact fold
 * bit for bit.  It reports mismatches (must be 0), fallbacks (a check failed: the chain then
 * folds exactly), and event counts.
 *
 *   gcc -O2 -ffp-contract=off -fno-fast-math -shared -fPIC tools/chain_events.c -o /tmp/ce.so
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define IDX(j, i) ((size_t)(j) * nx + (i))

static inline uint64_t bits(double x) { uint64_t u; memcpy(&u, &x, 8); return u; }
static inline int expf_(double x) { return (int)((bits(x) >> 52) & 0x7ff); }
static inline double ulp_of(double x) { return ldexp(1.0, expf_(x) - 1075); }

/* distance of |s| to the edges of its binade minus one ulp: the largest |d| for which the
 * shift argument holds at this step; < 0 means never */
static inline double margin(double s)
{
    const int e = expf_(s);
    if (e == 0 || e >= 0x7fd) return -1.0;
    const double a = fabs(s), lo = ldexp(1.0, e - 1023), hi = 2.0 * lo, u = ulp_of(s);
    const double d = fmin(a - lo, hi - a);
    return d - u;
}

typedef struct {
    long fits, fits_dyn, fallback, mismatch, fb_binade, fb_margin, fb_path;
    long ev_hist[64];       /* max events per lane */
    long post_hist[64];     /* max events per lane from the critical dynamic term on */
    long nd_hist[96];
    long b_after_crit_hist[64];
    double worst_rel_d;     /* max |d| / M over passed checks */
    long u_hist[96], upost_hist[96], u_fb, u_mm;
    long dr_hist[96], dops_hist[96], d_fb, d_mm;
} Stats;

/* one sum: terms t[0..n) (static value or dynamic: dyn[m] != 0, product from cf[m]*v[m]),
 * predicted values vp[m] for the dynamic ones.  Returns 0 ok (out = event result),
 * 1 fallback.  ev: events, post: events at m >= mcrit. */
static int event_sum(int n, const int *dyn, const double *cf, const double *v, const double *vp,
                     const double *st, int mcrit, double *out, int *ev, int *post, int *bcrit,
                     Stats *S)
{
    double sh[96];
    int isev[96];
    double M[96];   /* block margin after event m (valid where isev) */
    int m0 = 0;
    while (m0 < n && !dyn[m0]) ++m0;
    double P = 0.0;
    for (int m = 0; m < m0; ++m) P += st[m];
    *ev = 0; *post = 0; *bcrit = 0;
    if (m0 == n) { *out = P; return 0; }
    /* predicted path and events */
    double prev = P;
    int E = 0, last = -1;
    for (int m = m0; m < n; ++m) {
        const double t = dyn[m] ? cf[m] * vp[m] : st[m];
        const double s = prev + t;
        /* TwoSum error of the predicted step */
        const double bb = s - prev, err = (prev - (s - bb)) + (t - bb);
        sh[m] = s;
        const int e = expf_(s);
        const double u = ulp_of(s);
        const int tie = fabs(err) == 0.5 * u || fabs(err) == 0.25 * u;
        const double mg = margin(s);
        if (e == 0 || e >= 0x7fd) { S->fb_path++; return 1; }
        isev[m] = dyn[m] || e > E || (tie && e == E) || !(mg > 0.0);
        if (isev[m]) { E = e; last = m; M[m] = INFINITY; }
        else M[last] = fmin(M[last], mg);
        prev = s;
    }
    /* walk with the actual values */
    double d = 0.0;
    for (int m = m0; m < n; ++m) {
        if (!isev[m]) continue;
        ++*ev;
        if (m >= mcrit) { ++*post; if (!dyn[m]) ++*bcrit; }
        const double sp = (m == m0 ? P : sh[m - 1]) + d;
        const double t = dyn[m] ? cf[m] * v[m] : st[m];
        const double s = sp + t;
        if ((bits(s) >> 52) != (bits(sh[m]) >> 52)) { S->fb_binade++; return 1; }
        d = s - sh[m];
        if (!(fabs(d) <= M[m])) { S->fb_margin++; return 1; }
        if (M[m] < INFINITY && M[m] > 0 && fabs(d) / M[m] > S->worst_rel_d)
            S->worst_rel_d = fabs(d) / M[m];
    }
    *out = sh[n - 1] + d;
    return 0;
}


/* the six sums with one event set (the union over the sums: positions where any sum needs
 * an event are events for all -- what the GPU walk does, uniform across lanes).  Returns 0 ok
 * (out[6]), 1 fallback.  nev: union events, npost: union events at m >= mcrit. */
static int event_union(int n, const int *dyn, double cf[3][96], double va[2][96],
                       double vp[2][96], double st[6][96], int mcrit, double *out, int *nev,
                       int *npost, Stats *S)
{
    static double sh[6][96], M[6][96];
    int isev[96];
    int m0 = 0;
    while (m0 < n && !dyn[m0]) ++m0;
    double P[6];
    for (int k = 0; k < 6; ++k) { P[k] = 0.0; for (int m = 0; m < m0; ++m) P[k] += st[k][m]; }
    *nev = 0; *npost = 0;
    if (m0 == n) { for (int k = 0; k < 6; ++k) out[k] = P[k]; return 0; }
    double prev[6];
    int E[6], last = -1;
    for (int k = 0; k < 6; ++k) { prev[k] = P[k]; E[k] = 0; }
    for (int m = m0; m < n; ++m) {
        int ev = dyn[m];
        double s[6], mg[6];
        for (int k = 0; k < 6; ++k) {
            const double t = dyn[m] ? cf[k % 3][m] * vp[k < 3 ? 0 : 1][m] : st[k][m];
            s[k] = prev[k] + t;
            const double bb = s[k] - prev[k], err = (prev[k] - (s[k] - bb)) + (t - bb);
            const int e = expf_(s[k]);
            const double u = ulp_of(s[k]);
            const int tie = fabs(err) == 0.5 * u || fabs(err) == 0.25 * u;
            mg[k] = margin(s[k]);
            if (e == 0 || e >= 0x7fd) { S->fb_path++; return 1; }
            if (e > E[k] || (tie && e == E[k]) || !(mg[k] > 0.0)) ev = 1;
            sh[k][m] = s[k];
            prev[k] = s[k];
        }
        isev[m] = ev;
        for (int k = 0; k < 6; ++k) {
            if (ev) { E[k] = expf_(s[k]); M[k][m] = INFINITY; }
            else M[k][last] = fmin(M[k][last], mg[k]);
        }
        if (ev) last = m;
    }
    double d[6] = {0, 0, 0, 0, 0, 0};
    for (int m = m0; m < n; ++m) {
        if (!isev[m]) continue;
        ++*nev;
        if (m >= mcrit) ++*npost;
        for (int k = 0; k < 6; ++k) {
            const double sp = (m == m0 ? P[k] : sh[k][m - 1]) + d[k];
            const double t = dyn[m] ? cf[k % 3][m] * va[k < 3 ? 0 : 1][m] : st[k][m];
            const double s = sp + t;
            if ((bits(s) >> 52) != (bits(sh[k][m]) >> 52)) { S->fb_binade++; return 1; }
            d[k] = s - sh[k][m];
            if (!(fabs(d[k]) <= M[k][m])) { S->fb_margin++; return 1; }
        }
    }
    for (int k = 0; k < 6; ++k) out[k] = sh[k][n - 1] + d[k];
    return 0;
}


/* The post-critical walk with the chain-side re-basing ("delta trick"): the predicted path
 * (all dynamic values predicted) is built chip-wide; the dynamic terms before the critical
 * one (mcrit, the fit's latest source in chain order) are real events processed before the
 * critical arrival; after it, every NON-critical dynamic term m (its value known before the
 * arrival) is folded into the shift instead of being an event:
 *     s'_m = RN(s^_{m-1} + t_m),  D_m = s'_m - s^_m      (before the arrival)
 *     at the arrival: d += D_m                            (one exact add)
 * valid when s'_m, s^_m and the block's binade E coincide, y_m = s^_{m-1} + t_m is no tie,
 * and |d| + sum|D| stays within the margins.  Critical-path ops after the arrival are
 * counted: 3 per real event (the critical term, predicted-path events), 1 per folded-in D,
 * 1 final add. */
long g_why[8];
static int event_delta(int n, const int *dyn, double cf[3][96], double va[2][96],
                       double vp[2][96], double st[6][96], int mcrit, double *out, int *nreal,
                       int *nops, Stats *S)
{
    static double sh[6][96];
    int isev[96];
    int m0 = 0;
    while (m0 < n && !dyn[m0]) ++m0;
    double P[6];
    for (int k = 0; k < 6; ++k) { P[k] = 0.0; for (int m = 0; m < m0; ++m) P[k] += st[k][m]; }
    *nreal = 0; *nops = 0;
    if (m0 == n) { for (int k = 0; k < 6; ++k) out[k] = P[k]; return 0; }
    /* predicted path: events = dyn terms before or at mcrit, binade-ups, ties, bad margins */
    double prev[6];
    int E[6];
    for (int k = 0; k < 6; ++k) { prev[k] = P[k]; E[k] = 0; }
    for (int m = m0; m < n; ++m) {
        int ev = dyn[m] && m <= mcrit;
        for (int k = 0; k < 6; ++k) {
            const double t = dyn[m] ? cf[k % 3][m] * vp[k < 3 ? 0 : 1][m] : st[k][m];
            const double s = prev[k] + t;
            const double bb = s - prev[k], err = (prev[k] - (s - bb)) + (t - bb);
            const int e = expf_(s);
            const double u = ulp_of(s);
            const int tie = fabs(err) == 0.5 * u || fabs(err) == 0.25 * u;
            if (e == 0 || e >= 0x7fd) { S->fb_path++; return 1; }
            if (e > E[k] || (tie && e == E[k]) || !(margin(s) > 0.0)) ev = 1;
            sh[k][m] = s;
            prev[k] = s;
        }
        isev[m] = ev;
        if (ev) for (int k = 0; k < 6; ++k) E[k] = expf_(sh[k][m]);
    }
    /* chain side, before the arrival: the non-critical dynamic terms after mcrit.  A term
     * that cannot be folded into the shift becomes a real event (union over the sums). */
    static double Dm[6][96], Mg[6][96];
    for (int k = 0; k < 6; ++k) E[k] = 0;
    for (int m = m0; m < n; ++m) {
        if (isev[m]) { for (int k = 0; k < 6; ++k) E[k] = expf_(sh[k][m]); continue; }
        int bad = 0;
        for (int k = 0; k < 6; ++k) {
            Dm[k][m] = 0.0;
            Mg[k][m] = margin(sh[k][m]);
            if (!dyn[m] || m <= mcrit) continue;
            const double pm = sh[k][m - 1];
            const double t = cf[k % 3][m] * va[k < 3 ? 0 : 1][m];
            const double s2 = pm + t;
            const double bb = s2 - pm, err = (pm - (s2 - bb)) + (t - bb);
            const double u = ulp_of(s2);
            const int tie = fabs(err) == 0.5 * u || fabs(err) == 0.25 * u;
            if (expf_(s2) != E[k] || expf_(sh[k][m]) != E[k] || (bits(s2) >> 63) != (bits(sh[k][m]) >> 63)
                || (tie && expf_(s2) == E[k])) bad = 1;
            if (expf_(s2) != E[k]) g_why[0]++;
            if (expf_(sh[k][m]) != E[k]) g_why[1]++;
            if (tie) g_why[2]++;
            g_why[3]++;
            Dm[k][m] = s2 - sh[k][m];
            Mg[k][m] = fmin(Mg[k][m], margin(s2));
        }
        if (dyn[m] && m > mcrit) { g_why[4]++; if (bad) g_why[5]++; }
        if (bad) {
            isev[m] = 1;
            for (int k = 0; k < 6; ++k) E[k] = expf_(sh[k][m]);
        }
    }
    /* the walk with the actual values; ops counted from mcrit on */
    double d[6] = {0, 0, 0, 0, 0, 0};
    double used[6] = {0, 0, 0, 0, 0, 0};   /* sum |D| since the last event */
    for (int m = m0; m < n; ++m) {
        const int post = m >= mcrit;
        if (isev[m]) {
            if (post) { ++*nreal; *nops += 3; }
            for (int k = 0; k < 6; ++k) {
                const double sp = (m == m0 ? P[k] : sh[k][m - 1]) + d[k];
                const double t = dyn[m] ? cf[k % 3][m] * va[k < 3 ? 0 : 1][m] : st[k][m];
                const double s = sp + t;
                if ((bits(s) >> 52) != (bits(sh[k][m]) >> 52)) { S->fb_binade++; return 1; }
                d[k] = s - sh[k][m];
                used[k] = fabs(d[k]);
            }
            continue;
        }
        int anyD = 0;
        for (int k = 0; k < 6; ++k) {
            /* the step is exact under the shift d (+ the D's so far) if within the margin */
            if (!(used[k] <= Mg[k][m])) { S->fb_margin++; return 1; }
            if (Dm[k][m] != 0.0 || (dyn[m] && m > mcrit)) anyD = 1;
            d[k] += Dm[k][m];
            used[k] += fabs(Dm[k][m]);
        }
        if (anyD && post) *nops += 1;
    }
    *nops += 1;
    for (int k = 0; k < 6; ++k) out[k] = sh[k][n - 1] + d[k];
    return 0;
}

long ce_run(const double *X1, const double *X2, const double *phi, const double *P1,
            const double *P2, int ny, int nx, double dx, double dy, int max_layers,
            double *X1e, double *X2e, long *stats_out, int pred_mode)
{
    Stats S;
    memset(&S, 0, sizeof S);
    size_t n = (size_t)ny * nx;
    memcpy(X1e, X1, n * sizeof(double));
    memcpy(X2e, X2, n * sizeof(double));
    unsigned char *known = malloc(n), *target = malloc(n), *stat = malloc(n);
    int *key = malloc(n * sizeof(int));   /* chain key of a filled cell: (j + 5L) * 8 + L */
    for (size_t k = 0; k < n; ++k) { known[k] = phi[k] < 0; stat[k] = known[k]; key[k] = -1; }
    double r = 4 * sqrt(dx * dx + dy * dy);
    const double r2 = r * r;
    long filled = 0;
    for (int layer = 0; layer < max_layers; ++layer) {
        int any = 0;
        memset(target, 0, n);
        for (int j = 1; j < ny - 1; ++j)
            for (int i = 1; i < nx - 1; ++i) {
                if (known[IDX(j, i)]) continue;
                for (int dj = -1; dj <= 1 && !target[IDX(j, i)]; ++dj)
                    for (int di = -1; di <= 1; ++di)
                        if (known[IDX(j + dj, i + di)]) { target[IDX(j, i)] = 1; any = 1; break; }
            }
        if (!any) break;
        for (int j = 1; j < ny - 1; ++j)
            for (int i = 1; i < nx - 1; ++i) {
                if (!target[IDX(j, i)]) continue;
                double x0 = dx * i, y0 = dy * j;
                double Aw00 = 0, Aw01 = 0, Aw02 = 0, Aw11 = 0, Aw12 = 0, Aw22 = 0;
                double B[6] = {0, 0, 0, 0, 0, 0};
                int count = 0;
                int dyn[96];
                double cf[3][96], va[2][96], vp[2][96], stv[6][96];
                long ck[96];
                int jlo = j - 4 > 0 ? j - 4 : 0, jhi = j + 5 < ny ? j + 5 : ny;
                int ilo = i - 4 > 0 ? i - 4 : 0, ihi = i + 5 < nx ? i + 5 : nx;
                for (int jj = jlo; jj < jhi; ++jj)
                    for (int ii = ilo; ii < ihi; ++ii) {
                        if (!known[IDX(jj, ii)]) continue;
                        double xi = dx * ii, yi = dy * jj;
                        double ddx = xi - x0, ddy = yi - y0;
                        double d2 = ddx * ddx + ddy * ddy;
                        if (!(d2 <= r2)) continue;
                        double w = exp(-d2 / r2);
                        double b1 = X1e[IDX(jj, ii)], b2 = X2e[IDX(jj, ii)];
                        double wa0 = w * 1.0, wa1 = w * xi, wa2 = w * yi;
                        B[0] += wa0 * b1; B[1] += wa1 * b1; B[2] += wa2 * b1;
                        B[3] += wa0 * b2; B[4] += wa1 * b2; B[5] += wa2 * b2;
                        Aw00 += wa0 * 1.0; Aw01 += wa0 * xi; Aw02 += wa0 * yi;
                        Aw11 += wa1 * xi; Aw12 += wa1 * yi; Aw22 += wa2 * yi;
                        dyn[count] = !stat[IDX(jj, ii)];
                        ck[count] = dyn[count] ? key[IDX(jj, ii)] : -1;
                        cf[0][count] = wa0; cf[1][count] = wa1; cf[2][count] = wa2;
                        va[0][count] = b1; va[1][count] = b2;
                        vp[0][count] = pred_mode == 1 ? 0.0 : P1[IDX(jj, ii)];
                        vp[1][count] = pred_mode == 1 ? 0.0 : P2[IDX(jj, ii)];
                        for (int k = 0; k < 6; ++k) stv[k][count] = cf[k % 3][count] * (k < 3 ? b1 : b2);
                        ++count;
                    }
                if (count < 3) continue;
                double A[9] = {Aw00, Aw01, Aw02, Aw01, Aw11, Aw12, Aw02, Aw12, Aw22};
                double det = (A[0] * (A[4] * A[8] - A[5] * A[7])
                            - A[1] * (A[3] * A[8] - A[5] * A[6])
                            + A[2] * (A[3] * A[7] - A[4] * A[6]));
                if (!(fabs(det) > 1e-10)) continue;
                /* event fold of the six sums */
                int nd = 0, mcrit = count;
                long kmax = -1;
                for (int m = 0; m < count; ++m)
                    if (dyn[m]) { ++nd; if (ck[m] > kmax) { kmax = ck[m]; mcrit = m; } }
                S.fits++;
                if (nd) S.fits_dyn++;
                S.nd_hist[nd < 95 ? nd : 95]++;
                int fb = 0, evmax = 0, postmax = 0, bcmax = 0;
                for (int k = 0; k < 6 && !fb; ++k) {
                    double o;
                    int ev, post, bc;
                    fb = event_sum(count, dyn, cf[k % 3], va[k < 3 ? 0 : 1], vp[k < 3 ? 0 : 1],
                                   stv[k], mcrit, &o, &ev, &post, &bc, &S);
                    if (!fb && bits(o) != bits(B[k])) {
                        S.mismatch++;
                        if (S.mismatch < 10)
                            fprintf(stderr, "MISMATCH fit (%d,%d) L%d sum %d: %.17g vs %.17g\n",
                                    j, i, layer, k, o, B[k]);
                    }
                    if (ev > evmax) evmax = ev;
                    if (post > postmax) postmax = post;
                    if (bc > bcmax) bcmax = bc;
                }
                {
                    double uo[6];
                    int nev, npost;
                    if (event_union(count, dyn, cf, va, vp, stv, mcrit, uo, &nev, &npost, &S)) S.u_fb++;
                    else {
                        for (int k = 0; k < 6; ++k) if (bits(uo[k]) != bits(B[k])) S.u_mm++;
                        S.u_hist[nev < 95 ? nev : 95]++;
                        S.upost_hist[npost < 95 ? npost : 95]++;
                    }
                }
                {
                    double uo[6];
                    int nr, nops;
                    if (event_delta(count, dyn, cf, va, vp, stv, mcrit, uo, &nr, &nops, &S)) S.d_fb++;
                    else {
                        for (int k = 0; k < 6; ++k) if (bits(uo[k]) != bits(B[k])) S.d_mm++;
                        S.dr_hist[nr < 95 ? nr : 95]++;
                        S.dops_hist[nops < 95 ? nops : 95]++;
                    }
                }
                if (fb) S.fallback++;
                else {
                    S.ev_hist[evmax < 63 ? evmax : 63]++;
                    S.post_hist[postmax < 63 ? postmax : 63]++;
                    S.b_after_crit_hist[bcmax < 63 ? bcmax : 63]++;
                }
                /* the reference's solve (utils.py:134-166) on the exact sums */
                double c1[3], c2[3];
                for (int q = 0; q < 2; ++q) {
                    const double *b = B + 3 * q;
                    double *c = q ? c2 : c1;
                    const double inv = 1.0 / det;
                    c[0] = (b[0] * (A[4] * A[8] - A[5] * A[7]) - A[1] * (b[1] * A[8] - A[5] * b[2])
                            + A[2] * (b[1] * A[7] - A[4] * b[2])) * inv;
                    c[1] = (A[0] * (b[1] * A[8] - A[5] * b[2]) - b[0] * (A[3] * A[8] - A[5] * A[6])
                            + A[2] * (A[3] * b[2] - b[1] * A[6])) * inv;
                    c[2] = (A[0] * (A[4] * b[2] - b[1] * A[7]) - A[1] * (A[3] * b[2] - b[1] * A[6])
                            + b[0] * (A[3] * A[7] - A[4] * A[6])) * inv;
                }
                X1e[IDX(j, i)] = c1[0] + c1[1] * x0 + c1[2] * y0;
                X2e[IDX(j, i)] = c2[0] + c2[1] * x0 + c2[2] * y0;
                known[IDX(j, i)] = 1;
                key[IDX(j, i)] = (j + 5 * layer) * 8 + layer;
                ++filled;
            }
    }
    free(known); free(target); free(stat); free(key);
    long *o = stats_out;
    o[0] = S.fits; o[1] = S.fits_dyn; o[2] = S.fallback; o[3] = S.mismatch;
    o[4] = S.fb_binade; o[5] = S.fb_margin; o[6] = S.fb_path;
    memcpy(o + 8, S.ev_hist, 64 * sizeof(long));
    memcpy(o + 72, S.post_hist, 64 * sizeof(long));
    memcpy(o + 136, S.nd_hist, 96 * sizeof(long));
    memcpy(o + 232, S.b_after_crit_hist, 64 * sizeof(long));
    memcpy(o + 296, S.u_hist, 96 * sizeof(long));
    memcpy(o + 392, S.upost_hist, 96 * sizeof(long));
    o[488] = S.u_fb; o[489] = S.u_mm;
    memcpy(o + 490, S.dr_hist, 96 * sizeof(long));
    memcpy(o + 586, S.dops_hist, 96 * sizeof(long));
    o[682] = S.d_fb; o[683] = S.d_mm;
    double w = S.worst_rel_d;
    memcpy(o + 7, &w, 8);
    return filled;
}
