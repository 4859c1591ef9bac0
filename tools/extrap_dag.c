/* extrap_dag.c -- dependency structure of the exact extrapolation chain (functions.py:48-163)
 * on a disc band, for sizing k_ex_chain.  Runs the serial sweep and records, per fit, every
 * earlier fit inside its included window ("dynamic" terms) and how many included terms follow
 * each of them in window order (the adds that must wait for that value).
 *   gcc -O2 -o /tmp/extrap_dag tools/extrap_dag.c -lm && /tmp/extrap_dag 4096 3 [deform]
 * Prints: targets/accepted per layer, DAG depth (fits), and the weighted critical path
 * sum over a chain of (adds after the dependency + SOLVE) for SOLVE = 10 dependent ops. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int main(int argc, char **argv) {
    int N = argc > 1 ? atoi(argv[1]) : 4096, ML = argc > 2 ? atoi(argv[2]) : 3;
    int deform = argc > 3 ? atoi(argv[3]) : 0;
    int ny = N, nx = N;
    double dx = 1.0 / (nx - 1), dy = 1.0 / (ny - 1);
    size_t n = (size_t)ny * nx;
    double *X1 = malloc(n * 8), *X2 = malloc(n * 8);
    unsigned char *known = calloc(n, 1), *target = calloc(n, 1);
    int *fid = malloc(n * sizeof(int));   /* fit id of a fitted cell, -1 otherwise */
    for (int j = 0; j < ny; ++j)
        for (int i = 0; i < nx; ++i) {
            double x = dx * i, y = dy * j, a = x, b = y;
            if (deform) { a = x + 0.05 * sin(2 * M_PI * y) * cos(M_PI * x); b = y + 0.03 * sin(2 * M_PI * x); }
            double phi = sqrt((a - 0.6) * (a - 0.6) + (b - 0.5) * (b - 0.5)) - 0.2;
            size_t c = (size_t)j * nx + i;
            known[c] = phi < 0; X1[c] = known[c] ? a : 0; X2[c] = known[c] ? b : 0; fid[c] = -1;
        }
    double r = 4 * sqrt(dx * dx + dy * dy), r2 = r * r;
    int cap = 1 << 20;
    double *fin = malloc(cap * 8);      /* weighted finish time */
    int *lev = malloc(cap * sizeof(int)), *lev1 = malloc(cap * sizeof(int)), *lay = malloc(cap * sizeof(int));
    double *fin1 = malloc(cap * 8);
    long s_inc = 0, s_after1 = 0, s_dyn1 = 0; int maxlev1[16] = {0}; double maxfin1[16] = {0};
    int nf = 0, maxlev = 0;
    long *fkey = malloc(sizeof(long) * cap); int *pa = malloc(4 * (cap * 20)), *pb = malloc(4 * (cap * 20)); long np = 0;
    double maxfin = 0, SOLVE = 10;
    long hist[100] = {0};
    long ndyn = 0;
    for (int L = 0; L < ML; ++L) {
        int nt = 0, na = 0;
        memset(target, 0, n);
        for (int j = 1; j < ny - 1; ++j)
            for (int i = 1; i < nx - 1; ++i) {
                size_t c = (size_t)j * nx + i;
                if (known[c]) continue;
                for (int dj = -1; dj <= 1 && !target[c]; ++dj)
                    for (int di = -1; di <= 1; ++di)
                        if (known[c + (long)dj * nx + di]) { target[c] = 1; break; }
                nt += target[c];
            }
        for (int j = 1; j < ny - 1; ++j)
            for (int i = 1; i < nx - 1; ++i) {
                size_t c = (size_t)j * nx + i;
                if (!target[c]) continue;
                double x0 = dx * i, y0 = dy * j;
                double A00 = 0, A01 = 0, A02 = 0, A11 = 0, A12 = 0, A22 = 0;
                int count = 0, q = 0, dq[81], dsrc[81], nd = 0, incq[81];
                for (int jj = j - 4; jj <= j + 4; ++jj)
                    for (int ii = i - 4; ii <= i + 4; ++ii, ++q) {
                        incq[q] = 0;
                        if (jj < 0 || jj >= ny || ii < 0 || ii >= nx) continue;
                        size_t cc = (size_t)jj * nx + ii;
                        if (!known[cc]) continue;
                        double xi = dx * ii, yi = dy * jj, ax = xi - x0, ay = yi - y0;
                        double d2 = ax * ax + ay * ay;
                        if (!(d2 <= r2)) continue;
                        double w = exp(-d2 / r2), wa1 = w * xi, wa2 = w * yi;
                        A00 += w * 1.0; A01 += w * xi; A02 += w * yi;
                        A11 += wa1 * xi; A12 += wa1 * yi; A22 += wa2 * yi;
                        ++count; incq[q] = 1;
                        if (fid[cc] >= 0) { dq[nd] = q; dsrc[nd] = fid[cc]; ++nd; }
                    }
                if (count < 3) continue;
                double det = A00 * (A11 * A22 - A12 * A12) - A01 * (A01 * A22 - A12 * A02) +
                             A02 * (A01 * A12 - A11 * A02);
                if (!(fabs(det) > 1e-10)) continue;
                /* weighted finish: wait for each dependency, then the included adds after it */
                double f = 0; int lv = 0;
                for (int k = 0; k < nd; ++k) {
                    int after = 0;
                    for (int qq = dq[k] + 1; qq < 81; ++qq) after += incq[qq];
                    double t = fin[dsrc[k]] + after + 1;
                    if (t > f) f = t;
                    if (lev[dsrc[k]] + 1 > lv) lv = lev[dsrc[k]] + 1;
                    if (k == nd - 1 || 1) { }
                }
                /* the latest-finishing dependency's suffix histogram */
                if (nd) {
                    int best = 0; double bt = -1;
                    for (int k = 0; k < nd; ++k) if (fin[dsrc[k]] > bt) { bt = fin[dsrc[k]]; best = k; }
                    int after = 0;
                    for (int qq = dq[best] + 1; qq < 81; ++qq) after += incq[qq];
                    hist[after < 99 ? after : 99]++;
                }
                ndyn += nd;
                for (int k = 0; k < nd && np < cap * 20; ++k) { pa[np] = nf; pb[np] = dsrc[k]; ++np; }
                fkey[nf] = ((long)(j + 5 * L) * ML + L) * nx + i;
                { int lv1 = 0, qf = 81, nd1 = 0; double f1 = 0;
                  for (int k = 0; k < nd; ++k) if (lay[dsrc[k]] == L) {
                      ++nd1; if (dq[k] < qf) qf = dq[k];
                      if (lev1[dsrc[k]] + 1 > lv1) lv1 = lev1[dsrc[k]] + 1;
                      int after = 0; for (int qq = dq[k] + 1; qq < 81; ++qq) after += incq[qq];
                      if (fin1[dsrc[k]] + after + 1 > f1) f1 = fin1[dsrc[k]] + after + 1; }
                  for (int qq = 0; qq < 81; ++qq) { s_inc += incq[qq]; if (qq >= qf) s_after1 += incq[qq]; }
                  s_dyn1 += nd1; lev1[nf] = lv1; fin1[nf] = f1 + SOLVE; lay[nf] = L;
                  if (lv1 > maxlev1[L]) maxlev1[L] = lv1; if (f1 + SOLVE > maxfin1[L]) maxfin1[L] = f1 + SOLVE; }
                f += SOLVE;
                fin[nf] = f; lev[nf] = lv;
                if (f > maxfin) maxfin = f;
                if (lv > maxlev) maxlev = lv;
                fid[c] = nf++; known[c] = 1; ++na;
                X1[c] = 0; X2[c] = 0;
            }
        printf("layer %d: targets %d accepted %d\n", L, nt, na);
    }
    printf("fits %d, avg dynamic deps %.1f, depth (levels) %d, weighted critical path %.0f adds "
           "(%.1f per level)\n", nf, (double)ndyn / nf, maxlev + 1, maxfin, maxfin / (maxlev + 1));
    printf("layer-sequential: avg included %.1f, avg same-layer deps %.1f, avg terms from first same-layer dep %.1f\n", (double)s_inc/nf, (double)s_dyn1/nf, (double)s_after1/nf);
    { int tot = 0; double tf = 0; for (int L = 0; L < ML; ++L) { printf("  layer %d depth %d weighted %.0f\n", L, maxlev1[L] + 1, maxfin1[L]); tot += maxlev1[L] + 1; tf += maxfin1[L]; }
      printf("  sum of layer depths %d, weighted %.0f\n", tot, tf); }
    { /* chain order (j + 5L, L, i) over all targets: max distance fit -> source */
      long *srt = malloc(sizeof(long) * nf); int *rank = malloc(4 * nf);
      for (int k = 0; k < nf; ++k) srt[k] = fkey[k] * 65536L + k;
      int cmp(const void *a, const void *b) { long x = *(long *)a, y = *(long *)b; return x < y ? -1 : x > y; }
      qsort(srt, nf, sizeof(long), cmp);
      for (int k = 0; k < nf; ++k) rank[srt[k] & 65535 ? srt[k] % 65536 : srt[k] % 65536] = k;
      long md = 0; for (long p = 0; p < np; ++p) { long d = rank[pa[p]] - rank[pb[p]]; if (d > md) md = d; if (d <= 0) printf("non-topological!\n"); }
      printf("max chain distance fit->source: %ld\n", md); }
    printf("suffix length after latest dependency (hist):");
    for (int k = 0; k < 60; ++k) if (hist[k]) printf(" %d:%ld", k, hist[k]);
    printf("\n");
    return 0;
}
