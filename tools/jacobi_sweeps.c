/* jacobi_sweeps.c -- how many Jacobi sweeps of the reference's own fit arithmetic does the
 * narrow-band extrapolation (functions.py:48-163) need before it reaches the serial result
 * bit for bit?  ("next round" item 1.)
 *
 * The fits, their windows and their acceptance are value-independent (the known set alone
 * decides them), so a layer is a fixed lower-triangular system in raster order: fit t reads
 * the initially known cells of its 9x9 window and the earlier accepted fits inside it.  A
 * Jacobi sweep recomputes EVERY fit at once from the previous sweep's values with the
 * reference's exact arithmetic (sums in window order, Cramer on absolute coordinates,
 * utils.py:134-166; glibc exp weights, as Numba lowers them).  A sweep that changes no bit is
 * the serial result (the rounded system is triangular: by induction on DAG order its fixed
 * point is unique).  This probe measures the number of sweeps to that point, the fits still
 * wrong after each sweep, and the exact DAG depth, from three seeds:
 *   seed 0: zeros;  seed 1: the advected map value at the target (X̂, what the chain's
 *   residue variant predicted from);  seed 2: today's parallel mode (the same fits solved
 *   in centred integer offsets, oracle ex_mode 2, serial).
 *
 *   gcc -O2 -o /tmp/jacobi_sweeps tools/jacobi_sweeps.c -lm
 *   /tmp/jacobi_sweeps N [deform]                      synthetic disc map (as extrap_dag.c)
 *   /tmp/jacobi_sweeps N file X1.bin X2.bin phi.bin    a recorded state (N*N raw f64 each)
 * Output: one JSON object on stdout.  TEST/ANALYSIS INFRASTRUCTURE, not on the product path.
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define IDX(j, i) ((size_t)(j) * nx + (i))

typedef struct { int cell; int src0; int nsrc; int layer; double x0, y0; double A[9]; } Fit;
typedef struct { int cell; int fit; double w, xi, yi; } Src;   /* fit < 0: initially known */

static void solve3(const double *A, const double *b, double *x) {   /* utils.py:134-166 */
    double det = (A[0] * (A[4] * A[8] - A[5] * A[7]) - A[1] * (A[3] * A[8] - A[5] * A[6]) +
                  A[2] * (A[3] * A[7] - A[4] * A[6]));
    if (fabs(det) < 1e-15) { x[0] = x[1] = x[2] = 0.0; return; }
    double d0 = (b[0] * (A[4] * A[8] - A[5] * A[7]) - A[1] * (b[1] * A[8] - A[5] * b[2]) +
                 A[2] * (b[1] * A[7] - A[4] * b[2]));
    double d1 = (A[0] * (b[1] * A[8] - A[5] * b[2]) - b[0] * (A[3] * A[8] - A[5] * A[6]) +
                 A[2] * (A[3] * b[2] - b[1] * A[6]));
    double d2 = (A[0] * (A[4] * b[2] - b[1] * A[7]) - A[1] * (A[3] * b[2] - b[1] * A[6]) +
                 b[0] * (A[3] * A[7] - A[4] * A[6]));
    x[0] = d0 / det; x[1] = d1 / det; x[2] = d2 / det;
}

static int load(const char *path, double *a, size_t n) {
    FILE *f = fopen(path, "rb");
    if (!f) return -1;
    size_t r = fread(a, 8, n, f);
    fclose(f);
    return r == n ? 0 : -1;
}

int main(int argc, char **argv) {
    int N = argc > 1 ? atoi(argv[1]) : 4096, ML = 3;
    int ny = N, nx = N;
    size_t n = (size_t)ny * nx;
    double *X1 = malloc(n * 8), *X2 = malloc(n * 8), *phi = malloc(n * 8);
    double dx = 1.0 / (nx - 1), dy = 1.0 / (ny - 1);   /* np.linspace(0, 1, N) spacing */
    const char *state = "synthetic";
    if (argc > 2 && !strcmp(argv[2], "file")) {
        if (argc < 6 || load(argv[3], X1, n) || load(argv[4], X2, n) || load(argv[5], phi, n)) {
            fprintf(stderr, "cannot read the state files\n");
            return 1;
        }
        state = argv[3];
    } else {
        int deform = argc > 2 ? atoi(argv[2]) : 0;
        for (int j = 0; j < ny; ++j)
            for (int i = 0; i < nx; ++i) {
                double x = dx * i, y = dy * j, a = x, b = y;
                if (deform) {
                    a = x + 0.05 * sin(2 * M_PI * y) * cos(M_PI * x);
                    b = y + 0.03 * sin(2 * M_PI * x);
                }
                double ph = sqrt((a - 0.6) * (a - 0.6) + (b - 0.5) * (b - 0.5)) - 0.2;
                size_t c = IDX(j, i);
                phi[c] = ph; X1[c] = ph <= 0 ? a : 0.0; X2[c] = ph <= 0 ? b : 0.0;
            }
        state = deform ? "synthetic deformed disc" : "synthetic disc (identity map)";
    }
    unsigned char *known = malloc(n), *target = malloc(n);
    int *fid = malloc(n * sizeof(int));
    for (size_t k = 0; k < n; ++k) { known[k] = phi[k] < 0; fid[k] = -1; }
    const double r = 4 * sqrt(dx * dx + dy * dy), r2 = r * r;
    size_t capf = 1 << 16, caps = 1 << 22, nf = 0, ns = 0;
    Fit *F = malloc(capf * sizeof(Fit));
    Src *S = malloc(caps * sizeof(Src));
    /* the fits in the reference's order, with their sources (the serial sweep's known sets) */
    for (int layer = 0; layer < ML; ++layer) {
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
                double A00 = 0, A01 = 0, A02 = 0, A11 = 0, A12 = 0, A22 = 0;
                size_t s0 = ns;
                int count = 0;
                int jlo = j - 4 > 0 ? j - 4 : 0, jhi = j + 5 < ny ? j + 5 : ny;
                int ilo = i - 4 > 0 ? i - 4 : 0, ihi = i + 5 < nx ? i + 5 : nx;
                for (int jj = jlo; jj < jhi; ++jj)
                    for (int ii = ilo; ii < ihi; ++ii) {
                        if (!known[IDX(jj, ii)]) continue;
                        double xi = dx * ii, yi = dy * jj, ddx = xi - x0, ddy = yi - y0;
                        double d2 = ddx * ddx + ddy * ddy;
                        if (!(d2 <= r2)) continue;
                        double w = exp(-d2 / r2);
                        if (ns == caps) { caps *= 2; S = realloc(S, caps * sizeof(Src)); }
                        S[ns++] = (Src){(int)IDX(jj, ii), fid[IDX(jj, ii)], w, xi, yi};
                        double wa0 = w * 1.0, wa1 = w * xi, wa2 = w * yi;
                        A00 += wa0 * 1.0; A01 += wa0 * xi; A02 += wa0 * yi;
                        A11 += wa1 * xi; A12 += wa1 * yi; A22 += wa2 * yi;
                        ++count;
                    }
                double A[9] = {A00, A01, A02, A01, A11, A12, A02, A12, A22};
                double det = (A[0] * (A[4] * A[8] - A[5] * A[7]) - A[1] * (A[3] * A[8] - A[5] * A[6]) +
                              A[2] * (A[3] * A[7] - A[4] * A[6]));
                if (count < 3 || !(fabs(det) > 1e-10)) { ns = s0; continue; }
                if (nf == capf) { capf *= 2; F = realloc(F, capf * sizeof(Fit)); }
                Fit *f = &F[nf];
                f->cell = (int)IDX(j, i); f->src0 = (int)s0; f->nsrc = (int)(ns - s0);
                f->layer = layer; f->x0 = x0; f->y0 = y0;
                memcpy(f->A, A, sizeof A);
                fid[IDX(j, i)] = (int)nf++;
                known[IDX(j, i)] = 1;
            }
    }
    /* one fit's value from the given fit values (initially known cells: the input map) */
    #define FIT(t, V1, V2, out1, out2) do {                                                   \
        const Fit *f_ = &F[t];                                                              \
        double B10 = 0, B11 = 0, B12 = 0, B20 = 0, B21 = 0, B22 = 0;                        \
        for (int k_ = 0; k_ < f_->nsrc; ++k_) {                                             \
            const Src *s_ = &S[f_->src0 + k_];                                              \
            double b1 = s_->fit < 0 ? X1[s_->cell] : V1[s_->fit];                           \
            double b2 = s_->fit < 0 ? X2[s_->cell] : V2[s_->fit];                           \
            double wa0 = s_->w * 1.0, wa1 = s_->w * s_->xi, wa2 = s_->w * s_->yi;           \
            B10 += wa0 * b1; B11 += wa1 * b1; B12 += wa2 * b1;                              \
            B20 += wa0 * b2; B21 += wa1 * b2; B22 += wa2 * b2;                              \
        }                                                                                   \
        double bb1[3] = {B10, B11, B12}, bb2[3] = {B20, B21, B22}, c1[3], c2[3];           \
        solve3(f_->A, bb1, c1); solve3(f_->A, bb2, c2);                                     \
        out1 = c1[0] + c1[1] * f_->x0 + c1[2] * f_->y0;                                     \
        out2 = c2[0] + c2[1] * f_->x0 + c2[2] * f_->y0;                                     \
    } while (0)
    double *E1 = malloc(nf * 8), *E2 = malloc(nf * 8);   /* the serial (reference) result */
    for (size_t t = 0; t < nf; ++t) FIT(t, E1, E2, E1[t], E2[t]);
    /* the exact DAG depth (longest chain of fits, each reading the previous one) */
    int *hop = calloc(nf, sizeof(int)), depth = 0;
    for (size_t t = 0; t < nf; ++t) {
        int h = 0;
        for (int k = 0; k < F[t].nsrc; ++k) {
            int s = S[F[t].src0 + k].fit;
            if (s >= 0 && hop[s] + 1 > h) h = hop[s] + 1;
        }
        hop[t] = h;
        if (h > depth) depth = h;
    }
    /* seed 2: the centred (parallel-mode) restatement, serial in raster order */
    double *P1 = malloc(nf * 8), *P2 = malloc(nf * 8);
    for (size_t t = 0; t < nf; ++t) {
        const Fit *f = &F[t];
        double S0 = 0, Sx = 0, Sy = 0, Sxx = 0, Sxy = 0, Syy = 0;
        int ti = f->cell % nx, tj = f->cell / nx;
        for (int k = 0; k < f->nsrc; ++k) {
            const Src *s = &S[f->src0 + k];
            double w = s->w, a = s->cell % nx - ti, b = s->cell / nx - tj;
            S0 += w; Sx += w * a; Sy += w * b; Sxx += w * a * a; Sxy += w * a * b; Syy += w * b * b;
        }
        double c00 = Sxx * Syy - Sxy * Sxy, c01 = Sx * Syy - Sxy * Sy, c02 = Sx * Sxy - Sxx * Sy;
        double dc = S0 * c00 - Sx * c01 + Sy * c02;
        double y0c = c00 / dc, y1c = -c01 / dc, y2c = c02 / dc, v1 = 0, v2 = 0;
        for (int k = 0; k < f->nsrc; ++k) {
            const Src *s = &S[f->src0 + k];
            double a = s->cell % nx - ti, b = s->cell / nx - tj;
            double beta = s->w * (y0c + y1c * a + y2c * b);
            double b1 = s->fit < 0 ? X1[s->cell] : P1[s->fit], b2 = s->fit < 0 ? X2[s->cell] : P2[s->fit];
            v1 += beta * b1; v2 += beta * b2;
        }
        P1[t] = v1; P2[t] = v2;
    }
    double maxrel = 0;
    for (size_t t = 0; t < nf; ++t) {
        double d = fabs(P1[t] - E1[t]) / fmax(fabs(E1[t]), 1e-300);
        if (d > maxrel) maxrel = d;
    }
    printf("{\"N\": %d, \"state\": \"%s\", \"fits\": %zu, \"dag_depth\": %d, "
           "\"parallel_seed_max_rel\": %.3e, \"seeds\": {", N, state, nf, depth, maxrel);
    double *V1 = malloc(nf * 8), *V2 = malloc(nf * 8), *W1 = malloc(nf * 8), *W2 = malloc(nf * 8);
    const char *names[3] = {"zeros", "advected_value", "parallel_mode"};
    for (int seed = 0; seed < 3; ++seed) {
        for (size_t t = 0; t < nf; ++t) {
            V1[t] = seed == 0 ? 0.0 : seed == 1 ? X1[F[t].cell] : P1[t];
            V2[t] = seed == 0 ? 0.0 : seed == 1 ? X2[F[t].cell] : P2[t];
        }
        int sweeps = 0, first_exact = -1;
        /* wrong fits (vs the serial result) after sweeps 1, 2, 4, ... */
        char trail[4096];
        int tl = 0;
        trail[0] = 0;
        for (;;) {
            size_t changed = 0, wrong = 0;
            for (size_t t = 0; t < nf; ++t) {
                FIT(t, V1, V2, W1[t], W2[t]);
                if (memcmp(&W1[t], &V1[t], 8) || memcmp(&W2[t], &V2[t], 8)) ++changed;
                if (memcmp(&W1[t], &E1[t], 8) || memcmp(&W2[t], &E2[t], 8)) ++wrong;
            }
            double *x;
            x = V1; V1 = W1; W1 = x;
            x = V2; V2 = W2; W2 = x;
            ++sweeps;
            if (wrong == 0 && first_exact < 0) first_exact = sweeps;
            if ((sweeps & (sweeps - 1)) == 0 && tl < 3800)
                tl += snprintf(trail + tl, sizeof trail - tl, "%s[%d, %zu]", tl ? ", " : "",
                               sweeps, wrong);
            if (changed == 0 || sweeps > 4 * depth + 16) break;
        }
        printf("%s\"%s\": {\"sweeps_to_no_change\": %d, \"first_exact_sweep\": %d, "
               "\"wrong_after_sweep\": [%s]}", seed ? ", " : "", names[seed], sweeps, first_exact,
               trail);
        fflush(stdout);
    }
    printf("}}\n");
    return 0;
}
