// Standalone driver for the checked momentum kernels (debug tool, not shipped).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <cmath>
#include "../include/rmt.h"
int main(int argc, char **argv) {
    int N = argc > 1 ? atoi(argv[1]) : 129;
    size_t n = (size_t)N * N;
    std::vector<double> h(n);
    double *d[12];
    for (int k = 0; k < 12; ++k) { hipMalloc(&d[k], n * 8); hipMemset(d[k], 0, n * 8); }
    double dx = 1.0 / (N - 1);
    for (size_t c = 0; c < n; ++c) h[c] = 1.0;                       // phi = 1
    hipMemcpy(d[5], h.data(), n * 8, hipMemcpyHostToDevice);
    for (size_t c = 0; c < n; ++c) h[c] = (c % N) * dx;              // X1
    hipMemcpy(d[3], h.data(), n * 8, hipMemcpyHostToDevice);
    for (size_t c = 0; c < n; ++c) h[c] = (c / N) * dx;              // X2
    hipMemcpy(d[4], h.data(), n * 8, hipMemcpyHostToDevice);
    rmt_ctx *ctx;
    printf("create %d\n", rmt_ctx_create(N, N, 0, nullptr, &ctx));
    rmt_momentum_params P{};
    P.bc_kind = 1; P.lid = 1.0; P.rho_f = 1.0; P.mu_f = 1e-3; P.w_t = 2 * dx;
    P.dx = dx; P.dy = dx; P.dt = 3e-3; P.detg_clamp = 3.0;
    int s = rmt_momentum_step_rk4(ctx, &P, d[0], d[1], d[2], d[3], d[4], d[5], d[6], d[7], d[8],
                                  d[9], d[10], d[11]);
    printf("momentum status %d: %s\n", s, rmt_last_error());
    hipError_t e = hipDeviceSynchronize();
    printf("sync: %s\n", hipGetErrorString(e));
    return 0;
}
