// ubench_f64.hip -- measured fp64 VALU peak of one MI355X (the roof k_mom_stage is bound by).
// Every lane runs 8 independent v_fma_f64 chains (enough to cover the dependent-issue latency),
// 4 waves per SIMD, grid >> CUs; FLOP = 2 per FMA lane.  Prints TFLOP/s of the best of 5 runs.
//   hipcc -O3 --offload-arch=gfx950 -o tools/ubench_f64 tools/ubench_f64.hip && tools/ubench_f64
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int CH = 8, IT = 4096;

__global__ void __launch_bounds__(256) k_fma(double *out, double a, double b) {
    double x[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) x[c] = threadIdx.x * 1e-3 + c;
    for (int i = 0; i < IT; ++i) {
#pragma unroll
        for (int c = 0; c < CH; ++c) x[c] = __builtin_fma(x[c], a, b);
    }
    double s = 0.0;
#pragma unroll
    for (int c = 0; c < CH; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;   // vector store: keeps the chains live
}

int main() {
    int dev = 0, cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int blocks = cus * 16, threads = 256;
    double *out;
    if (hipMalloc(&out, sizeof(double) * blocks * threads) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    k_fma<<<blocks, threads>>>(out, 0.999999, 1e-9);
    hipDeviceSynchronize();
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
        hipEventRecord(e0);
        k_fma<<<blocks, threads>>>(out, 0.999999, 1e-9);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0.f;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    const double flop = 2.0 * CH * IT * (double)blocks * threads;
    printf("fp64 FMA VALU: %d CUs, %.3f ms, %.2f TFLOP/s\n", cus, best, flop / (best * 1e-3) / 1e12);
    hipFree(out);
    return 0;
}
