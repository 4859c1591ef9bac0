// ubench_chain.hip -- latency calibration for the extrapolation chain kernel (k_ex_chain):
// dependent fp64 add chain, LDS ping-pong between two waves, and an LDS-fed fold.
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/ubench tools/ubench_chain.hip && /tmp/ubench
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_add_chain(const double *in, double *out, long long *cyc, int n) {
    double a = in[threadIdx.x], b = in[64 + threadIdx.x];
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < n; ++k) {
#pragma unroll
        for (int u = 0; u < 16; ++u) { a = a + b; asm volatile("" : "+v"(a)); }
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = a;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void k_pingpong(long long *cyc, int n) {
    __shared__ int flag;
    const int w = threadIdx.x >> 6;
    if (threadIdx.x == 0) flag = 0;
    __syncthreads();
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < n; ++k) {
        const int want = 2 * k + w;
        while (__hip_atomic_load(&flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != want) {}
        if ((threadIdx.x & 63) == 0)
            __hip_atomic_store(&flag, want + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) cyc[1] = t1 - t0;
}

__global__ void k_lds_fold(const double *in, double *out, long long *cyc, int reps) {
    __shared__ __attribute__((aligned(16))) double t[6][88];
    for (int s = threadIdx.x; s < 6 * 88; s += 64) (&t[0][0])[s] = in[s & 127];
    __syncthreads();
    double acc = 0;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < reps; ++r) {
        if (threadIdx.x < 6) {
            const double2 *p = (const double2 *)t[threadIdx.x];
#pragma unroll
            for (int c = 0; c < 5; ++c) {
                double2 v[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) v[u] = p[4 * c + u];
#pragma unroll
                for (int u = 0; u < 4; ++u) { acc += v[u].x; acc += v[u].y; }
            }
        }
        asm volatile("" : "+v"(acc));
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[2] = t1 - t0;
}

int main() {
    double *in, *out; long long *cyc;
    hipMalloc(&in, 1024 * 8); hipMalloc(&out, 1024 * 8); hipMalloc(&cyc, 64);
    double h[1024]; for (int i = 0; i < 1024; ++i) h[i] = 1.0 + i * 1e-3;
    hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
    long long c[3];
    const int n = 1000;
    for (int it = 0; it < 2; ++it) {
        k_add_chain<<<1, 64>>>(in, out, cyc, n);
        k_pingpong<<<1, 128>>>(cyc, n);
        k_lds_fold<<<1, 64>>>(in, out, cyc, n);
        hipDeviceSynchronize();
    }
    hipMemcpy(c, cyc, sizeof(c), hipMemcpyDeviceToHost);
    printf("dependent v_add_f64: %.2f cyc\n", (double)c[0] / (16.0 * n));
    printf("LDS ping-pong one-way handoff: %.1f cyc\n", (double)c[1] / (2.0 * n));
    printf("LDS-fed fold of 40 terms: %.1f cyc (%.2f per term)\n", (double)c[2] / n,
           (double)c[2] / n / 40);
    return 0;
}
