// ubench_lat.hip -- dependent-latency probes for the chain kernel's inner sequences on gfx950:
// a chain of v_add_f64, a chain of LDS reads (ds_read_b64, address from the last value),
// and a readlane/DPP round trip, with 1 wave and with 12 waves on one CU.
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_lat.hip -o /tmp/ubench_lat && /tmp/ubench_lat
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_lat(double *out, long long *clk, int n, int mode) {
    __shared__ double lds[4096];
    for (int k = threadIdx.x; k < 4096; k += blockDim.x) lds[k] = (double)((k * 7 + 1) & 4095);
    __syncthreads();
    double a = out[threadIdx.x & 63], b = 1e-300;
    long long t0 = __builtin_amdgcn_s_memtime();
    if (mode == 0) {
        for (int k = 0; k < n; ++k) {
            a += b; a += b; a += b; a += b; a += b; a += b; a += b; a += b;
        }
    } else if (mode == 1) {
        int idx = threadIdx.x & 63;
        for (int k = 0; k < n; ++k) {
            const double v = lds[idx];
            idx = ((int)v) & 4095;
            a += v;
        }
    } else {
        for (int k = 0; k < n; ++k) {
            const int lo = __double2loint(a), hi = __double2hiint(a);
            const int l2 = __builtin_amdgcn_update_dpp(0, lo, 0x101, 0xf, 0xf, false);
            const int h2 = __builtin_amdgcn_update_dpp(0, hi, 0x101, 0xf, 0xf, false);
            a = __hiloint2double(h2, l2) + b;
        }
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = a;
    if ((threadIdx.x & 63) == 0) clk[blockIdx.x * 16 + (threadIdx.x >> 6)] = t1 - t0;
}

int main() {
    double *out; long long *clk;
    hipMalloc(&out, 1024 * sizeof(double)); hipMemset(out, 0, 1024 * sizeof(double));
    hipMalloc(&clk, 16 * sizeof(long long));
    const char *names[3] = {"v_add_f64 dependent", "ds_read_b64 dependent", "dpp row_shl + add"};
    for (int mode = 0; mode < 3; ++mode)
        for (int waves : {1, 4, 12}) {
            const int n = 2000;
            k_lat<<<1, 64 * waves>>>(out, clk, n, mode);
            hipDeviceSynchronize();
            k_lat<<<1, 64 * waves>>>(out, clk, n, mode);
            long long h[16];
            hipMemcpy(h, clk, sizeof(h), hipMemcpyDeviceToHost);
            const double per = mode == 0 ? 8.0 * n : (double)n;
            printf("%-24s waves %2d: %.1f clk per op (wave 0)\n", names[mode], waves, h[0] / per);
        }
    return 0;
}
