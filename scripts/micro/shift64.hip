// Throughput of 64-bit vs 32-bit shifts (v_lshlrev_b64 vs v_lshlrev_b32 / v_bfm_b32) on gfx950:
// 8 independent chains per lane, many waves per SIMD.  hipcc -O3 --offload-arch=gfx950 shift64.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s\n", hipGetErrorString(e)); return 1; } } while (0)
template <int MODE>
__global__ __launch_bounds__(256) void k(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 7 + i + seed;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint32_t s = a[i] & 31u;
            if (MODE == 0) a[i] = (uint32_t)(1ull << (s + 1)) ^ a[i];         // v_lshlrev_b64
            else if (MODE == 1) a[i] = (1u << s) ^ a[i];                    // v_lshlrev_b32
            else a[i] = __builtin_amdgcn_ubfe(a[i], s, 5) ^ (a[i] + 1u);    // v_bfe_u32 (+ add)
        }
    }
    uint32_t r = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) r ^= a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
int main() {
    uint32_t* d; CK(hipMalloc(&d, 4u << 22));
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    const int blocks = 256 * 8, iters = 4096;
    for (int mode = 0; mode < 3; ++mode) {
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(e0);
            if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, d, iters, 1u);
            if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, d, iters, 1u);
            if (mode == 2) hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, d, iters, 1u);
            hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1);
            const double winst = (double)blocks * 4 * iters * 8 * 3;  // ~3 VALU per chain step
            if (rep) printf("mode %d: %.3f ms, %.1f ps per wave-step\n", mode, ms, ms * 1e9 / ((double)blocks * 4 * iters * 8));
            (void)winst;
        }
    }
    return 0;
}
