// Calibration: GPU time of trivial kernels at the pileup kernel's launch shape.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ __launch_bounds__(512) void k_empty(int* out) { if (threadIdx.x == 9999) out[0] = 1; }
__global__ __launch_bounds__(512) void k_lds(int* out) {
    __shared__ int s[11 * 1024];  // 44 KB
    s[threadIdx.x] = threadIdx.x;
    __syncthreads();
    if (s[(threadIdx.x + 1) & 511] == 9999) out[0] = 1;
}
__global__ __launch_bounds__(512) void k_vgpr(int* out, int n) {
    float a[96];
#pragma unroll
    for (int i = 0; i < 96; ++i) a[i] = (float)(threadIdx.x * i);
    for (int k = 0; k < n; ++k) {
#pragma unroll
        for (int i = 0; i < 96; ++i) a[i] = a[i] * 1.0001f + a[(i + 1) % 96];
    }
    float s = 0;
#pragma unroll
    for (int i = 0; i < 96; ++i) s += a[i];
    if (s == 12345.f) out[0] = 1;
}
__global__ void k_lds_vgpr(int* out, int n) {
    __shared__ int sm[11 * 1024];
    float a[96];
#pragma unroll
    for (int i = 0; i < 96; ++i) a[i] = (float)(threadIdx.x * i);
    for (int k = 0; k < n; ++k) {
#pragma unroll
        for (int i = 0; i < 96; ++i) a[i] = a[i] * 1.0001f + a[(i + 1) % 96];
    }
    float s = 0;
#pragma unroll
    for (int i = 0; i < 96; ++i) s += a[i];
    sm[threadIdx.x] = (int)s;
    __syncthreads();
    if (sm[(threadIdx.x + 3) & 511] == 12345) out[0] = 1;
}

template <class F>
float timeit(F f, hipStream_t st, int reps) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    for (int i = 0; i < 5; ++i) f();
    hipStreamSynchronize(st);
    hipEventRecord(a, st);
    for (int i = 0; i < reps; ++i) f();
    hipEventRecord(b, st);
    hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    return ms * 1000.f / reps;
}

int main() {
    int* d; CK(hipMalloc(&d, 64));
    hipStream_t st; CK(hipStreamCreate(&st));
    const int reps = 200;
    for (int blocks : {1, 256, 468, 1024}) {
        printf("blocks=%4d empty %.2f us | lds44K %.2f us | vgpr96 %.2f us | lds+vgpr %.2f us\n", blocks,
               timeit([&] { hipLaunchKernelGGL(k_empty, dim3(blocks), dim3(512), 0, st, d); }, st, reps),
               timeit([&] { hipLaunchKernelGGL(k_lds, dim3(blocks), dim3(512), 0, st, d); }, st, reps),
               timeit([&] { hipLaunchKernelGGL(k_vgpr, dim3(blocks), dim3(512), 0, st, d, 0); }, st, reps),
               timeit([&] { hipLaunchKernelGGL(k_lds_vgpr, dim3(blocks), dim3(512), 0, st, d, 0); }, st, reps));
    }
    // graph of one empty kernel
    hipGraph_t g; hipGraphExec_t ge;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    hipLaunchKernelGGL(k_empty, dim3(468), dim3(512), 0, st, d);
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    printf("graph replay empty 468x512: %.2f us\n", timeit([&] { hipGraphLaunch(ge, st); }, st, reps));
    return 0;
}
