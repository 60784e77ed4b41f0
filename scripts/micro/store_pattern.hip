// Store-pattern microbenchmark for k_pileup_solo's output stream (C5): per position 5 int32
// count planes (stride L), cov int32, ent/sec f64 = 36 B.  Each wave sweeps a contiguous run of
// tiles.  Modes: 0 dword stores, 64 positions per tile; 1 16-B stores, 4 positions per lane
// (256 per tile); 2 mode 1 with non-temporal stores; 3 one contiguous array of the same bytes
// (upper bound); 4 mode 1 with L = 2 mod 4 (misaligned odd planes -> 8-B stores).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef double f64x2 __attribute__((ext_vector_type(2)));

template <int MODE>
__global__ __launch_bounds__(256) void k_store(int32_t* counts, int32_t* cov, double* ent, double* sec, int64_t L,
                                               int64_t n_tiles, int64_t run, int64_t total_waves, int stagger) {
    const int lane = threadIdx.x & 63;
    const int64_t w = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int64_t n_runs = (n_tiles + run - 1) / run;
    for (int64_t r = w; r < n_runs; r += total_waves) {
    const int64_t t0 = r * run, t1 = t0 + run < n_tiles ? t0 + run : n_tiles;
    const int64_t len = t1 - t0;
    const int64_t rot = stagger ? (w * 7919) % (len > 0 ? len : 1) : 0;
    for (int64_t i = 0; i < len; ++i) {
        int64_t t = t0 + i + rot;
        if (t >= t1) t -= len;
        if (MODE == 0) {
            const int64_t P = t * 64 + lane;
            if (P < L) {
#pragma unroll
                for (int c = 0; c < 5; ++c) counts[c * L + P] = 0;
                cov[P] = 0;
                ent[P] = 1.0;
                sec[P] = 1.0;
            }
        } else if (MODE == 3) {
            // 36 B x 256 positions = 9216 B per tile = 576 uint4, 9 per lane
            uint4* d = (uint4*)counts + t * 576;
            const uint4 z = make_uint4(0, 0, 0, 0);
#pragma unroll
            for (int i = 0; i < 9; ++i) d[i * 64 + lane] = z;
        } else {
            const int64_t P = t * 256 + 4 * lane;
            if (P + 4 <= L) {
                const uint4 z = make_uint4(0, 0, 0, 0);
                const double2 one = make_double2(1.0, 1.0);
#pragma unroll
                for (int c = 0; c < 5; ++c) {
                    int32_t* d = counts + c * L + P;
                    if (((uintptr_t)d & 15) == 0) {
                        if (MODE == 2) __builtin_nontemporal_store(u32x4{0, 0, 0, 0}, (u32x4*)d);
                        else *(uint4*)d = z;
                    } else {
                        ((uint2*)d)[0] = make_uint2(0, 0);
                        ((uint2*)d)[1] = make_uint2(0, 0);
                    }
                }
                if (MODE == 2) {
                    const f64x2 o2 = {1.0, 1.0};
                    __builtin_nontemporal_store(u32x4{0, 0, 0, 0}, (u32x4*)(cov + P));
                    __builtin_nontemporal_store(o2, (f64x2*)(ent + P));
                    __builtin_nontemporal_store(o2, (f64x2*)(ent + P) + 1);
                    __builtin_nontemporal_store(o2, (f64x2*)(sec + P));
                    __builtin_nontemporal_store(o2, (f64x2*)(sec + P) + 1);
                } else {
                    *(uint4*)(cov + P) = z;
                    ((double2*)(ent + P))[0] = one;
                    ((double2*)(ent + P))[1] = one;
                    ((double2*)(sec + P))[0] = one;
                    ((double2*)(sec + P))[1] = one;
                }
            }
        }
    }
    }
}

template <int MODE>
void run_mode(int32_t* counts, int32_t* cov, double* ent, double* sec, int64_t L) {
    const int64_t per = MODE == 0 ? 64 : 256;
    const int64_t n_tiles = (L + per - 1) / per;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int64_t waves = 8192;
    for (int stagger = 0; stagger < 2; ++stagger)
        for (int64_t run : {(n_tiles + waves - 1) / waves, 64L, 16L, 4L, 1L}) {
            if (stagger && run < 16) continue;
            const int64_t n_runs = (n_tiles + run - 1) / run;
            int64_t tw = waves < n_runs ? waves : n_runs;
            const int blocks = (int)((tw + 3) / 4);
            tw = (int64_t)blocks * 4;
            auto go = [&] {
                hipLaunchKernelGGL(k_store<MODE>, dim3(blocks), dim3(256), 0, 0, counts, cov, ent, sec, L, n_tiles, run,
                                   tw, stagger);
            };
            go();
            hipDeviceSynchronize();
            hipEventRecord(a);
            for (int i = 0; i < 5; ++i) go();
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            ms /= 5;
            printf("mode %d L %ld run %5ld stagger %d: %.3f ms  %.0f GB/s\n", MODE, (long)L, (long)run, stagger, ms,
                   36.0 * L / ms / 1e6);
        }
}

int main() {
    const int64_t Lmax = 248956424;
    int32_t *counts, *cov;
    double *ent, *sec;
    if (hipMalloc(&counts, 9 * Lmax * 4 + 65536) != hipSuccess) return 1;
    if (hipMalloc(&cov, Lmax * 4) != hipSuccess) return 1;
    if (hipMalloc(&ent, Lmax * 8) != hipSuccess) return 1;
    if (hipMalloc(&sec, Lmax * 8) != hipSuccess) return 1;
    run_mode<0>(counts, cov, ent, sec, 248956424);
    run_mode<1>(counts, cov, ent, sec, 248956424);
    run_mode<3>(counts, cov, ent, sec, 248956424);
    run_mode<4>(counts, cov, ent, sec, 248956422);
    return 0;
}
