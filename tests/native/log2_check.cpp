// Host build of the kernels' log2 (basecount_amd/csrc/bc_log2.h) against the C library's log2,
// which CPython's math.log2 calls (tests/test_log2.py compiles and runs this).  Inputs: the
// probabilities c / cov the entropies use (main.py:40-53), values near 1 (the second polynomial),
// and uniform (0, 1].  Prints "<inputs> <mismatches>".
#define BC_LOG2_HD inline
#include <cmath>
#include <cstdint>
#include <cstdio>

#include "bc_log2.h"

int main() {
    uint64_t s = 0x9E3779B97F4A7C15ull, n = 0, bad = 0;
    auto next = [&]() {
        s ^= s << 13;
        s ^= s >> 7;
        s ^= s << 17;
        return s;
    };
    auto check = [&](double x) {
        ++n;
        if (bc::glibc_log2(x) != std::log2(x)) ++bad;
    };
    for (int i = 0; i < 2000000; ++i) {
        const uint64_t cov = 1 + next() % 3000000, c = 1 + next() % cov;
        check((double)c / (double)cov);
    }
    for (uint64_t cov = 1; cov <= 600; ++cov)
        for (uint64_t c = 1; c <= cov; ++c) check((double)c / (double)cov);
    for (int i = 0; i < 500000; ++i) check(0.9 + 0.2 * (double)(next() >> 11) * 0x1p-53);
    for (int i = 0; i < 500000; ++i) check((double)((next() >> 11) + 1) * 0x1p-53);
    std::printf("%llu %llu\n", (unsigned long long)n, (unsigned long long)bad);
    return 0;
}
