// bc_log2.h — the host C library's log2, evaluated on the GPU, so the entropies match the
// reference bit for bit.
//
// The reference sums -(p * math.log2(p)) (main.py:10-11); CPython's math.log2 is glibc's log2
// (glibc 2.35 in this image: one non-FMA implementation on every x86-64 CPU).  That algorithm is
// not correctly rounded (≈0.2 % of the p = c / cov values sit one ulp away from the correctly
// rounded log2), and the GPU's own log2 differs from it on ≈1.4 % of the entropies, so kernel 2
// evaluates the same algorithm with the same constants: table lookup by the top mantissa bits,
// log2(x) = k + log2(c) + log2(z / c) with the reduction and the polynomial exactly as
// sysdeps/ieee754/dbl-64/e_log2.c (Arm optimized-routines) writes them for targets without FMA.
// Every operation is a plain IEEE double add/multiply in the source's order, which holds because
// the library is built with -ffp-contract=off (no fused multiply-adds).  Constants:
// bc_log2_table.h (generated and verified against math.log2 by scripts/gen_log2_table.py).
//
// Domain: 0 < x < inf, the only inputs the entropies use (p = c / cov with 0 < c <= cov).
#pragma once
#include <cstdint>

#include "bc_log2_table.h"

// device code by default; a host build (tests/native/log2_check.cpp) defines BC_LOG2_HD first
#ifndef BC_LOG2_HD
#define BC_LOG2_HD __device__ __forceinline__
#endif

namespace bc {

// TAB: the (invc, logc, chi, clo) table, indexable as tab[i][j] (log2d::kTab, or a copy in LDS)
template <typename TAB>
BC_LOG2_HD double glibc_log2_t(double x, const TAB& kTab) {
    using log2d::kA;
    using log2d::kB;
    using log2d::kInvLn2Hi;
    using log2d::kInvLn2Lo;
    const uint64_t ix = __builtin_bit_cast(uint64_t, x);
    if (ix - 0x3feea4af00000000ull < 0x3ff0b55900000000ull - 0x3feea4af00000000ull) {
        // close to 1.0: log2(1 + r) by the second polynomial, r exact
        if (ix == 0x3ff0000000000000ull) return 0.0;
        const double r = x - 1.0;
        const double rhi = __builtin_bit_cast(double, __builtin_bit_cast(uint64_t, r) & 0xffffffff00000000ull);
        const double rlo = r - rhi;
        const double hi = rhi * kInvLn2Hi;
        double lo = rlo * kInvLn2Hi + r * kInvLn2Lo;
        const double r2 = r * r;
        const double r4 = r2 * r2;
        const double p = r2 * (kB[0] + r * kB[1]);
        const double y = hi + p;
        lo += hi - y + p;
        lo += r4 * (kB[2] + r * kB[3] + r2 * (kB[4] + r * kB[5]) +
                    r4 * (kB[6] + r * kB[7] + r2 * (kB[8] + r * kB[9])));
        return y + lo;
    }
    // x = 2^k z, z in [0x1.6p-1, 0x1.6p0); subinterval i of 64 by the top mantissa bits
    const uint64_t tmp = ix - 0x3fe6000000000000ull;
    const int i = (int)((tmp >> 46) & 63u);
    const int64_t k = (int64_t)tmp >> 52;
    const double z = __builtin_bit_cast(double, ix - (tmp & (0xfffull << 52)));
    const double invc = kTab[i][0], logc = kTab[i][1], chi = kTab[i][2], clo = kTab[i][3];
    const double r = (z - chi - clo) * invc;
    const double rhi = __builtin_bit_cast(double, __builtin_bit_cast(uint64_t, r) & 0xffffffff00000000ull);
    const double rlo = r - rhi;
    const double t1 = rhi * kInvLn2Hi;
    const double t2 = rlo * kInvLn2Hi + r * kInvLn2Lo;
    const double t3 = (double)k + logc;
    const double hi = t3 + t1;
    const double lo = t3 - hi + t1 + t2;
    const double r2 = r * r;
    const double r4 = r2 * r2;
    const double p = kA[0] + r * kA[1] + r2 * (kA[2] + r * kA[3]) + r4 * (kA[4] + r * kA[5]);
    return lo + r2 * p + hi;
}

BC_LOG2_HD double glibc_log2(double x) { return glibc_log2_t(x, log2d::kTab); }

}  // namespace bc
