// bc_stats.h — kernel 2 for ONE position, evaluated by the position's lane: coverage,
// percentages and the two entropies of main.py:29-53, in CPython's order of operations.
//
// Used where a kernel finalises positions one per lane (k_pileup's and k_pileup_solo's tiles;
// k_stats_lane restates it with a NULL check per output).  k_stats spreads the same terms over
// one wave per column and adds them in the same column order, so every path gives the same bits.
#pragma once
#include <cstdint>

#include "bc_log2.h"

namespace bc {

// c: the K column counts of position P (< L).  Writes cov[P], pc[j * L + P] (pc may be NULL),
// ent[P], sec[P]; returns the entropy.
//   cov = sum(counts); pj = c_j / cov; pc_j = 100 * pj (-1 when cov == 0);
//   ent = nf * sum_{c_j != 0} -(pj log2 pj)          (1.0 when cov == 0);
//   sec = nf2 * sum_{j != argmax, c_j != 0} -(q log2 q), q = c_j / (cov - c_argmax)
//         (1.0 when cov == 0 or cov == c_argmax); argmax = np.argmax (first maximum).
template <int K>
__device__ __forceinline__ double position_stats(const uint32_t* c, int64_t L, int64_t P, double nf, double nf2,
                                                 int32_t* cov_out, double* pc, double* ent, double* sec) {
    int64_t cov = 0;
    int am = 0;
    uint32_t mx = c[0];  // (no c[am]: a register array indexed at run time would go to scratch)
#pragma unroll
    for (int j = 0; j < K; ++j) {
        cov += c[j];
        if (c[j] > mx) mx = c[j], am = j;  // np.argmax: first maximum
    }
    cov_out[P] = (int32_t)cov;
    double h = 1.0, h2 = 1.0;
    if (cov != 0 && cov == (int64_t)mx) {
        // one class only (most covered positions of a shallow batch): p = 1 for it and 0 for the
        // rest, so the terms are exactly what the loops below would give: -(1 * log2 1) = -0.0,
        // 0.0 + -0.0 = 0.0, h = nf * 0.0 = 0.0; pc 100.0 and 0.0; cov2 = 0 leaves h2 = 1.0
        if (pc) {
#pragma unroll
            for (int j = 0; j < K; ++j) pc[(int64_t)j * L + P] = j == am ? 100.0 : 0.0;
        }
        h = 0.0;
    } else if (cov != 0) {
        double s = 0.0;
#pragma unroll
        for (int j = 0; j < K; ++j) {
            const double pj = (double)c[j] / (double)cov;
            if (pc) pc[(int64_t)j * L + P] = 100.0 * pj;
            if (c[j] != 0) s = s + (-(pj * glibc_log2(pj)));
        }
        h = nf * s;
        const int64_t cov2 = cov - (int64_t)mx;
        if (cov2 != 0) {
            double s2 = 0.0;
#pragma unroll
            for (int j = 0; j < K; ++j)
                if (j != am && c[j] != 0) {
                    const double q = (double)c[j] / (double)cov2;
                    s2 = s2 + (-(q * glibc_log2(q)));
                }
            h2 = nf2 * s2;
        }
    } else if (pc) {
#pragma unroll
        for (int j = 0; j < K; ++j) pc[(int64_t)j * L + P] = -1.0;
    }
    ent[P] = h;
    sec[P] = h2;
    return h;
}

// The coverage and the entropy of position_stats alone (the same operations in the same order,
// so the same bits), for the summary-only sweep: main.py:469-499 averages coverage and entropy
// only, and neither the percentages nor the secondary entropy are computed.
template <int K>
__device__ __forceinline__ double position_entropy(const uint32_t* c, double nf, uint32_t& cov_out) {
    int64_t cov = 0;
#pragma unroll
    for (int j = 0; j < K; ++j) cov += c[j];
    cov_out = (uint32_t)cov;
    double h = 1.0;
    uint32_t mx = 0;
#pragma unroll
    for (int j = 0; j < K; ++j) mx = c[j] > mx ? c[j] : mx;
    if (cov != 0 && cov == (int64_t)mx) {
        h = 0.0;  // one class only: -(1 * log2 1) = -0.0 summed from 0.0, times nf (as above)
    } else if (cov != 0) {
        double s = 0.0;
#pragma unroll
        for (int j = 0; j < K; ++j) {
            const double pj = (double)c[j] / (double)cov;
            if (c[j] != 0) s = s + (-(pj * glibc_log2(pj)));
        }
        h = nf * s;
    }
    return h;
}

}  // namespace bc
