/*
 * ORACLE — test infrastructure only (see bcount_oracle.c header for the usage rule).
 *
 * Plain-C restatement of get_stats / get_entropy (/root/reference/basecount/main.py:10-79) for
 * one reference, producing the same per-position struct-of-arrays as kernel 2:
 *
 *   main.py:19-31  drop N (column 5) unless show_n_bases; k = 5 or 6
 *   main.py:24-25  nf = 1/log2(k), nf2 = 1/log2(k-1)                         (passed in)
 *   main.py:37     coverage = sum(base_count)                                   (ints)
 *   main.py:40-41  p = count / coverage ; pc = 100 * p                          (IEEE double)
 *   main.py:11,42  entropy = nf * sum([-(x*log2(x)) if x != 0 else 0 ...])      (left to right)
 *   main.py:44-53  drop the first argmax (np.argmax), same over cov2; cov2 == 0 -> int 1
 *   main.py:34-36  coverage == 0 -> pc = [-1]*k, entropy = secondary = 1       (ints)
 *
 * CPython's math.log2 is the C library's log2, and int/int true division of values below 2^53 is
 * one IEEE division, so with -ffp-contract=off this reproduces the reference's floats bit for bit
 * (checked against the reference's own get_stats on the golden fixtures, tests/test_oracle.py).
 * Int-typed outputs are returned as doubles -1.0 / 1.0; the formatter derives the int/float type
 * from the counts exactly as the reference's control flow does.
 */
#include <math.h>
#include <stdint.h>

/* positions [p0, p1) of a reference of L positions (the multi-threaded driver, mt_oracle.c,
 * splits the positions; every position is independent) */
void oracle_stats_range(const uint32_t* counts6, int64_t p0, int64_t p1, int64_t L, int show_n, double nf,
                        double nf2, int32_t* cov_out, double* pc, double* ent, double* sec) {
    const int k = show_n ? 6 : 5;
    for (int64_t p = p0; p < p1; ++p) {
        int64_t c[6];
        int64_t cov = 0;
        for (int j = 0; j < k; ++j) {
            c[j] = counts6[p * 6 + j];
            cov += c[j];
        }
        cov_out[p] = (int32_t)cov;
        if (cov == 0) {
            for (int j = 0; j < k; ++j) pc[j * L + p] = -1.0;
            ent[p] = 1.0;
            sec[p] = 1.0;
            continue;
        }
        double s = 0.0;
        for (int j = 0; j < k; ++j) {
            const double x = (double)c[j] / (double)cov;
            pc[j * L + p] = 100.0 * x;
            if (x != 0) s += -(x * log2(x));
        }
        ent[p] = nf * s;
        int am = 0;
        for (int j = 1; j < k; ++j)
            if (c[j] > c[am]) am = j;
        const int64_t cov2 = cov - c[am];
        if (cov2 == 0) {
            sec[p] = 1.0;
            continue;
        }
        double s2 = 0.0;
        for (int j = 0; j < k; ++j) {
            if (j == am) continue;
            const double x = (double)c[j] / (double)cov2;
            if (x != 0) s2 += -(x * log2(x));
        }
        sec[p] = nf2 * s2;
    }
}

void oracle_stats(const uint32_t* counts6 /* [L][6] as returned by bcount */, int64_t L, int show_n, double nf,
                  double nf2, int32_t* cov_out, double* pc /* [k][L] */, double* ent, double* sec) {
    oracle_stats_range(counts6, 0, L, L, show_n, nf, nf2, cov_out, pc, ent, sec);
}
