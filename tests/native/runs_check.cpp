// Host check of the event image's fast CIGAR decode (decode_fast2, bc_runs.h) against the run
// table decoder the kernels use elsewhere (decode_runs<2>): wherever decode_fast2 reports the read
// as decodable, every field k_rc reads must be identical.  Random CIGARs over all 16 op codes
// (zero lengths, leading / trailing D, I and clips, long ops, up to 10 ops), plus the C3 shapes.
//   g++ -O2 -std=c++17 -I basecount_amd/csrc tests/native/runs_check.cpp && ./a.out [iterations]
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#define BC_HD inline
#include "bc_runs.h"

int main(int argc, char** argv) {
    const long iters = argc > 1 ? std::atol(argv[1]) : 2000000;
    std::mt19937_64 g(12345);
    long sure = 0, two = 0;
    for (long it = 0; it < iters; ++it) {
        const int mode = (int)(g() % 4);
        uint32_t cn = (uint32_t)(g() % 11);
        uint32_t w[kPre] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (uint32_t k = 0; k < cn && k < (uint32_t)kPre; ++k) {
            uint32_t op, len;
            if (mode == 0) {  // C3-like: clips, M blocks, one short I/D/=/X block
                static const uint32_t ops[] = {0, 0, 0, 1, 2, 4, 5, 7, 8, 3};
                op = ops[g() % 10];
                len = (uint32_t)(g() % 80);
            } else if (mode == 1) {  // any op code, short lengths including zero
                op = (uint32_t)(g() % 16);
                len = (uint32_t)(g() % 4);
            } else if (mode == 2) {  // long lengths near the 13-bit limits
                op = (uint32_t)(g() % 10);
                len = (uint32_t)(g() % 3 == 0 ? 8000 + g() % 400 : g() % 100000);
            } else {
                op = (uint32_t)(g() % 10);
                len = (uint32_t)(g() % (1u << 28));
            }
            w[k] = len << 4 | op;
        }
        int cmax = (int)(cn < (uint32_t)kPre ? cn : (uint32_t)kPre);
        if (g() % 3 == 0 && cmax < kPre) cmax += (int)(g() % (kPre - cmax + 1));  // the wave's longer reads
        alignas(16) uint32_t scr[8];
        RunTable F;
        const bool ok = decode_fast2(w, cn, cmax, scr, F);
        const RunTable R = decode_runs<2>(w, cn, cmax);
        if (!ok) continue;
        ++sure;
        two += R.nrun == 2;
        bool eq = F.complex == R.complex;
        if (!R.complex)
            eq = eq && F.nrun == R.nrun && F.span == R.span && F.qlen == R.qlen && F.gap == R.gap &&
                 F.st[0] == R.st[0] && F.en[0] == R.en[0] && F.qd[0] == R.qd[0] && F.st[1] == R.st[1] &&
                 F.en[1] == R.en[1] && F.qd[1] == R.qd[1];
        if (!eq) {
            std::printf("MISMATCH it=%ld cn=%u cmax=%d\n", it, cn, cmax);
            for (uint32_t k = 0; k < (uint32_t)kPre; ++k) std::printf("  op %u len %u\n", w[k] & 15u, w[k] >> 4);
            std::printf("fast: nrun %d span %u qlen %u gap %d cx %d run0 [%u,%u) qd %d run1 [%u,%u) qd %d\n", F.nrun,
                        F.span, F.qlen, F.gap, F.complex, F.st[0], F.en[0], F.qd[0], F.st[1], F.en[1], F.qd[1]);
            std::printf("ref:  nrun %d span %u qlen %u gap %d cx %d run0 [%u,%u) qd %d run1 [%u,%u) qd %d\n", R.nrun,
                        R.span, R.qlen, R.gap, R.complex, R.st[0], R.en[0], R.qd[0], R.st[1], R.en[1], R.qd[1]);
            return 1;
        }
    }
    std::printf("ok %ld decodable of %ld (%ld with two runs)\n", sure, iters, two);
    return 0;
}
