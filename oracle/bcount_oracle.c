/*
 * ORACLE — test infrastructure only.  Never linked into or called by the product path
 * (basecount_amd/).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it,
 * and only as the checker.
 *
 * Plain-C restatement of the reference's native operator count.bcount
 * (/root/reference/basecount/count.cpp:7-99) over the struct-of-arrays batch layout of
 * include/basecount_hip.h (bc_reads):
 *
 *   count.cpp:17      baseCounts(refLen, 6)                    -> out[refLen][6], zeroed
 *   count.cpp:35-38   refPos = starts[i]; readPos = 0          -> rp = pos[i]; qp = seq_nib[i]
 *   count.cpp:51-70   ops 0/7/8: per base, if quals[readPos] >= minBaseQuality,
 *                     'A'->0 'C'->1 'G'->2 'T'->3 'N'->5 (.at() bounds-checked); readPos++, refPos++
 *   count.cpp:74-75   op 1: readPos += len
 *   count.cpp:80-90   ops 2/3: per position col 4 += 1 (.at() bounds-checked), no quality test
 *   count.cpp:92-95   ops 4/5/6/9: nothing
 *
 * The letter comes from pysam's decode of the 4-bit SEQ code through "=ACMGRSVTWYHKDBN".
 * A bounds failure aborts the whole call (std::out_of_range -> IndexError); here it returns 1
 * with the read index and the refPos that .at() rejected.
 *
 * Pinned against the reference's own compiled count.cpp (oracle/_ref) and the golden fixtures in
 * tests/golden/ (tests/test_oracle.py).
 */
#include <stdint.h>
#include <string.h>

static const char kNt16[] = "=ACMGRSVTWYHKDBN";

int oracle_bcount(int64_t ref_len, uint32_t mbq, int64_t n, const int32_t* pos, const uint32_t* cig_beg,
                  const uint32_t* cig_n, const uint32_t* seq_nib, const uint32_t* cigar, const uint8_t* seq,
                  const uint8_t* qual, uint32_t* out, int64_t* bad_read, int64_t* bad_pos) {
    memset(out, 0, (size_t)ref_len * 6 * sizeof(uint32_t));
    *bad_read = -1;
    *bad_pos = -1;
    for (int64_t i = 0; i < n; ++i) {
        uint64_t refPos = (uint64_t)(int64_t)pos[i];
        uint64_t readPos = seq_nib[i];
        const uint32_t* tups = cigar + cig_beg[i];
        for (uint32_t t = 0; t < cig_n[i]; ++t) {
            const uint32_t operation = tups[t] & 0xF, opLen = tups[t] >> 4;
            if (operation == 0 || operation == 7 || operation == 8) {
                for (uint32_t j = 0; j < opLen; j++) {
                    const unsigned q = qual ? qual[readPos] : 0u;
                    if (q >= mbq) {
                        const unsigned b = seq[readPos >> 1];
                        const char letter = kNt16[(readPos & 1) ? (b & 0xF) : (b >> 4)];
                        int col = -1;
                        switch (letter) {
                            case 'A': col = 0; break;
                            case 'C': col = 1; break;
                            case 'G': col = 2; break;
                            case 'T': col = 3; break;
                            case 'N': col = 5; break;
                        }
                        if (col >= 0) {
                            if (refPos >= (uint64_t)ref_len) {
                                *bad_read = i;
                                *bad_pos = (int64_t)refPos;
                                return 1;
                            }
                            out[refPos * 6 + (uint64_t)col] += 1;
                        }
                    }
                    readPos += 1;
                    refPos += 1;
                }
            } else if (operation == 1) {
                readPos += opLen;
            } else if (operation == 2 || operation == 3) {
                for (uint32_t j = 0; j < opLen; j++) {
                    if (refPos >= (uint64_t)ref_len) {
                        *bad_read = i;
                        *bad_pos = (int64_t)refPos;
                        return 1;
                    }
                    out[refPos * 6 + 4] += 1;
                    refPos += 1;
                }
            }
        }
    }
    return 0;
}
