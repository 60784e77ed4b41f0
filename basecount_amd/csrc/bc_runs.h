// bc_runs.h — a read's CIGAR as a run table (count.cpp:40-96 semantics), on the device and on the
// host.  The kernels decode CIGAR words into these tables; bc_reads_upload decodes each read of a
// sorted batch once, with the same function, into a 16-byte run record (bc_reads.read_runs) that
// the read-chunked kernel then loads instead of decoding.
//
// Included inside namespace bc::{anonymous} of each kernel file (through bc_walk.h) and of
// bc_capi.hip.
#pragma once
#include <cstdint>

#ifndef BC_HD
#define BC_HD __host__ __device__ __forceinline__
#endif

constexpr int kPre = 8;  // CIGAR words decoded per read (more -> complex path)

BC_HD bool mlike(uint32_t op) { return op == 0 || op == 7 || op == 8; }
BC_HD bool dlike(uint32_t op) { return op == 2 || op == 3; }
BC_HD bool qcons(uint32_t op) { return op == 0 || op == 1 || op == 7 || op == 8; }

// Run table of a read: its aligned (M/=/X) bases as at most 4 runs [st, en) of reference
// offsets from the read start, each with a query delta qd (query offset = reference offset +
// qd; consecutive M/=/X ops with the same delta merge, so the M/=/X distinction and S/H/P
// between them vanish).  Every other reference offset in [0, span) is a deletion / ref-skip.
// count.cpp:40-96 semantics: M/=/X consume both, I the query only, D/N the reference only.
constexpr int kMaxRuns = 4;

struct RunTable {
    uint32_t st[kMaxRuns], en[kMaxRuns];
    int32_t qd[kMaxRuns];
    uint32_t span;
    uint32_t qlen;  // query bases consumed (M/=/X/I) by the decoded ops
    int nrun;
    bool gap;       // some reference offset in [0, span) is a deletion / ref-skip
    bool complex;
};

// NSLOT < kMaxRuns fills only the first NSLOT runs' st / en / qd (nrun, complex and the rest are
// those of the full table): callers re-decode with the full table when a read has more runs.
template <int NSLOT = kMaxRuns>
BC_HD RunTable decode_runs(const uint32_t (&w)[kPre], uint32_t cn, int cmax) {
    // Branch-free: every op updates the table through selects (a divergent if/else chain here
    // compiles to hundreds of register moves per read).
    RunTable T;
#pragma unroll
    for (int i = 0; i < kMaxRuns; ++i) T.st[i] = T.en[i] = 0, T.qd[i] = 0;
    bool cx = cn > (uint32_t)kPre, gap = false;
    uint32_t rc = 0, qc = 0, last_en = 0xFFFFFFFFu;
    int last_qd = 0, nrun = 0;
#pragma unroll
    for (int k = 0; k < kPre; ++k) {
        if (k >= cmax) break;  // wave-uniform: no lane has more ops
        const uint32_t op = w[k] & 15u, len = (uint32_t)k < cn ? w[k] >> 4 : 0u;
        const bool m = mlike(op) && len != 0u;  // M/=/X: a run (new, or extending the last one)
        const bool d = dlike(op) && len != 0u;  // D/N: reference only
        const int qd = (int)qc - (int)rc;
        const bool ext = m && last_en == rc && last_qd == qd;
        const bool nw = m && !ext;
        cx = cx || (m && (qd < -32768 || qd > 32767)) || (nw && nrun >= kMaxRuns);
        const uint32_t e = rc + len;
#pragma unroll
        for (int i = 0; i < NSLOT; ++i) {
            const bool sn = nw && nrun == i, se = ext && nrun == i + 1;
            T.st[i] = sn ? rc : T.st[i];
            T.qd[i] = sn ? qd : T.qd[i];
            T.en[i] = (sn || se) ? e : T.en[i];
        }
        nrun += nw ? 1 : 0;
        gap = gap || d;
        rc = (m || d) ? e : rc;
        qc += (m || op == 1u) ? len : 0u;  // I: query only
        last_en = m ? e : last_en;
        last_qd = m ? qd : last_qd;
    }
    T.nrun = nrun;
    T.gap = gap;
    T.complex = cx || rc >= 0x1FFFu;
    T.span = rc;
    T.qlen = qc;
    return T;
}

// The 16-byte run record (bc_reads.read_runs, 4 words per read) of a read's first two runs:
//   x = st0 | en0 << 13 | min(nrun, 7) << 26 | gap << 29 | complex << 30
//   y = st1 | en1 << 13
//   z = qd0 (int16) | qd1 (int16) << 16
//   w = span | qlen << 16
// Offsets fit 13 bits and qd 16 (decode_runs marks a read complex otherwise); a read whose query
// length exceeds 16 bits is recorded as complex.  unpack(pack(T)) equals decode_runs<2>'s table
// (runs 2 and 3 left empty: a chunk with more runs decodes its CIGARs again).
BC_HD void pack_runs(const RunTable& T, uint32_t* r) {
    const bool cx = T.complex || T.qlen > 0xFFFFu;
    const uint32_t nr = (uint32_t)(T.nrun < 7 ? T.nrun : 7);
    r[0] = (T.st[0] & 0x1FFFu) | (T.en[0] & 0x1FFFu) << 13 | nr << 26 | (T.gap ? 1u : 0u) << 29 | (cx ? 1u : 0u) << 30;
    r[1] = (T.st[1] & 0x1FFFu) | (T.en[1] & 0x1FFFu) << 13;
    r[2] = ((uint32_t)T.qd[0] & 0xFFFFu) | ((uint32_t)T.qd[1] & 0xFFFFu) << 16;
    r[3] = (T.span & 0xFFFFu) | (T.qlen & 0xFFFFu) << 16;
}
BC_HD RunTable unpack_runs(uint32_t x, uint32_t y, uint32_t z, uint32_t w) {
    RunTable T;
    T.st[0] = x & 0x1FFFu;
    T.en[0] = (x >> 13) & 0x1FFFu;
    T.st[1] = y & 0x1FFFu;
    T.en[1] = (y >> 13) & 0x1FFFu;
    T.st[2] = T.en[2] = T.st[3] = T.en[3] = 0;
    T.qd[0] = (int32_t)(int16_t)(z & 0xFFFFu);
    T.qd[1] = (int32_t)(int16_t)(z >> 16);
    T.qd[2] = T.qd[3] = 0;
    T.nrun = (int)((x >> 26) & 7u);
    T.gap = ((x >> 29) & 1u) != 0;
    T.complex = ((x >> 30) & 1u) != 0;
    T.span = w & 0xFFFFu;
    T.qlen = w >> 16;
    return T;
}

// ---- the CIGAR decode of the event image (the first two runs), ~12 VALU per op ------------------
// decode_runs updates a whole run table through selects at every op (~33 VALU per op).  Here each
// op only adds its reference / query lengths into a packed prefix P[k] = rc | qc << 16 (before op
// k) and marks itself in a bit string F (bit 2k: M/=/X, bit 2k + 1: I/D/N, zero lengths
// excluded).  Runs are the M groups between I/D/N ops, so the op indices where they start and end
// are found bit-parallel (v_ffbl on F), and their bounds are P at those indices (one LDS round
// trip through the lane's own 8 scratch words, `scr`, 16-byte aligned).  The result equals decode_runs<2>'s table
// whenever the read has at most two runs and every op length is below 2^13; the function returns
// false otherwise (the caller then runs decode_runs).
BC_HD uint32_t ffbl_or_none(uint32_t x) { return (uint32_t)(__builtin_ffs((int)x) - 1); }  // 0xFFFFFFFF if x == 0
// bits [off & 31, (off & 31) + w) of x (one v_bfe_u32 on the device)
BC_HD uint32_t ubfe(uint32_t x, uint32_t off, uint32_t w) { return (x >> (off & 31u)) & ((1u << w) - 1u); }
BC_HD bool decode_fast2(const uint32_t (&w)[kPre], uint32_t cn, int cmax, uint32_t* scr,
                     RunTable& T) {
    // 2-bit fields at 2 * op: kMB 1 = M/=/X (0, 7, 8), 2 = I/D/N (1, 2, 3); kRQ bit 0 = consumes the
    // reference (M D N = X), bit 1 = consumes the query (M I = X)
    constexpr uint32_t kMB = 1u | 2u << 2 | 2u << 4 | 2u << 6 | 1u << 14 | 1u << 16;
    constexpr uint32_t kRQ = 3u | 2u << 2 | 1u << 4 | 1u << 6 | 3u << 14 | 3u << 16;
    uint32_t P[kPre + 1];
    P[0] = 0u;
    uint32_t F = 0u, big = 0u;
#pragma unroll
    for (int k = 0; k < kPre; ++k) {
        if (k >= cmax) {  // (uniform) no lane has more ops
            P[k + 1] = P[k];
            continue;
        }
        const uint32_t o2 = w[k] << 1, len = w[k] >> 4;  // v_bfe reads the low 5 bits of o2: 2 * op
        uint32_t fl = ubfe(kMB, o2, 2);
        fl = fl < (len << 1) ? fl : (len << 1);  // zero-length ops are no run and no break
        F |= fl << (2 * k);
        const uint32_t rq = ubfe(kRQ, o2, 2);
        P[k + 1] = P[k] + (len & 0xFFFFFFu) * ((rq * 0x8001u) & 0x10001u);  // rq -> 1 | 1 << 16 (v_mad_u32_u24)
        big |= len;
    }
    uint32_t* s16 = (uint32_t*)__builtin_assume_aligned(scr, 16);
#pragma unroll
    for (int k = 0; k < kPre; ++k) s16[k] = P[k];
    scr = s16;
    const uint32_t Mb = F & 0x5555u, Bb = (F >> 1) & 0x5555u;
    // first M op, the first I/D/N after it, the next M (run 1), the next I/D/N, a third run
    const uint32_t p1 = ffbl_or_none(Mb);
    const uint32_t p2 = ffbl_or_none(Bb & (0xFFFFFFFFu << (p1 & 31u)));
    const uint32_t p3 = ffbl_or_none(Mb & (0xFFFFFFFFu << (p2 & 31u)));
    const uint32_t p4 = ffbl_or_none(Bb & (0xFFFFFFFFu << (p3 & 31u)));
    const uint32_t p5 = ffbl_or_none(Mb & (0xFFFFFFFFu << (p4 & 31u)));
    const uint32_t X1 = scr[(p1 >> 1) & 7u], X2 = scr[(p2 >> 1) & 7u], X3 = scr[(p3 >> 1) & 7u],
                   X4 = scr[(p4 >> 1) & 7u];
    const uint32_t span = P[kPre] & 0xFFFFu;
    const int nrun = p1 == 0xFFFFFFFFu ? 0 : (p3 == 0xFFFFFFFFu ? 1 : (p5 == 0xFFFFFFFFu ? 2 : 3));
    T.span = span;
    T.qlen = P[kPre] >> 16;
    T.nrun = nrun;
    T.st[2] = T.en[2] = T.st[3] = T.en[3] = 0u;
    T.qd[2] = T.qd[3] = 0;
    T.st[0] = nrun >= 1 ? X1 & 0xFFFFu : 0u;
    T.qd[0] = nrun >= 1 ? (int)(X1 >> 16) - (int)(X1 & 0xFFFFu) : 0;
    T.en[0] = nrun >= 1 ? (p2 != 0xFFFFFFFFu ? X2 & 0xFFFFu : span) : 0u;
    T.st[1] = nrun >= 2 ? X3 & 0xFFFFu : 0u;
    T.qd[1] = nrun >= 2 ? (int)(X3 >> 16) - (int)(X3 & 0xFFFFu) : 0;
    T.en[1] = nrun >= 2 ? (p4 != 0xFFFFFFFFu ? X4 & 0xFFFFu : span) : 0u;
    // a deletion / ref-skip of positive length <=> the span exceeds the runs' lengths
    T.gap = span != (T.en[0] - T.st[0]) + (T.en[1] - T.st[1]);
    const bool qd_ok = T.qd[0] >= -32768 && T.qd[0] <= 32767 && T.qd[1] >= -32768 && T.qd[1] <= 32767;
    T.complex = cn > (uint32_t)kPre || !qd_ok || span >= 0x1FFFu;
    return cn > (uint32_t)kPre || (nrun <= 2 && big < 0x2000u);
}

// ---- chunk summaries of the read-chunked kernel (bc_reads.read_runs after the records) ----
constexpr int kRcChunkReads = 256;  // reads per k_rc chunk (one per thread of its block)

// A simple read's run shape for k_rc: its run count when the event image can take it (first run
// at the read start, last run at its end) or when it has more than two runs, else 3 (a chunk
// holding such a read walks the run tables).
BC_HD uint32_t run_shape(const RunTable& T) {
    return ((T.nrun >= 1 && T.st[0] == 0u && (T.nrun == 1 ? T.en[0] : T.en[1]) == T.span) || T.nrun > 2)
               ? (uint32_t)T.nrun
               : 3u;
}

// A complex read's reference span (M/=/X/D/N), capped at 2^30 - 1.
BC_HD uint32_t full_span(const uint32_t* cg, uint32_t cn) {
    uint64_t sp = 0;
    for (uint32_t k = 0; k < cn; ++k)
        if (mlike(cg[k] & 15u) || dlike(cg[k] & 15u)) sp += cg[k] >> 4;
    return sp > 0x3FFFFFFFu ? 0x3FFFFFFFu : (uint32_t)sp;
}

