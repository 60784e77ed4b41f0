// bc_walk.h — device building blocks shared by the two pileup kernels (the position-tiled
// k_pileup and the read-chunked k_rc): CIGAR run tables, the BC_SEQ_EVENT window fetch and the
// SWAR window counters.  Included inside namespace bc::{anonymous} of each kernel file.
//
// Event classes (BC_SEQ_EVENT, include/basecount_hip.h): one nibble per base,
//   A 0001, C 0010, G 0100, T 1000, N 0011, not counted 0000, and, synthesized by the walk for
//   reference offsets inside a read's span not covered by an aligned base, deletion 1100.
// count.cpp:40-96 semantics: M/=/X bases count their letter (subject to the quality test),
// D/N count DS, I/S/H/P/B count nothing.
#pragma once

#include "bc_runs.h"

constexpr unsigned long long kNibCol6 = 0x6666666366625106ull;  // class -> column, 6 = none
constexpr uint32_t kM1 = 0x11111111u;      // bit 0 of every nibble
constexpr uint32_t kClsDel = 0xCCCCCCCCu;  // class 1100 (deletion / ref-skip) in every nibble
constexpr uint32_t kNone = 0xFFFFFFFFu;  // packed event: none
constexpr uint32_t kDel = 0x80000000u;   // packed event: deletion / ref-skip

__device__ __forceinline__ unsigned nib_col6(unsigned nib) { return (unsigned)(kNibCol6 >> (nib * 4)) & 0xFu; }
__device__ __forceinline__ uint32_t rdl(uint32_t v, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, l); }

// Wave-wide max / min (result in every lane's SGPR): a prefix max / min within each 16-lane row
// (DPP row_shr 1, 2, 4, 8), then the four rows' last lanes combined on the scalar unit.  The
// DPP source's `old` operand is the operation's identity, so each step compiles to ONE fused
// v_max/min_u32_dpp (with `old = v` the compiler keeps a separate mov + op per step: 18 VALU
// instead of 4).
template <bool MAX>
__device__ __forceinline__ uint32_t wave_reduce(uint32_t v) {
    constexpr int id = MAX ? 0 : -1;
    auto op = [](uint32_t a, uint32_t b) { return MAX ? (a > b ? a : b) : (a < b ? a : b); };
    v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(id, (int)v, 0x111, 0xF, 0xF, false));  // row_shr:1
    v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(id, (int)v, 0x112, 0xF, 0xF, false));  // row_shr:2
    v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(id, (int)v, 0x114, 0xF, 0xF, false));  // row_shr:4
    v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(id, (int)v, 0x118, 0xF, 0xF, false));  // row_shr:8
    const uint32_t r0 = (uint32_t)__builtin_amdgcn_readlane((int)v, 15);
    const uint32_t r1 = (uint32_t)__builtin_amdgcn_readlane((int)v, 31);
    const uint32_t r2 = (uint32_t)__builtin_amdgcn_readlane((int)v, 47);
    const uint32_t r3 = (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
    return op(op(r0, r1), op(r2, r3));
}


// ---- SWAR counters of a lane's 8-position window ------------------------------------------
// a4[c]: nibble k = count of column c at window position k; at most 15 reads are added before
// the wave folds them into cnt[] (a sum over the 8 read slots is then <= 120: fits a byte).
struct Swar {
    uint32_t a4[6];
};

__device__ __forceinline__ uint32_t lo32_bit(int sh) { return (uint32_t)(1ull << sh); }  // sh in [0, 32]
// nibbles [kl, kh) of a window word, 0 <= kl <= kh <= 8
__device__ __forceinline__ uint32_t nib_range(int kl, int kh) { return lo32_bit(4 * kh) - lo32_bit(4 * kl); }

template <int NC>
__device__ __forceinline__ void swar_add(Swar& W, uint32_t x) {
    const uint32_t x1 = x >> 1, x2 = x >> 2, x3 = x >> 3;
    W.a4[0] += x & ~x1 & kM1;   // A  0001
    W.a4[1] += x1 & ~x & kM1;   // C  0010
    W.a4[2] += x2 & ~x3 & kM1;  // G  0100
    W.a4[3] += x3 & ~x2 & kM1;  // T  1000
    W.a4[4] += x2 & x3 & kM1;   // DS 1100
    if (NC == 6) W.a4[5] += x & x1 & kM1;  // N 0011
}

// sum over the 8 read slots (lanes 8g .. 8g+7): quad xor 1, quad xor 2, half-row mirror
__device__ __forceinline__ uint32_t sum8(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);
    return v;
}

// Fold the window counters into cnt[] of this lane's own position (8g + s == lane).  Must be
// called by the whole wave.  Byte b of the even / odd half holds window position 2b / 2b + 1.
template <int NC>
__device__ __forceinline__ void swar_fold(Swar& W, uint32_t (&cnt)[6], int s8) {
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const uint32_t b0 = sum8(W.a4[c] & 0x0F0F0F0Fu), b1 = sum8((W.a4[c] >> 4) & 0x0F0F0F0Fu);
        cnt[c] += (((s8 & 1) ? b1 : b0) >> (8 * (s8 >> 1))) & 0xFFu;
        W.a4[c] = 0;
    }
}

// SWAR mask of 8 bases that pass the quality test, from their 8 quality bytes (q0: bases 0-3).
__device__ __forceinline__ uint32_t ge_bytes(uint32_t q, uint32_t m) {  // per byte q >= m, m in [1, 255]
    const uint32_t H = 0x80808080u;
    const uint32_t t = (q | H) - (m & 0x7Fu) * 0x01010101u;  // high bit: low7(q) >= low7(m)
    return (m & 0x80u) ? (q & t & H) : ((q | t) & H);
}
__device__ __forceinline__ uint32_t qual_nibmask(uint32_t q0, uint32_t q1, uint32_t m) {
    if (m > 255u) return 0u;
    uint32_t b0 = (ge_bytes(q0, m) >> 7) * 15u, b1 = (ge_bytes(q1, m) >> 7) * 15u;
    b0 |= b0 >> 4;
    b1 |= b1 >> 4;
    return __builtin_amdgcn_perm(b1, b0, 0x06040200u);
}

// ---- LDS-DMA staging (global_load_lds_dwordx4): bytes [src, src + bytes) -> LDS [dst, ...) -----
// One wave-instruction moves 1 KiB lane-linearly (dst + 16 * lane), with no VGPR destination, so
// all passes of a chunk's copy are in flight together (a register copy waits for every load
// before its LDS write: one full memory round trip per KiB).  `dst` and `src` are 16-B aligned;
// the source buffer is readable up to the next 16-B boundary.  `tid` / `nthreads`: the copying
// threads (a wave: lane / 64; a block: threadIdx.x / blockDim.x).  hipcc does not count these
// loads: the caller waits with stage_wait() before anything reads the stage.
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void gbl_void_t;
// The pass offset is kept uniform (an SGPR: the source base, the LDS base in M0 and the loop are
// scalar work), and only a pass that ends past `bytes` masks its lanes: a full pass costs no VALU.
template <int NTHREADS>
__device__ __forceinline__ void stage_dma(uint8_t* dst, const uint8_t* src, uint32_t bytes, int tid) {
    const uint32_t wave_base = (uint32_t)__builtin_amdgcn_readfirstlane((tid & ~63) * 16);
    const uint32_t l16 = (uint32_t)(tid & 63) * 16u;
    for (uint32_t off = wave_base; off < bytes; off += NTHREADS * 16u) {  // wave-uniform
        const uint8_t* s = src + off;
        if (off + 1024u <= bytes || l16 < bytes - off)
            __builtin_amdgcn_global_load_lds((gbl_void_t*)(s + l16), (lds_void_t*)(dst + off), 16, 0, 0);
    }
}
__device__ __forceinline__ void stage_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// The 8 event classes at nibble indices n0 .. n0+7 of the sequence (unstaged: global memory).

// Where a walk reads its event classes: the chunk's stage in LDS (nibble indices relative to the
// stage; one readable pad word before and after, lim = last word index) or the whole
// BC_SEQ_EVENT buffer in HBM (lim = readable words).  Qualities only for unstaged walks.
struct SeqSrc {
    const uint32_t* words;
    int64_t lim;
    const uint8_t* qual;
    int64_t qual_bytes;
    uint32_t mbq;
};

// The 8 event classes at nibble indices n0 .. n0+7.
template <bool STAGED>
__device__ __forceinline__ uint32_t fetch8(const SeqSrc& S, int64_t n0) {
    const uint32_t* words = S.words;
    if (STAGED) {
        // windows that matter have n0 >= -7; anything else is masked off after the fetch
        const int n = (int)n0;
        int w0 = n >> 3;
        const int lim = (int)S.lim;
        w0 = w0 < -1 ? -1 : (w0 > lim ? lim : w0);
        return __builtin_amdgcn_alignbit(words[w0 + 1], words[w0], (uint32_t)n << 2);
    }
    const int64_t w0 = n0 >> 3, nw = S.lim;
    const int64_t i0 = w0 < 0 ? 0 : (w0 >= nw ? nw - 1 : w0);
    const int64_t i1 = w0 + 1 < 0 ? 0 : (w0 + 1 >= nw ? nw - 1 : w0 + 1);
    const uint32_t lo = (w0 >= 0 && w0 < nw) ? words[i0] : 0u;
    const uint32_t hi = (w0 + 1 >= 0 && w0 + 1 < nw) ? words[i1] : 0u;
    return __builtin_amdgcn_alignbit(hi, lo, (uint32_t)(n0 & 7) * 4u);
}

// quality mask of bases n0 .. n0+7 (unstaged chunks only; staged ones are masked at staging)
__device__ __forceinline__ uint32_t qual_mask_at(const SeqSrc& S, int64_t n0) {
    uint32_t m = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int64_t i = n0 + k;
        if (i >= 0 && i < S.qual_bytes && (uint32_t)S.qual[i] >= S.mbq) m |= 0xFu << (4 * k);
    }
    return m;
}

// Walk record of a read (3 x uint4 in LDS, written at chunk load):
//   [0] = {pos, 4*span, rr0, nb0}  [1] = {rr1, nb1, rr2, nb2}  [2] = {rr3, nb3, 0, 0}
// M run k: rr = 4*st | 4*en << 16 (empty: st == en), nb = nibble index (staged: relative to the
// stage) of the base at reference offset 0, i.e. seq_nib + qd.
__device__ __forceinline__ uint32_t pack_rr(uint32_t st, uint32_t en) { return (st * 4u) | ((en * 4u) << 16); }

// mask of the window nibbles whose reference offsets (from the read start, x4) lie in
// [lo4, hi4); j4 = 4 * window start
__device__ __forceinline__ uint32_t range_mask(int lo4, int hi4, int j4) {
    int kl = lo4 - j4;
    kl = kl < 0 ? 0 : (kl > 32 ? 32 : kl);
    int kh = hi4 - j4;
    kh = kh < kl ? kl : (kh > 32 ? 32 : kh);
    return lo32_bit(kh) - lo32_bit(kl);
}

// The 8 event classes (x) one read has in the lane's window [gb, gb + 8): its M runs' bases
// (one funnel-shifted fetch each) and, GAP, class 1100 on the rest of [0, span).
template <int NR, bool GAP, bool STAGED, bool QUAL>
__device__ __forceinline__ uint32_t window_events(const SeqSrc& S, const uint4* rec, int r, int gb) {
    const uint4 a = rec[r * 3];
    uint4 b = make_uint4(0u, 0u, 0u, 0u);
    uint2 c = make_uint2(0u, 0u);
    if (NR > 1) b = rec[r * 3 + 1];
    if (NR > 3) c = *(const uint2*)&rec[r * 3 + 2];
    const int j0 = gb - (int)a.x;  // window start relative to the read start
    const int j4 = j0 * 4;
    const uint32_t rr[4] = {a.z, b.x, b.z, c.x};
    const uint32_t nb[4] = {a.w, b.y, b.w, c.y};
    uint32_t x = 0, mm = 0;
#pragma unroll
    for (int k = 0; k < NR; ++k) {
        const uint32_t m = range_mask((int)(rr[k] & 0xFFFFu), (int)(rr[k] >> 16), j4);
        const int64_t n0 = STAGED ? (int64_t)((int)nb[k] + j0) : (int64_t)(int32_t)nb[k] + j0;
        uint32_t v = fetch8<STAGED>(S, n0);
        if (QUAL && !STAGED) v &= qual_mask_at(S, n0);
        x |= v & m;
        if (GAP) mm |= m;
    }
    if (GAP) x |= kClsDel & range_mask(0, (int)a.y, j4) & ~mm;
    return x;
}

