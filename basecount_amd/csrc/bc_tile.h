// bc_tile.h — the position-tiled walk shared by the fused pileup kernels (bc_pileup.hip) and the
// read-parallel summary (bc_sum.hip): kernel arguments, the per-chunk CIGAR decode + staging +
// SWAR walk of one 64-position tile (process_chunk), the read-range search and numpy's leaf
// sums.  Included once per translation unit (anonymous namespace: each gets its own copy).
#pragma once
#include <cstdio>
#include <cstring>

#include "bc_internal.h"
#include "bc_log2.h"
#include "bc_stats.h"

namespace bc {
namespace {

constexpr int kStage = 6144;     // LDS bytes per wave for a chunk's sequence (64 reads x <= 190 bp)
#include "bc_walk.h"

constexpr int kTile = 64;
constexpr int kField = 10;  // packed counter: six 10-bit fields + junk at bit 60; flush < 1024
constexpr int kJunk = 60;
constexpr int kBatch = 8;   // reads whose sequence loads are in flight together
constexpr int kStageRegion = kStage + 32;  // + one 16-byte pad before and after

struct PileArgs {
    const int32_t* pos;
    const uint32_t* cig_beg;
    const uint32_t* cig_n;
    const uint32_t* seq_nib;
    const uint32_t* cigar;
    const uint8_t* seq;
    const uint8_t* qual;
    int64_t n;
    int64_t L;
    int64_t n_tiles;  // tiles incl. edge tiles up to the furthest read end
    int max_span;
    uint32_t mbq;
    int S;            // waves per tile group
    int accumulate;
    double nf, nf2;
    int32_t* counts;  // [k][L]
    int32_t* cov;
    double* pc;       // [k][L] or NULL
    double* ent;
    double* sec;
    unsigned long long* err;
    const int2* trange;  // bc_reads.tile_reads: [lo, hi) per tile t < n_trange, else searched
    int64_t n_trange;
    int64_t seq_words;   // readable 32-bit words of seq (bc_seq_event_bytes / 4)
    int64_t qual_bytes;
    int64_t tiles_per_wave;  // k_pileup_solo: consecutive tiles swept by one wave
    // k_pileup_solo with summary partials (bc_pileup_partials): for every quarter (2048
    // positions, a subtree of numpy's pairwise tree) of the whole buffers [0, full_chunks), its
    // pairwise entropy sum and exact coverage / non-zero sums
    double* sub_ent;
    long long* sub_cov;
    long long* sub_nz;
    int64_t full_chunks;
    // k_pileup_solo without per-position stores (STORE = false, summary only): the coverage and
    // entropy of the positions >= full_chunks * 8192 (the last partial buffer), at P - that
    int32_t* cov_tail;
    double* ent_tail;
    // the read-parallel summary (k_sum_reads / k_sum_exact / k_sum_buffers): per 128-position
    // leaf of the whole buffers, the counted positions of single-read coverage (leaf_cnt) and
    // the slot + 1 of a leaf some position of which two reads cover (leaf_mark, 0 = none); per
    // slot the leaf (dlist) and its exact pairwise sum / coverage (dval / dcov)
    int32_t* leaf_cnt;
    int32_t* leaf_mark;
    int32_t* dlist;
    int32_t* ndirty;
    double* dval;
    long long* dcov;
    int64_t nleaf;
    int64_t n_tail_tiles;  // tiles of the last partial buffer (k_sum_exact's first work items)
    int ablate;  // diagnostic only (BC_ABLATE): 1 no reads, 2 no search, 4 no walk, 8 no stats
                 // math, 16 no stores, 32 no sequence staging
    unsigned long long* trace;  // diagnostic only (BC_TRACE): per-wave phase stamps, else null
};

// Diagnostic phase stamps (BC_TRACE builds the buffer; null otherwise): s_memrealtime (100 MHz,
// chip-wide) of phase `ph` of this wave, written by lane 0 with a vector store.
constexpr int kTracePhases = 12;
// Compiled in only with -DBC_PHASE_TRACE (scripts/trace_phases.py): the stamps cost registers.
__device__ __forceinline__ void trace_stamp(const PileArgs& A, int ph) {
#ifdef BC_PHASE_TRACE
    if (A.trace && (threadIdx.x & 63) == 0)
        A.trace[((size_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * kTracePhases + ph] =
            __builtin_amdgcn_s_memrealtime();
#else
    (void)A;
    (void)ph;
#endif
}

// Packed event of a "complex" read (more than 8 CIGAR ops, more than 4 runs, or huge indels)
// at event index j (lane position - start): nibble index of the aligned base, kDel for a deletion
// / skip, kNone otherwise.  The op loop is uniform (scalar loads); only ops overlapping the tile
// window [jlo, jlo + 63] do per-lane work.  Rare: typical reads take the run tables below.
__device__ __forceinline__ uint32_t resolve_slow(int j, int jlo, uint32_t cn, uint32_t sn, const uint32_t* cg) {
    uint32_t e = kNone;
    const int jhi = jlo + kTile - 1;
    uint32_t rc = 0, qc = 0;
    for (uint32_t k = 0; k < cn && (int)rc <= jhi; ++k) {
        const uint32_t wk = cg[k];
        const uint32_t op = wk & 15u, len = wk >> 4;
        if (mlike(op) || dlike(op)) {
            if ((int)(rc + len) > jlo) {
                const uint32_t d = (uint32_t)(j - (int)rc);
                if (d < len) e = mlike(op) ? sn + qc + d : kDel;
            }
            rc += len;
        }
        if (qcons(op)) qc += len;
    }
    return e;
}

// First indices with pos >= v_lo (lanes 0-31) and pos >= v_hi (lanes 32-63), searched together:
// 32 probes per half-wave per round.  Returns {lower_bound(v_lo), lower_bound(v_hi)}.  IT: the
// index arithmetic (uint32_t for batches of < 2^31 reads: the rounds are mostly 64-bit VALU
// otherwise).
template <typename IT>
__device__ __forceinline__ void lower_bound_pair_t(const int32_t* pos, IT n, int64_t v_lo, int64_t v_hi, int lane,
                                                   int64_t& r_lo, int64_t& r_hi) {
    const int h = lane >> 5, l = lane & 31;
    const int64_t v = h ? v_hi : v_lo;
    IT lo = 0, hi = n;  // answer in [lo, hi] (per half)
    while (__any(hi - lo > 32)) {
        const bool act = hi - lo > 32;
        const IT s = act ? ((hi - lo) / 33 > 0 ? (hi - lo) / 33 : 1) : 1;
        const IT idx = lo + (IT)(l + 1) * s;
        const bool less = act && idx < hi && (int64_t)pos[idx] < v;
        const unsigned long long m = __ballot(less);
        const IT c = (IT)__popc(h ? (unsigned)(m >> 32) : (unsigned)m);
        if (act) {
            const IT nlo = c ? lo + c * s + 1 : lo;
            const IT nhi = (c < 32 && lo + (c + 1) * s < hi) ? lo + (c + 1) * s : hi;
            lo = nlo;
            hi = nhi;
        }
    }
    const IT idx = lo + (IT)l;
    const bool less = idx < hi && (int64_t)pos[idx] < v;
    const unsigned long long m = __ballot(less);
    const int64_t res = (int64_t)lo + __popc(h ? (unsigned)(m >> 32) : (unsigned)m);
    // wave-uniform results (SGPRs): the chunk loops over [r_lo, r_hi) stay scalar
    const uint32_t rl = (uint32_t)res, rh = (uint32_t)((uint64_t)res >> 32);
    r_lo = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)rh, 0) << 32) |
                     (uint32_t)__builtin_amdgcn_readlane((int)rl, 0));
    r_hi = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)rh, 32) << 32) |
                     (uint32_t)__builtin_amdgcn_readlane((int)rl, 32));
}
__device__ __forceinline__ void lower_bound_pair(const int32_t* pos, int64_t n, int64_t v_lo, int64_t v_hi, int lane,
                                                 int64_t& r_lo, int64_t& r_hi) {
    if (n < (int64_t)0x7FFFFFC0)
        lower_bound_pair_t<uint32_t>(pos, (uint32_t)n, v_lo, v_hi, lane, r_lo, r_hi);
    else
        lower_bound_pair_t<int64_t>(pos, n, v_lo, v_hi, lane, r_lo, r_hi);
}

// Four lower bounds searched together, a quarter-wave (16 lanes, 16 probes per round) per key:
// about as many rounds as lower_bound_pair's two (17-ary instead of 33-ary), for two tiles' ranges
// at once.  r[q] = lower_bound(v[q]), wave-uniform.
template <typename IT>
__device__ __forceinline__ void lower_bound_quad_t(const int32_t* pos, IT n, const int64_t (&v)[4], int lane,
                                                   int64_t (&r)[4]) {
    const int h = lane >> 4, l = lane & 15;
    const int64_t key = h == 0 ? v[0] : h == 1 ? v[1] : h == 2 ? v[2] : v[3];
    IT lo = 0, hi = n;  // answer in [lo, hi] (per quarter)
    while (__any(hi - lo > 16)) {
        const bool act = hi - lo > 16;
        const IT s = act ? ((hi - lo) / 17 > 0 ? (hi - lo) / 17 : 1) : 1;
        const IT idx = lo + (IT)(l + 1) * s;
        const bool less = act && idx < hi && (int64_t)pos[idx] < key;
        const unsigned long long m = __ballot(less);
        const IT c = (IT)__popc((unsigned)(m >> (16 * h)) & 0xFFFFu);
        if (act) {
            const IT nlo = c ? lo + c * s + 1 : lo;
            const IT nhi = (c < 16 && lo + (c + 1) * s < hi) ? lo + (c + 1) * s : hi;
            lo = nlo;
            hi = nhi;
        }
    }
    const IT idx = lo + (IT)l;
    const bool less = idx < hi && (int64_t)pos[idx] < key;
    const unsigned long long m = __ballot(less);
    const int64_t res = (int64_t)lo + __popc((unsigned)(m >> (16 * h)) & 0xFFFFu);
    const uint32_t rl = (uint32_t)res, rh = (uint32_t)((uint64_t)res >> 32);
#pragma unroll
    for (int q = 0; q < 4; ++q)
        r[q] = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)rh, 16 * q) << 32) |
                         (uint32_t)__builtin_amdgcn_readlane((int)rl, 16 * q));
}
__device__ __forceinline__ void lower_bound_quad(const int32_t* pos, int64_t n, const int64_t (&v)[4], int lane,
                                                 int64_t (&r)[4]) {
    if (n < (int64_t)0x7FFFFFC0)
        lower_bound_quad_t<uint32_t>(pos, (uint32_t)n, v, lane, r);
    else
        lower_bound_quad_t<int64_t>(pos, n, v, lane, r);
}

__device__ __forceinline__ void flush_acc(unsigned long long& acc, uint32_t (&cnt)[6]) {
#pragma unroll
    for (int c = 0; c < 6; ++c) cnt[c] += (uint32_t)(acc >> (kField * c)) & ((1u << kField) - 1);
    acc = 0;
}

// Count one event: acc field += 1 for its column (junk field when not counted).  A counted
// event at a position >= L is the reference's out_of_range: remember the read.
template <bool QUAL>
__device__ __forceinline__ void count_event(uint32_t e, uint32_t byte, uint32_t qv, uint32_t mbq, bool beyond,
                                            int64_t ridx, unsigned long long& acc, int64_t& bad) {
    unsigned col;
    bool ok;
    if (e == kDel) {
        col = 4;
        ok = true;
    } else {
        col = nib_col6((byte >> ((e & 1u) * 4)) & 15u);
        ok = e != kNone && col != 6u;
        if (QUAL) ok = ok && qv >= mbq;
    }
    if (beyond) {
        if (ok && ridx < bad) bad = ridx;
        ok = false;
    }
    acc += 1ull << (ok ? col * kField : (unsigned)kJunk);
}

// Fused kernel 2, part 1: the fp64 terms -(p*log2(p)) of a tile's primary (c < K) and
// secondary (K <= s < 2K) distributions, one per lane over the group (main.py:37-53), plus the
// percentages.  Kept out of line: inlined, the log2 constants would be hoisted into registers
// for the whole kernel and push the read walk into spills.
template <int K>
__device__ __attribute__((noinline)) void tile_terms(const PileArgs& A, const uint32_t* fin_g, double* terms_g,
                                                     int64_t t0, int first, int stride) {
    const int64_t L = A.L;
    for (int slot = first; slot < 2 * K * kTile; slot += stride) {
        // slot order A C G T, A2 C2 G2 T2, DS DS2 [N N2]: the deletion / N columns, zero in most
        // batches, fall in the last (partial) round of the group's lanes
        const int q = slot / kTile, p = slot % kTile;
        const int sc = q < 4 ? q : (q < 8 ? K + q - 4 : 4 + ((q - 8) >> 1) + ((q - 8) & 1) * K);
        const int64_t Pp = t0 + p;
        if (Pp >= L) continue;
        uint32_t c[6];
        int64_t cov = 0;
        int am = 0;
#pragma unroll
        for (int j = 0; j < K; ++j) {
            c[j] = fin_g[j * kTile + p];
            cov += c[j];
            if (c[j] > c[am]) am = j;  // np.argmax: first maximum
        }
        double term = 0.0;
        if (sc < K) {
            if (cov != 0) {
                if (c[sc] != 0) {
                    const double pj = (double)c[sc] / (double)cov;
                    if (A.pc) A.pc[(int64_t)sc * L + Pp] = 100.0 * pj;
                    term = -(pj * glibc_log2(pj));
                } else if (A.pc) {
                    A.pc[(int64_t)sc * L + Pp] = 0.0;  // 100 * (0 / cov), exactly
                }
            } else if (A.pc) {
                A.pc[(int64_t)sc * L + Pp] = -1.0;
            }
        } else {
            const int j = sc - K;
            const int64_t cov2 = cov - c[am];
            if (cov2 != 0 && j != am && c[j] != 0) {
                const double q = (double)c[j] / (double)cov2;
                term = -(q * glibc_log2(q));
            }
        }
        terms_g[sc * kTile + p] = term;
    }
}

// Complex chunks (a read with more than 8 CIGAR ops, more than 4 runs or huge indels): lanes own
// positions, each read of the chunk is resolved at the lane's position by walking its CIGAR
// from memory (records in LDS hold absolute sequence nibble indices), kBatch reads at a time.
template <bool QUAL>
__device__ __forceinline__ void walk_complex(const PileArgs& A, const uint4* rec, int nr, int64_t P, int64_t t0,
                                             int64_t rbase, bool beyond, uint32_t mcn, uint32_t mcb,
                                             unsigned long long& acc, int64_t& bad) {
    const uint8_t* sp = A.seq ? A.seq : (const uint8_t*)A.pos;  // never dereferenced at a bad index
    for (int r0 = 0; r0 < nr; r0 += kBatch) {
        uint32_t e[kBatch];
        for (int u = 0; u < kBatch; ++u) {
            const int r = r0 + u;
            uint32_t x = kNone;
            if (r < nr) {
                const uint4 a = rec[r * 3];
                x = resolve_slow((int)(P - (int64_t)(int32_t)a.x), (int)(t0 - (int32_t)a.x), rdl(mcn, r), a.y,
                                 A.cigar + rdl(mcb, r));
            }
#pragma unroll
            for (int v = kBatch - 1; v > 0; --v) e[v] = e[v - 1];
            e[0] = x;
        }
#pragma unroll
        for (int u = 0; u < kBatch / 2; ++u) {  // e[kBatch-1-u] holds read r0+u
            const uint32_t t = e[u];
            e[u] = e[kBatch - 1 - u];
            e[kBatch - 1 - u] = t;
        }
        uint32_t byte[kBatch], qv[kBatch];
#pragma unroll
        for (int u = 0; u < kBatch; ++u) {
            const uint32_t idx = e[u] < kDel ? e[u] : 0u;
            byte[u] = (uint32_t)sp[idx >> 1];
            qv[u] = QUAL ? (uint32_t)A.qual[idx] : 0u;
        }
#pragma unroll
        for (int u = 0; u < kBatch; ++u)
            count_event<QUAL>(e[u], byte[u], qv[u], A.mbq, beyond, rbase + r0 + u, acc, bad);
    }
}

// Walk a chunk of nr reads (records padded with empty ones to 64) with lane = (window g, read
// slot s): reads it*8 + s and it*8 + 8 + s in step it (two independent LDS chains in flight;
// rounding the steps up to even only ever touches padding records).  NR: the chunk's largest
// run count (1, 2, 4).  nr and it4 are wave-uniform.
template <int NR, bool GAP, bool STAGED, bool QUAL, int NC>
__device__ __forceinline__ void walk_swar(const PileArgs& A, const uint4* rec, const uint32_t* words, int nr, int gb,
                                          int s8, int64_t rbase, bool edge, uint32_t bmask, Swar& W, int& it4,
                                          uint32_t (&cnt)[6], int64_t& bad) {
    const SeqSrc src{words, STAGED ? (int64_t)(kStage / 4) : A.seq_words, A.qual, A.qual_bytes, A.mbq};
    const int iters = (((nr + 7) >> 3) + 1) & ~1;
    for (int it = 0; it < iters; it += 2) {
        const int r0 = it * 8 + s8, r1 = r0 + 8;
        uint32_t x0 = window_events<NR, GAP, STAGED, QUAL>(src, rec, r0, gb);
        uint32_t x1 = window_events<NR, GAP, STAGED, QUAL>(src, rec, r1, gb);
        if (edge) {  // events at positions >= L: the reference's out_of_range
            if ((x0 & bmask) && rbase + r0 < bad) bad = rbase + r0;
            if ((x1 & bmask) && rbase + r1 < bad) bad = rbase + r1;
            x0 &= ~bmask;
            x1 &= ~bmask;
        }
        swar_add<NC>(W, x0);
        swar_add<NC>(W, x1);
        it4 += 2;
        if (it4 >= 14) {  // every a4 field <= 14
            swar_fold<NC>(W, cnt, s8);
            it4 = 0;
        }
    }
}

constexpr int kFinBytes = 4 * 6 * kTile * 4;

// dynamic LDS: [rec: nw x 3 KB][stage: nw x kStageRegion][fin: 6 KB].  Once a tile's walk is
// done, a wave's stage region holds its partial counts for the group reduction, and the first
// wave's region of a group then holds the group's fp64 terms (12 x 64 x 8 B).
constexpr int kRecBytes = kTile * 3 * 16;
static_assert(12 * kTile * 8 <= kStageRegion, "terms must fit a stage region");
__host__ __device__ inline size_t pileup_lds_bytes(int nw, int groups) {
    (void)groups;
    return (size_t)nw * (kRecBytes + kStageRegion) + kFinBytes;
}

// Per-read fields of a chunk (lane = read), loaded one chunk ahead of their use.
struct ReadFields {
    uint32_t pos, cb, cn, sn;
};
__device__ __forceinline__ ReadFields load_fields(const PileArgs& A, int64_t base, int nr, int lane) {
    ReadFields f{0u, 0u, 0u, 0u};
    if (lane < nr) {
        const int64_t r = base + lane;
        f.pos = (uint32_t)A.pos[r];
        f.cb = A.cig_beg[r];
        f.cn = A.cig_n[r];
        f.sn = A.seq_nib[r];
    }
    return f;
}

// Copy [lo, hi) of the BC_SEQ_EVENT buffer into the wave's stage with register loads, clearing the
// bases below min_base_quality (count.cpp:56).  Used with a quality threshold only (LDS-DMA
// cannot apply the mask).
template <bool QUAL>
__device__ __forceinline__ void stage_regs(const PileArgs& A, uint8_t* mystage, uint32_t seg_lo, uint32_t seg_hi,
                                           int lane, bool qual_vec) {
    for (uint32_t off = lane * 16u; off < seg_hi - seg_lo; off += 1024u) {
        uint4 v = *(const uint4*)(A.seq + seg_lo + off);  // padded buffer: in bounds
        if (QUAL) {
            const int64_t q0 = 2 * ((int64_t)seg_lo + off);  // first base of the piece
            uint32_t qw[8];
            if (qual_vec && q0 + 32 <= A.qual_bytes) {
                const uint4 qa = *(const uint4*)(A.qual + q0), qb = *(const uint4*)(A.qual + q0 + 16);
                qw[0] = qa.x, qw[1] = qa.y, qw[2] = qa.z, qw[3] = qa.w;
                qw[4] = qb.x, qw[5] = qb.y, qw[6] = qb.z, qw[7] = qb.w;
            } else {
                for (int i = 0; i < 8; ++i) {
                    qw[i] = 0;
                    for (int bb = 0; bb < 4; ++bb) {
                        const int64_t at = q0 + 4 * i + bb;
                        if (at < A.qual_bytes) qw[i] |= (uint32_t)A.qual[at] << (8 * bb);
                    }
                }
            }
            v.x &= qual_nibmask(qw[0], qw[1], A.mbq);
            v.y &= qual_nibmask(qw[2], qw[3], A.mbq);
            v.z &= qual_nibmask(qw[4], qw[5], A.mbq);
            v.w &= qual_nibmask(qw[6], qw[7], A.mbq);
        }
        *(uint4*)(mystage + off) = v;
    }
}

constexpr uint32_t kSpecSlack = 128;  // bytes staged beyond the last read's first base

// One chunk of nr <= 64 reads [base, base + nr) of a tile, walked by one wave: decode the reads'
// CIGARs (fields F were loaded one chunk ahead), stage their sequence into the wave's LDS region
// and walk them (SWAR windows, or the per-position CIGAR walk for complex reads).  Counts
// accumulate in W / cnt (lane = tile position t0 + lane), the first out-of-range read in `bad`.
// On return F holds the fields of the wave's next chunk [next_base, next_base + next_nr),
// loaded while this chunk is walked.
//
// Latency: without a quality threshold the sequence is staged SPECULATIVELY (reads of a sorted
// batch usually lie in file order: [first read's seq, last read's seq + slack)) by LDS-DMA,
// issued together with the CIGAR loads, so a chunk costs one memory round trip before its walk;
// the exact segment, known after the decode, is restaged only when it is not covered.
template <bool QUAL, int K>
__device__ __forceinline__ void process_chunk(const PileArgs& A, int64_t base, int nr, ReadFields& F,
                                              int64_t next_base, int next_nr, int lane, int s8, int gb, int64_t t0,
                                              int64_t P, bool edge, bool beyond, uint32_t bmask, uint4* myrec,
                                              uint8_t* mystage, bool qual_vec, Swar& W, int& it4, uint32_t (&cnt)[6],
                                              unsigned long long& acc, int& pending, int64_t& bad) {
    // ---- chunk load: CIGAR -> run table (VALU), speculative staging in flight meanwhile
    RunTable T;
    const uint32_t mpos = F.pos, mcb = F.cb, mcn = F.cn, msn = F.sn;
    T.nrun = 0;
    T.complex = false;
    T.gap = false;
    T.span = 0;
    T.qlen = 0;
#pragma unroll
    for (int i = 0; i < kMaxRuns; ++i) T.st[i] = T.en[i] = 0, T.qd[i] = 0;
    // ops to decode: the wave's largest CIGAR (more than kPre -> complex anyway)
    const int cmax = (int)wave_reduce<true>(mcn < (uint32_t)kPre ? mcn : (uint32_t)kPre);
    uint32_t w[kPre];
#pragma unroll
    for (int i = 0; i < kPre; ++i) {
        w[i] = 0u;
        if (lane < nr && i < cmax && (uint32_t)i < mcn) w[i] = A.cigar[mcb + i];
    }
    const bool dma = !QUAL && !(BC_ABL(A) & 32);
    uint32_t spec_lo = 0, spec_hi = 0;
    bool spec = false;
    if (dma && !(BC_ABL(A) & 512)) {
        const uint32_t buf_end = (uint32_t)(A.seq_words * 4 < 0xFFFFFFFFll ? A.seq_words * 4 : 0xFFFFFFF0ll);
        spec_lo = (rdl(msn, 0) >> 1) & ~15u;
        spec_hi = (rdl(msn, nr - 1) >> 1) + kSpecSlack;
        spec_hi = spec_hi < buf_end ? spec_hi : buf_end;
        spec = spec_hi > spec_lo && spec_hi - spec_lo <= (uint32_t)kStage;
        if (spec) stage_dma<64>(mystage, A.seq + spec_lo, spec_hi - spec_lo, lane);
    }
    if (lane < nr) T = decode_runs(w, mcn, cmax);
    const bool cx = __any(T.complex);
    const bool gap = __any(T.gap);
    const int maxrun = (int)wave_reduce<true>((uint32_t)T.nrun);
    // ---- the chunk's exact sequence segment (BC_SEQ_EVENT bytes)
    uint32_t blo = 0xFFFFFFFFu, bhi = 0;
    if (lane < nr && T.qlen) {
        blo = msn >> 1;
        bhi = (msn + T.qlen + 1) >> 1;
    }
    uint32_t seg_lo = wave_reduce<false>(blo);
    const uint32_t seg_hi = wave_reduce<true>(bhi);
    seg_lo = seg_hi > seg_lo ? (seg_lo & ~15u) : 0u;
    const bool spec_ok = spec && !cx && (seg_hi <= seg_lo || (seg_lo >= spec_lo && seg_hi <= spec_hi));
    if (spec_ok) seg_lo = spec_lo;  // the stage holds [spec_lo, spec_hi)
    const bool staged = !cx && (spec_ok || seg_hi - seg_lo <= (uint32_t)kStage) && !(BC_ABL(A) & 32);
    if (spec && !spec_ok) stage_wait();  // the speculative copy must land before it is overwritten
    if (staged && !spec_ok) {
        if (dma) stage_dma<64>(mystage, A.seq + seg_lo, seg_hi - seg_lo, lane);
        else stage_regs<QUAL>(A, mystage, seg_lo, seg_hi, lane, qual_vec);
    }
    const uint32_t qbase = staged ? 2u * seg_lo : 0u;
    if (cx) {  // walk_complex reads {pos, absolute seq_nib}
        myrec[lane * 3] = make_uint4(mpos, msn, 0u, 0u);
    } else {
        uint32_t rr[kMaxRuns], nb[kMaxRuns];
#pragma unroll
        for (int k = 0; k < kMaxRuns; ++k) {
            rr[k] = pack_rr(T.st[k], T.en[k]);
            nb[k] = msn - qbase + (uint32_t)T.qd[k];
        }
        myrec[lane * 3] = make_uint4(mpos, T.span * 4u, rr[0], nb[0]);
        myrec[lane * 3 + 1] = make_uint4(rr[1], nb[1], rr[2], nb[2]);
        myrec[lane * 3 + 2] = make_uint4(rr[3], nb[3], 0u, 0u);
    }
    if (dma) stage_wait();  // LDS-DMA landed (hipcc does not track it)
    F = load_fields(A, next_base, next_nr, lane);  // in flight during the walk
    __builtin_amdgcn_wave_barrier();
    const int64_t rbase = base;
    if (BC_ABL(A) & 4) {
    } else if (cx) {
        if (pending + nr >= (1 << kField) - 1) {
            flush_acc(acc, cnt);
            pending = 0;
        }
        pending += nr;
        walk_complex<QUAL>(A, myrec, nr, P, t0, rbase, edge && beyond, mcn, mcb, acc, bad);
    } else {
        // separate calls keep the LDS / global address spaces visible to the compiler
#define BC_WALK(NR, GP, ST)                                                                                 \
walk_swar<NR, GP, ST, QUAL, K>(A, myrec, ST ? (const uint32_t*)mystage : (const uint32_t*)A.seq, nr, gb,   \
                       s8, rbase, edge, bmask, W, it4, cnt, bad)
#define BC_WALK_NR(GP, ST)                                                                                  \
do {                                                                                                    \
if (maxrun <= 1) BC_WALK(1, GP, ST);                                                                \
else if (maxrun == 2) BC_WALK(2, GP, ST);                                                           \
else BC_WALK(4, GP, ST);                                                                            \
} while (0)
        if (staged) {
            if (gap) BC_WALK_NR(true, true);
            else BC_WALK_NR(false, true);
        } else {
            if (gap) BC_WALK_NR(true, false);
            else BC_WALK_NR(false, false);
        }
#undef BC_WALK_NR
#undef BC_WALK
    }
}

// numpy's pairwise_sum of one 128-element leaf (pw_leaf of bc_kernels.hip for n = 128) from two
// consecutive tiles' entropies, one per lane: r_j = a[j] + a[8 + j] + ... + a[120 + j] in that
// order (eight accumulators), then ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7)).  A tile's 64
// values go through the wave's LDS scratch `tr` (one store, then lanes 0-7 read their 8 strided
// values): leaf_half takes the first tile's half of the chains, leaf_finish the second's and the
// combine.  The leaf is valid in lane 0.
__device__ __forceinline__ double leaf_half(double ea, int lane, double* tr) {
    tr[lane] = ea;
    __builtin_amdgcn_wave_barrier();
    const int j = lane & 7;
    double v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = tr[8 * i + j];
    double r = v[0];
#pragma unroll
    for (int i = 1; i < 8; ++i) r = r + v[i];
    __builtin_amdgcn_wave_barrier();
    return r;
}
// ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7)) of lanes 0-7 (through tr)
__device__ __forceinline__ double leaf_combine(double r, int lane, double* tr) {
    if (lane < 8) tr[lane] = r;
    __builtin_amdgcn_wave_barrier();
    const double leaf = ((tr[0] + tr[1]) + (tr[2] + tr[3])) + ((tr[4] + tr[5]) + (tr[6] + tr[7]));
    __builtin_amdgcn_wave_barrier();
    return leaf;
}
__device__ __forceinline__ double leaf_finish(double r, double eb, int lane, double* tr) {
    tr[lane] = eb;
    __builtin_amdgcn_wave_barrier();
    const int j = lane & 7;
    double v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = tr[8 * i + j];
#pragma unroll
    for (int i = 0; i < 8; ++i) r = r + v[i];
    __builtin_amdgcn_wave_barrier();
    return leaf_combine(r, lane, tr);
}
// The same for a tile with no reads (every entropy 1.0): no transposition needed.  The half is
// 1.0 + 1.0 + ... = 8.0 exactly; two such tiles make the leaf 128.0 exactly.
__device__ __forceinline__ double leaf_finish_ones(double r, int lane, double* tr) {
#pragma unroll
    for (int i = 0; i < 8; ++i) r = r + 1.0;
    return leaf_combine(r, lane, tr);
}

__device__ __forceinline__ long long wave_sum_i64(long long v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

PileArgs make_args(const bc_reads& r, int64_t L, uint32_t mbq) {
    PileArgs A;
    std::memset(&A, 0, sizeof A);
    A.pos = r.pos;
    A.cig_beg = r.cig_beg;
    A.cig_n = r.cig_n;
    A.seq_nib = r.seq_nib;
    A.cigar = r.cigar;
    A.seq = r.seq;
    A.qual = r.qual;
    A.n = r.n_reads;
    A.L = L;
    A.max_span = r.max_span;
    if (r.tile_reads && r.n_tiles > 0 && !((uintptr_t)r.tile_reads & 7u) && index_valid(r)) {
        A.trange = (const int2*)r.tile_reads;
        A.n_trange = r.n_tiles;
    }
    A.mbq = mbq;
    A.seq_words = (int64_t)(seq_event_bytes(r.seq_bytes) / 4);
    A.qual_bytes = r.qual ? r.qual_bytes : 0;
    return A;
}


}  // namespace
}  // namespace bc
