// bc_pileup.hip — the fused, position-tiled pileup kernel (kernel 1 + kernel 2 in ONE launch).
//
// Layout: the reference is cut into 64-position tiles; a tile is owned by a group of S waves
// whose 64 lanes each OWN one reference position.  Reads are coordinate-sorted, so the reads
// overlapping a tile form one contiguous index range, found in-kernel by a 64-ary search over
// pos[].  Each read of that range is resolved once per tile: every lane looks up the read's
// CIGAR at its own position (count.cpp:40-96) and adds the base / deletion it sees to a packed
// register counter.  No atomics and no histogram memset: the S waves of a group are reduced
// through LDS, the tile's counts are written once with coalesced stores (count.cpp's
// baseCounts), and the per-position statistics of main.py:29-53 are computed in the same
// launch (kernel 2 fused), the 2k fp64 terms of a tile spread over the group's lanes.
//
// Lanes at positions >= L (the last, partial tile and "edge" tiles past the reference end,
// up to the furthest read end) do not count: a counted event there is the reference's
// std::out_of_range (count.cpp:60-65,85) and is recorded as the first offending read index.
#include <cstring>

#include "bc_internal.h"

namespace bc {
namespace {

constexpr int kTile = 64;
// BAM 4-bit code -> count column (A0 C1 G2 T3 N5); 6 = not counted (junk field).
// Same letter mapping as count.cpp:58-65 through pysam's "=ACMGRSVTWYHKDBN" decode.
constexpr unsigned long long kNibCol6 = 0x5666666366626106ull;
constexpr int kField = 10;  // packed counter: six 10-bit fields + junk at bit 60; flush < 1024
constexpr int kJunk = 60;
constexpr int kBatch = 8;   // reads whose sequence loads are in flight together
constexpr int kPre = 8;     // CIGAR words preloaded per read (lane-parallel)
constexpr uint32_t kNone = 0xFFFFFFFFu;  // packed event: none
constexpr uint32_t kDel = 0x80000000u;   // packed event: deletion / ref-skip

__device__ __forceinline__ unsigned nib_col6(unsigned nib) { return (unsigned)(kNibCol6 >> (nib * 4)) & 0xFu; }
__device__ __forceinline__ bool mlike(uint32_t op) { return op == 0 || op == 7 || op == 8; }
__device__ __forceinline__ bool dlike(uint32_t op) { return op == 2 || op == 3; }
__device__ __forceinline__ bool qcons(uint32_t op) { return op == 0 || op == 1 || op == 7 || op == 8; }
__device__ __forceinline__ uint32_t rdl(uint32_t v, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, l); }

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
};

// First index i in [0, n) with pos[i] >= v (n if none), by one wave: 64 probes per round.
__device__ __forceinline__ int64_t lower_bound64(const int32_t* pos, int64_t n, int64_t v, int lane) {
    int64_t lo = 0, hi = n;  // answer in [lo, hi]
    while (hi - lo > 64) {
        const int64_t step = (hi - lo) / 65;
        const int64_t idx = lo + (int64_t)(lane + 1) * (step > 0 ? step : 1);
        const bool less = idx < hi && (int64_t)pos[idx] < v;
        const unsigned long long m = __ballot(less);
        const int c = __popcll(m);  // sorted: the lanes with pos < v are a prefix
        const int64_t s = step > 0 ? step : 1;
        const int64_t nlo = c ? lo + (int64_t)c * s + 1 : lo;
        const int64_t nhi = (c < 64 && lo + (int64_t)(c + 1) * s < hi) ? lo + (int64_t)(c + 1) * s : hi;
        lo = nlo;
        hi = nhi;
    }
    const int64_t idx = lo + lane;
    const bool less = idx < hi && (int64_t)pos[idx] < v;
    return lo + __popcll(__ballot(less));
}

// Packed event of read r (its CIGAR in w[]) at event index j (lane position - start):
// nibble index of the aligned base, kDel | 0 for a deletion / skip, kNone otherwise.  The op
// loop is uniform; only ops overlapping the tile window [jlo, jlo + 63] do per-lane work.
__device__ __forceinline__ uint32_t resolve(int j, int jlo, uint32_t cn, const uint32_t (&w)[kPre], uint32_t sn,
                                            const uint32_t* cg) {
    uint32_t e = kNone;
    const int jhi = jlo + kTile - 1;
    uint32_t rc = 0, qc = 0;
    const uint32_t nk = cn < (uint32_t)kPre ? cn : (uint32_t)kPre;
#pragma unroll
    for (int k = 0; k < kPre; ++k) {
        if ((uint32_t)k < nk) {
            const uint32_t op = w[k] & 15u, len = w[k] >> 4;
            if (mlike(op) || dlike(op)) {
                if ((int)(rc + len) > jlo && (int)rc <= jhi) {
                    const uint32_t d = (uint32_t)(j - (int)rc);
                    if (d < len) e = mlike(op) ? sn + qc + d : kDel;
                }
                rc += len;
            }
            if (qcons(op)) qc += len;
        }
    }
    for (uint32_t k = kPre; k < cn && (int)rc <= jhi; ++k) {  // long CIGARs: rest from memory
        const uint32_t wk = cg[k];
        const uint32_t op = wk & 15u, len = wk >> 4;
        if (mlike(op) || dlike(op)) {
            const uint32_t d = (uint32_t)(j - (int)rc);
            if (d < len) e = mlike(op) ? sn + qc + d : kDel;
            rc += len;
        }
        if (qcons(op)) qc += len;
    }
    return e;
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
        const unsigned nib = (e & 1u) ? (byte & 15u) : (byte >> 4);
        col = nib_col6(nib);
        ok = e != kNone && col != 6u;
        if (QUAL) ok = ok && qv >= mbq;
    }
    if (beyond) {
        if (ok && ridx < bad) bad = ridx;
        ok = false;
    }
    acc += 1ull << (ok ? col * kField : (unsigned)kJunk);
}

template <bool QUAL, int K, bool STATS>
__global__ __launch_bounds__(1024) void k_pileup(PileArgs A) {
    // reduction area: [16 waves][6][64] u32; reused as the stats terms [4 groups][12][64] f64
    __shared__ __attribute__((aligned(16))) unsigned char smem[16 * 6 * kTile * 4];
    __shared__ uint32_t fin[4][6][kTile];  // final counts of each group's tile
    uint32_t* red = (uint32_t*)smem;
    double* terms = (double*)smem;

    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nw = blockDim.x >> 6;
    const int S = A.S;
    const int g = wave / S, ws = wave - g * S;
    const int groups = nw / S;
    const int64_t nblk_tiles = (A.n_tiles + groups - 1) / groups;
    const int64_t L = A.L;

    for (int64_t bt = blockIdx.x; bt < nblk_tiles; bt += gridDim.x) {
        const int64_t t = bt * groups + g;
        const int64_t t0 = t * kTile;
        const int64_t P = t0 + lane;
        uint32_t cnt[6] = {0, 0, 0, 0, 0, 0};
        int64_t bad = INT64_MAX;
        if (t < A.n_tiles) {
            const int64_t lo = lower_bound64(A.pos, A.n, t0 - A.max_span + 1, lane);
            const int64_t hi = lower_bound64(A.pos, A.n, t0 + kTile, lane);
            const bool edge = t0 + kTile > L;  // uniform
            const bool beyond = P >= L;
            unsigned long long acc = 0;
            int pending = 0;
            for (int64_t base = lo + (int64_t)ws * 64; base < hi; base += (int64_t)S * 64) {
                const int nr = (int)((hi - base) < 64 ? (hi - base) : 64);
                uint32_t mpos = 0, mcn = 0, msn = 0, mcb = 0, mw[kPre];
#pragma unroll
                for (int i = 0; i < kPre; ++i) mw[i] = 0;
                bool simple = true;
                if (lane < nr) {
                    const int64_t r = base + lane;
                    mpos = (uint32_t)A.pos[r];
                    mcb = A.cig_beg[r];
                    mcn = A.cig_n[r];
                    msn = A.seq_nib[r];
                    mw[0] = mcn ? A.cigar[mcb] : 0u;
                    simple = mcn == 1 && mlike(mw[0] & 15u);
                }
                const bool fast = __all(simple);  // every read of the chunk is one M/=/X op
                if (!fast && lane < nr) {
#pragma unroll
                    for (int i = 1; i < kPre; ++i)
                        if ((uint32_t)i < mcn) mw[i] = A.cigar[mcb + i];
                }
                if (pending + nr >= (1 << kField) - 1) {
                    flush_acc(acc, cnt);
                    pending = 0;
                }
                pending += nr;
                for (int r0 = 0; r0 < nr; r0 += kBatch) {
                    uint32_t e[kBatch];
                    if (fast) {
#pragma unroll
                        for (int u = 0; u < kBatch; ++u) {
                            e[u] = kNone;
                            if (r0 + u < nr) {
                                const uint32_t j = (uint32_t)(P - (int64_t)(int32_t)rdl(mpos, r0 + u));
                                if (j < (rdl(mw[0], r0 + u) >> 4)) e[u] = rdl(msn, r0 + u) + j;
                            }
                        }
                    } else {
                        // rolled resolver; results shift through e[] (one code copy, 8 moves)
#pragma unroll
                        for (int u = 0; u < kBatch; ++u) e[u] = kNone;
                        for (int u = 0; u < kBatch; ++u) {
                            uint32_t x = kNone;
                            const int r = r0 + u;
                            if (r < nr) {
                                const int p0 = (int)rdl(mpos, r);
                                uint32_t w[kPre];
#pragma unroll
                                for (int i = 0; i < kPre; ++i) w[i] = rdl(mw[i], r);
                                x = resolve((int)(P - p0), (int)(t0 - p0), rdl(mcn, r), w, rdl(msn, r),
                                            A.cigar + rdl(mcb, r));
                            }
#pragma unroll
                            for (int v = kBatch - 1; v > 0; --v) e[v] = e[v - 1];
                            e[0] = x;  // after the loop e[kBatch-1-u] holds read r0+u
                        }
                    }
                    uint32_t byte[kBatch], qv[kBatch];
#pragma unroll
                    for (int u = 0; u < kBatch; ++u) {
                        byte[u] = 0;
                        qv[u] = 0;
                        if (e[u] < kDel) {
                            byte[u] = A.seq[e[u] >> 1];
                            if (QUAL) qv[u] = A.qual[e[u]];
                        }
                    }
#pragma unroll
                    for (int u = 0; u < kBatch; ++u) {
                        const int r = fast ? r0 + u : r0 + (kBatch - 1 - u);
                        count_event<QUAL>(e[u], byte[u], qv[u], A.mbq, edge && beyond, base + r, acc, bad);
                    }
                }
            }
            flush_acc(acc, cnt);
            if (edge) {  // first offending read of this tile (std::out_of_range in the reference)
                for (int o = 32; o > 0; o >>= 1) {
                    const int64_t b2 = __shfl_down(bad, o);
                    bad = b2 < bad ? b2 : bad;
                }
                if (lane == 0 && bad != INT64_MAX) atomicMin(A.err, (unsigned long long)bad);
            }
        }
        // ---- reduce the S waves of the group through LDS
        if (S > 1) {
#pragma unroll
            for (int c = 0; c < K; ++c) red[(wave * K + c) * kTile + lane] = cnt[c];
            __syncthreads();
            if (ws == 0)
                for (int w2 = wave + 1; w2 < wave + S; ++w2) {
#pragma unroll
                    for (int c = 0; c < K; ++c) cnt[c] += red[(w2 * K + c) * kTile + lane];
                }
        }
        const bool own = t < A.n_tiles && t0 < L;  // tile holds real positions
        if (ws == 0) {
#pragma unroll
            for (int c = 0; c < K; ++c) {
                if (own && P < L) {
                    int32_t* dst = A.counts + (int64_t)c * L + P;
                    if (A.accumulate) cnt[c] += (uint32_t)*dst;
                    *dst = (int32_t)cnt[c];
                }
                fin[g][c][lane] = cnt[c];
            }
        }
        if (!STATS) {
            if (S > 1) __syncthreads();
            continue;
        }
        __syncthreads();
        // ---- fused kernel 2: terms p*log2(p) of the primary (c < K) and secondary (K <= s < 2K)
        //      distributions, one per lane over the group, then ordered sums per position
        //      (main.py:37-53; CPython sums left to right from int 0)
        if (own) {
            for (int slot = ws * 64 + lane; slot < 2 * K * kTile; slot += S * 64) {
                const int sc = slot / kTile, p = slot % kTile;
                const int64_t Pp = t0 + p;
                if (Pp >= L) continue;
                uint32_t c[6];
                int64_t cov = 0;
                int am = 0;
#pragma unroll
                for (int j = 0; j < K; ++j) {
                    c[j] = fin[g][j][p];
                    cov += c[j];
                    if (c[j] > c[am]) am = j;  // np.argmax: first maximum
                }
                double term = 0.0;
                if (sc < K) {
                    if (cov != 0) {
                        const double pj = (double)c[sc] / (double)cov;
                        if (A.pc) A.pc[(int64_t)sc * L + Pp] = 100.0 * pj;
                        if (c[sc] != 0) term = -(pj * log2(pj));
                    } else if (A.pc) {
                        A.pc[(int64_t)sc * L + Pp] = -1.0;
                    }
                } else {
                    const int j = sc - K;
                    const int64_t cov2 = cov - c[am];
                    if (cov2 != 0 && j != am && c[j] != 0) {
                        const double q = (double)c[j] / (double)cov2;
                        term = -(q * log2(q));
                    }
                }
                terms[(g * 2 * K + sc) * kTile + p] = term;
            }
        }
        __syncthreads();
        if (own && ws == 0 && P < L) {
            int64_t cov = 0;
            uint32_t mx = 0;
#pragma unroll
            for (int j = 0; j < K; ++j) {
                cov += cnt[j];
                mx = cnt[j] > mx ? cnt[j] : mx;
            }
            A.cov[P] = (int32_t)cov;
            double h = 1.0, h2 = 1.0;
            if (cov != 0) {
                double s = 0.0;
#pragma unroll
                for (int j = 0; j < K; ++j)
                    if (cnt[j] != 0) s = s + terms[(g * 2 * K + j) * kTile + lane];
                h = A.nf * s;
                if (cov - (int64_t)mx != 0) {
                    double s2 = 0.0;
#pragma unroll
                    for (int j = 0; j < K; ++j) {
                        const double tj = terms[(g * 2 * K + K + j) * kTile + lane];
                        if (tj != 0.0) s2 = s2 + tj;
                    }
                    h2 = A.nf2 * s2;
                }
            }
            A.ent[P] = h;
            A.sec[P] = h2;
        }
        __syncthreads();
    }
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
    A.mbq = mbq;
    return A;
}

}  // namespace

hipError_t launch_pileup_tiles(hipStream_t s, const bc_reads& r, int64_t L, int64_t max_end, uint32_t mbq, int k,
                               bool stats, bool accumulate, double nf, double nf2, int32_t* counts, int32_t* cov,
                               double* pc, double* ent, double* sec, unsigned long long* d_err) {
    PileArgs A = make_args(r, L, mbq);
    const int64_t reach = max_end > L ? max_end : L;  // edge tiles up to the furthest read end
    A.n_tiles = (reach + kTile - 1) / kTile;
    if (A.n_tiles == 0) return hipSuccess;
    A.accumulate = accumulate ? 1 : 0;
    A.nf = nf;
    A.nf2 = nf2;
    A.counts = counts;
    A.cov = cov;
    A.pc = pc;
    A.ent = ent;
    A.sec = sec;
    A.err = d_err;
    // waves per tile from the mean number of reads a tile walks
    const double per_tile = L > 0 ? (double)r.n_reads * (double)(r.max_span + kTile) / (double)(kTile * (L + 1)) : 0.0;
    int S = 1;
    while (S < 16 && per_tile > 48.0 * S) S *= 2;
    if (const char* e = std::getenv("BC_TILE_WAVES")) S = std::max(1, std::min(16, std::atoi(e)));
    A.S = S;
    const int nw = S >= 4 ? S : 4;
    const int groups = nw / S;
    int64_t blocks = (A.n_tiles + groups - 1) / groups;
    const int64_t cap = 256 * 64;
    if (blocks > cap) blocks = cap;
    const dim3 grid((unsigned)blocks), block(64 * nw);
#define BC_PILE(Q, KK, ST) hipLaunchKernelGGL((k_pileup<Q, KK, ST>), grid, block, 0, s, A)
    if (mbq > 0) {
        if (k == 5) {
            if (stats) BC_PILE(true, 5, true); else BC_PILE(true, 5, false);
        } else {
            if (stats) BC_PILE(true, 6, true); else BC_PILE(true, 6, false);
        }
    } else {
        if (k == 5) {
            if (stats) BC_PILE(false, 5, true); else BC_PILE(false, 5, false);
        } else {
            if (stats) BC_PILE(false, 6, true); else BC_PILE(false, 6, false);
        }
    }
#undef BC_PILE
    return hipGetLastError();
}

}  // namespace bc
