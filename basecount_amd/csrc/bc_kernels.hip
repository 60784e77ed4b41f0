// bc_kernels.hip — gfx950 kernels of the pileup counter.
//
//   k_count     kernel 1: CIGAR-expand + scatter-add (count.cpp:22-97)
//   k_span      helper  : max reference span of a batch (sizes the LDS windows of kernel 1)
//   k_stats     kernel 2: per-position coverage / percentages / entropies (main.py:14-79)
//   k_sum_*     summary : numpy-exact mean of coverage and entropy (main.py:479-485)
//   k_amplicon  amplicon: numpy-exact mean / median per tile window (main.py:519-551)
//
// Integer scatter, not a contraction: no MFMA.  Kernel 1 is bound by HBM (read records) and by
// the LDS atomic rate; see DESIGN.md for the roofline accounting.
#include <cstring>

#include "bc_internal.h"
#include "bc_log2.h"

namespace bc {
namespace {

// BAM 4-bit code -> count column.  The reference switches on the ASCII letter of
// query_alignment_sequence (count.cpp:58-65), which pysam decodes through "=ACMGRSVTWYHKDBN":
// A(1)->0, C(2)->1, G(4)->2, T(8)->3, N(15)->5; every other code ('=' and IUPAC) counts nowhere.
// Packed LUT, 4 bits per code, 0xF = not counted.
constexpr unsigned long long kNibCol = 0x5FFFFFF3FFF2F10Full;
__device__ __forceinline__ unsigned nib_col(unsigned nib) { return (unsigned)(kNibCol >> (nib * 4)) & 0xFu; }
// BC_SEQ_EVENT class -> count column: A 1->0, C 2->1, G 4->2, T 8->3, N 3->5, else 0xF.
constexpr unsigned long long kEvCol = 0xFFFFFFF3FFF2510Full;
// BAM code -> BC_SEQ_EVENT class (A 1, C 2, G 4, T 8, N 15 -> 3, others 0).
constexpr unsigned long long kNibClass = 0x3000000800040210ull;

__device__ __forceinline__ int64_t uni64(int64_t v) {
    int lo = __builtin_amdgcn_readfirstlane((int)(v & 0xffffffff));
    int hi = __builtin_amdgcn_readfirstlane((int)(v >> 32));
    return ((int64_t)hi << 32) | (uint32_t)lo;
}

struct CountArgs {
    const int32_t* pos;
    const uint32_t* cig_beg;
    const uint32_t* cig_n;
    const uint32_t* seq_nib;
    const uint32_t* cigar;
    const uint8_t* seq;
    const uint8_t* qual;
    int64_t n;
    int64_t ref_len;
    uint32_t mbq;
    int ncols;
    int rpb;        // reads per workgroup chunk
    int max_span;   // upper bound of any read's reference span
    int sorted;
    int layout;     // BC_SEQ_BAM / BC_SEQ_EVENT
    int32_t* hist;  // [ncols][ref_len]
    unsigned long long* err;
};

// Walk one read with the whole wave (i is wave-uniform).  Lanes map to consecutive reference
// events: event e of the read lies at reference position pos + e (M/=/X/D/N ops consume the
// reference contiguously), so a 64-event window is 64 consecutive positions -> conflict-free
// LDS addresses.  A scalar cursor (k, rc, qc) over the CIGAR skips ops that end before the
// window; the per-window scan only touches ops overlapping it.
template <bool QUAL, class Add>
__device__ __forceinline__ bool walk_read(const CountArgs& A, int64_t i, unsigned lane, Add&& add) {
    const int64_t p0 = A.pos[i];
    const uint32_t* cg = A.cigar + A.cig_beg[i];
    const uint32_t cn = A.cig_n[i];
    const uint32_t sn = A.seq_nib[i];
    bool bad = false;
    uint32_t k = 0, rc = 0, qc = 0;  // op k starts at reference offset rc, query offset qc
    for (uint32_t e0 = 0;; e0 += 64) {
        // advance past ops that end at or before e0 (query-only ops on the way add to qc)
        while (k < cn) {
            const uint32_t w = cg[k], op = w & 15u, len = w >> 4;
            const bool cref = (op == 0) | (op == 2) | (op == 3) | (op == 7) | (op == 8);
            const bool cqry = (op == 0) | (op == 1) | (op == 7) | (op == 8);
            if (cref && rc + len > e0) break;
            rc += cref ? len : 0u;
            qc += cqry ? len : 0u;
            ++k;
        }
        if (k >= cn) break;
        const uint32_t j = e0 + lane;
        int typ = 0;  // 1 = aligned base, 2 = deletion / ref-skip
        uint32_t qoff = 0;
        uint32_t rcs = rc, qcs = qc;
        for (uint32_t kk = k; kk < cn && rcs < e0 + 64u; ++kk) {
            const uint32_t w = cg[kk], op = w & 15u, len = w >> 4;
            const bool mref = (op == 0) | (op == 7) | (op == 8);
            const bool dref = (op == 2) | (op == 3);
            if (mref | dref) {
                const uint32_t d = j - rcs;
                if (d < len) {
                    typ = mref ? 1 : 2;
                    qoff = qcs + d;
                }
                rcs += len;
            }
            if (mref | (op == 1)) qcs += len;
        }
        if (typ) {
            unsigned col = 4;  // DS: counted with no quality test (count.cpp:80-90)
            bool counted = true;
            if (typ == 1) {
                const uint32_t ni = sn + qoff;
                const unsigned byte = A.seq[ni >> 1];
                if (A.layout == BC_SEQ_EVENT)
                    col = (unsigned)(kEvCol >> (((byte >> ((ni & 1u) * 4)) & 15u) * 4)) & 0xFu;
                else
                    col = nib_col((ni & 1u) ? (byte & 15u) : (byte >> 4));
                counted = col != 0xFu;
                if (QUAL) counted = counted && (uint32_t)A.qual[ni] >= A.mbq;  // count.cpp:56
            }
            if (counted) {
                const int64_t rp = p0 + (int64_t)j;
                if (rp >= A.ref_len || rp < 0)
                    bad = true;  // .at() would throw (count.cpp:60-65,85)
                else if ((int)col < A.ncols)
                    add(col, rp);
            }
        }
    }
    return bad;
}

template <bool QUAL>
__global__ __launch_bounds__(kCountThreads) void k_count(CountArgs A) {
    __shared__ uint32_t win[3 * kWinMax];  // planes {A|C, G|T, DS|N}, 16-bit halves
    const int64_t r0 = (int64_t)blockIdx.x * A.rpb;
    const int64_t r1 = r0 + A.rpb < A.n ? r0 + A.rpb : A.n;
    const unsigned lane = threadIdx.x & 63u;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    constexpr int kWaves = kCountThreads / 64;

    int64_t wbase = 0, wlen = 0;
    bool use_lds = false;
    if (A.sorted && A.max_span > 0) {
        wbase = A.pos[r0];
        wlen = (int64_t)A.pos[r1 - 1] - wbase + A.max_span;
        use_lds = wlen <= kWinMax;
    }
    if (use_lds) {
        for (int t = threadIdx.x; t < wlen; t += kCountThreads) {
            win[t] = 0;
            win[kWinMax + t] = 0;
            win[2 * kWinMax + t] = 0;
        }
        __syncthreads();
        for (int64_t i = r0 + wave; i < r1; i += kWaves) {
            const int64_t iu = uni64(i);
            bool bad = walk_read<QUAL>(A, iu, lane, [&](unsigned col, int64_t rp) {
                const int64_t idx = rp - wbase;
                if (idx >= 0 && idx < wlen)  // always true when pos is sorted and max_span holds
                    atomicAdd(&win[(col >> 1) * kWinMax + (int)idx], 1u << ((col & 1u) * 16));
                else
                    atomicAdd(&A.hist[(int64_t)col * A.ref_len + rp], 1);
            });
            if (__any(bad) && lane == 0) atomicMin(A.err, (unsigned long long)iu);
        }
        __syncthreads();
        // flush: one global atomic per nonzero (position, column) of the window
        const int64_t L = A.ref_len;
        for (int t = threadIdx.x; t < wlen; t += kCountThreads) {
            const int64_t p = wbase + t;
            if (p >= L) break;
#pragma unroll
            for (int pl = 0; pl < 3; ++pl) {
                const uint32_t v = win[pl * kWinMax + t];
                const uint32_t lo = v & 0xFFFFu, hi = v >> 16;
                if (lo) atomicAdd(&A.hist[(int64_t)(2 * pl) * L + p], (int32_t)lo);
                if (hi) atomicAdd(&A.hist[(int64_t)(2 * pl + 1) * L + p], (int32_t)hi);
            }
        }
    } else {
        // sparse / unsorted chunk: global atomics straight into the histogram
        const int64_t L = A.ref_len;
        for (int64_t i = r0 + wave; i < r1; i += kWaves) {
            const int64_t iu = uni64(i);
            bool bad = walk_read<QUAL>(A, iu, lane, [&](unsigned col, int64_t rp) {
                atomicAdd(&A.hist[(int64_t)col * L + rp], 1);
            });
            if (__any(bad) && lane == 0) atomicMin(A.err, (unsigned long long)iu);
        }
    }
}

// max reference span over the batch (one thread per read)
__global__ void k_span(const uint32_t* cig_beg, const uint32_t* cig_n, const uint32_t* cigar, int64_t n,
                       int* out) {
    int best = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t* cg = cigar + cig_beg[i];
        uint32_t span = 0;
        for (uint32_t k = 0, cn = cig_n[i]; k < cn; ++k) {
            const uint32_t op = cg[k] & 15u;
            if (op == 0 || op == 2 || op == 3 || op == 7 || op == 8) span += cg[k] >> 4;
        }
        best = span > (uint32_t)best ? (int)span : best;
    }
    for (int o = 32; o > 0; o >>= 1) {
        int v = __shfl_down(best, o);
        best = v > best ? v : best;
    }
    if ((threadIdx.x & 63) == 0) atomicMax(out, best);
}

// BAM-packed sequence -> BC_SEQ_EVENT (in place allowed: every thread reads its 16 bytes before
// writing them).  Bytes in [nbytes, out_bytes) become zero padding.
__device__ __forceinline__ uint32_t event_byte(uint32_t b) {
    const uint32_t hi = (uint32_t)(kNibClass >> ((b >> 4) * 4)) & 15u;  // base 2m (BAM high nibble)
    const uint32_t lo = (uint32_t)(kNibClass >> ((b & 15u) * 4)) & 15u; // base 2m+1
    return hi | (lo << 4);
}

__global__ void k_seq_event(const uint8_t* src, int64_t nbytes, uint8_t* dst, int64_t out_bytes) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x * 16;
    for (int64_t o = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 16; o < out_bytes; o += stride) {
        uint32_t w[4];
        if (o + 16 <= nbytes && ((uintptr_t)(src + o) & 15u) == 0) {
            const uint4 v = *(const uint4*)(src + o);
            w[0] = v.x, w[1] = v.y, w[2] = v.z, w[3] = v.w;
        } else {
            for (int i = 0; i < 4; ++i) {
                w[i] = 0;
                for (int b = 0; b < 4; ++b) {
                    const int64_t at = o + 4 * i + b;
                    if (at < nbytes) w[i] |= (uint32_t)src[at] << (8 * b);
                }
            }
        }
        uint32_t r[4];
        for (int i = 0; i < 4; ++i) {
            r[i] = 0;
            for (int b = 0; b < 4; ++b) {
                const int64_t at = o + 4 * i + b;
                if (at < nbytes) r[i] |= event_byte((w[i] >> (8 * b)) & 0xFFu) << (8 * b);
            }
        }
        if (o + 16 <= out_bytes && ((uintptr_t)(dst + o) & 15u) == 0) {
            *(uint4*)(dst + o) = make_uint4(r[0], r[1], r[2], r[3]);
        } else {
            for (int i = 0; i < 4; ++i)
                for (int b = 0; b < 4; ++b)
                    if (o + 4 * i + b < out_bytes) dst[o + 4 * i + b] = (uint8_t)(r[i] >> (8 * b));
        }
    }
}

// ------------------------------------------------------------------------------ kernel 2
// Same operation order as CPython evaluating main.py:37-53 (IEEE double, no contraction:
// the file is compiled with -ffp-contract=off):
//   probabilities = count / coverage; percentages = 100 * probability;
//   entropy = nf * sum([-(x*log2(x)) if x != 0 else 0 ...])  (left to right from int 0)
//
// counts_out != NULL: `hist` is the library's accumulation scratch (k_rc adds into it): its
// counts are copied to counts_out and the scratch is left zeroed for the next launch, which
// saves the per-step memset.
//
// One block per 64-position tile, K waves: wave j loads column j of the tile and computes that
// column's percentage and entropy terms (one division and one log2 per term instead of a chain
// of K per thread); wave 0 then adds the terms in column order.  The sums are the same
// left-to-right sequences as main.py:40-53, so the results are unchanged by the split.
template <int K>
__global__ __launch_bounds__(64 * K) void k_stats(int32_t* __restrict__ hist, int64_t L, double nf, double nf2,
                                                   int32_t* __restrict__ counts_out, int32_t* __restrict__ cov_out,
                                                   double* __restrict__ pc, double* __restrict__ ent,
                                                   double* __restrict__ sec) {
    __shared__ int32_t cnt[K][64];
    __shared__ double t1[K][64], t2[K][64];
    // glibc log2's table copied to LDS with the first loads, so that each term's table lookup
    // is an LDS read instead of a dependent global round trip (kernel 2 is one tile deep: its
    // time is its chain of round trips)
    __shared__ __attribute__((aligned(16))) double tab[64][4];
    const int j = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t n_tiles = (L + 63) / 64;
    if (threadIdx.x < 128)
        *(double2*)&tab[threadIdx.x >> 1][2 * (threadIdx.x & 1)] =
            *(const double2*)&log2d::kTab[threadIdx.x >> 1][2 * (threadIdx.x & 1)];
    for (int64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
        const int64_t p = tile * 64 + lane;
        const bool in = p < L;
        int32_t cj = 0;
        if (in) {
            cj = hist[(int64_t)j * L + p];
            if (counts_out) {
                counts_out[(int64_t)j * L + p] = cj;
                hist[(int64_t)j * L + p] = 0;
            }
        }
        cnt[j][lane] = cj;
        __syncthreads();
        int64_t cov = 0;
        int am = 0;
        int32_t c[K];
#pragma unroll
        for (int i = 0; i < K; ++i) {
            c[i] = cnt[i][lane];
            cov += c[i];
        }
#pragma unroll
        for (int i = 1; i < K; ++i)
            if (c[i] > c[am]) am = i;  // np.argmax: first maximum
        double e1 = 0.0, e2 = 0.0;
        if (in && cov != 0) {
            const double pj = (double)cj / (double)cov;
            if (pc) pc[(int64_t)j * L + p] = 100.0 * pj;
            if (cj != 0) e1 = -(pj * glibc_log2_t(pj, tab));
            const int64_t cov2 = cov - c[am];
            if (sec && j != am && cj != 0 && cov2 != 0) {
                const double q = (double)cj / (double)cov2;
                e2 = -(q * glibc_log2_t(q, tab));
            }
        } else if (in && pc) {
            pc[(int64_t)j * L + p] = -1.0;
        }
        t1[j][lane] = e1;
        t2[j][lane] = e2;
        __syncthreads();
        if (j == 0 && in) {
            if (cov_out) cov_out[p] = (int32_t)cov;
            double h = 1.0, h2 = 1.0;
            if (cov != 0) {
                double s = 0.0;
#pragma unroll
                for (int i = 0; i < K; ++i)
                    if (c[i] != 0) s = s + t1[i][lane];
                h = nf * s;
                if (cov - c[am] != 0) {
                    double s2 = 0.0;
#pragma unroll
                    for (int i = 0; i < K; ++i)
                        if (i != am && c[i] != 0) s2 = s2 + t2[i][lane];
                    h2 = nf2 * s2;
                }
            }
            if (ent) ent[p] = h;
            if (sec) sec[p] = h2;
        }
        __syncthreads();  // cnt / t1 / t2 reused by the next tile
    }
}

// Kernel 2 with one lane per position (all K columns in the lane, the terms independent so they
// overlap) and no block barrier but the table copy's: a launch of ~L / 256 blocks whose chain is
// the counts' load (issued before the table copy, so both are in flight together), the fp64
// terms and the stores.  The arithmetic is bc_stats.h's position_stats (the fused kernels'), so the
// results are those of k_stats bit for bit; NULL cov / pc / ent / sec are skipped as in k_stats.
// LEAVES (the fused --summarise-with-bed tail, launch_stats_leaves): the block's 256 positions
// are two of numpy's 128-position pairwise leaves when they lie in a whole 8192-position buffer,
// and the block also writes each leaf's entropy sum (eight strided accumulators, added in
// numpy's order), its exact coverage sum and its non-zero count, so no summary pass re-reads
// the entropies (k_tail adds the leaves up the buffer's tree).  The last, partial buffer's blocks
// are its 64 nodes of numpy's tree one level above the leaves (pw_node: each <= 256 positions,
// contiguous, together all of [full, L)), one block per node: the block's positions are the
// node's, and it writes the node's sum -- its leaf, or its two leaves added -- so k_tail adds the
// partial buffer up the same way as a whole one, from 64 values.
constexpr int kLv = 7;  // 8192 -> 4096 -> ... -> 128: six splits; one spare level
__device__ __forceinline__ void pw_node(int m, int level, int idx, int& off, int& len) {
    // node idx of the given level (level 0: the root) of numpy's recursion over m elements
    // (branch-free: an unsplit node is its own left child, n2 = len, and an empty right one)
    off = 0;
    len = m;
    for (int l = 0; l < level; ++l) {
        const int bit = (idx >> (level - 1 - l)) & 1;
        const int n2 = len > 128 ? (len >> 1) & ~7 : len;  // numpy: n/2 less its remainder mod 8
        off += bit ? n2 : 0;
        len = bit ? len - n2 : n2;
    }
}
struct Leaves {
    double* ent;  // [full buffers * 64]
    long long* cov;
    long long* nz;
    int64_t full;  // positions in whole 8192-position buffers
};
template <int K, bool LEAVES = false>
__global__ __launch_bounds__(256) void k_stats_lane(int32_t* __restrict__ hist, int64_t L, double nf, double nf2,
                                                    int32_t* __restrict__ counts_out, int32_t* __restrict__ cov_out,
                                                    double* __restrict__ pc, double* __restrict__ ent,
                                                    double* __restrict__ sec, Leaves lv = Leaves{}) {
    __shared__ __attribute__((aligned(16))) double tab[64][4];
    int64_t P = (int64_t)blockIdx.x * 256 + threadIdx.x;
    bool in = P < L;
    int node = -1, n6 = 0;  // LEAVES: a block of the partial buffer: its node and the node's length
    if (LEAVES && (int64_t)blockIdx.x >= lv.full / 256) {  // (uniform)
        node = (int)(blockIdx.x - lv.full / 256);
        int o6;
        pw_node((int)(L - lv.full), kLv - 1, node, o6, n6);
        P = lv.full + o6 + threadIdx.x;
        in = (int)threadIdx.x < n6;
    }
    uint32_t c[K];
#pragma unroll
    for (int j = 0; j < K; ++j) c[j] = in ? (uint32_t)hist[(int64_t)j * L + P] : 0u;
    if (threadIdx.x < 128)
        *(double2*)&tab[threadIdx.x >> 1][2 * (threadIdx.x & 1)] =
            *(const double2*)&log2d::kTab[threadIdx.x >> 1][2 * (threadIdx.x & 1)];
    __syncthreads();
    if (!in && !LEAVES) return;
    if (counts_out && in) {
#pragma unroll
        for (int j = 0; j < K; ++j) {
            counts_out[(int64_t)j * L + P] = (int32_t)c[j];
            hist[(int64_t)j * L + P] = 0;
        }
    }
    int64_t cov = 0;
    int am = 0;
    uint32_t mx = c[0];
#pragma unroll
    for (int j = 0; j < K; ++j) {
        cov += c[j];
        if (c[j] > mx) mx = c[j], am = j;  // np.argmax: first maximum
    }
    if (cov_out && in) cov_out[P] = (int32_t)cov;
    double h = 1.0, h2 = 1.0;
    if (cov != 0) {
        double s = 0.0;
#pragma unroll
        for (int j = 0; j < K; ++j) {
            const double pj = (double)c[j] / (double)cov;
            if (pc) pc[(int64_t)j * L + P] = 100.0 * pj;
            if (c[j] != 0) s = s + (-(pj * glibc_log2_t(pj, tab)));
        }
        h = nf * s;
        const int64_t cov2 = cov - (int64_t)mx;
        if (cov2 != 0 && sec) {
            double s2 = 0.0;
#pragma unroll
            for (int j = 0; j < K; ++j)
                if (j != am && c[j] != 0) {
                    const double q = (double)c[j] / (double)cov2;
                    s2 = s2 + (-(q * glibc_log2_t(q, tab)));
                }
            h2 = nf2 * s2;
        }
    } else if (pc && in) {
#pragma unroll
        for (int j = 0; j < K; ++j) pc[(int64_t)j * L + P] = -1.0;
    }
    if (in) {
        if (ent) ent[P] = h;
        if (sec) sec[P] = h2;
    }
    if (LEAVES && node >= 0) {  // (uniform) a node of the partial buffer: its leaf or two
        __shared__ double s_n[256];
        __shared__ long long s_q[8];
        const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
        s_n[t] = h;
        long long cs = cov, nzc = cov != 0;  // (0 past the node)
        for (int o = 32; o > 0; o >>= 1) {
            cs += __shfl_down(cs, o);
            nzc += __shfl_down(nzc, o);
        }
        if (lane == 0) s_q[wave] = cs, s_q[4 + wave] = nzc;
        __syncthreads();
        if (t < 16) {  // leaf t >> 3 (left, right), accumulator j = t & 7, numpy's pairwise_sum
            const int n2 = n6 > 128 ? (n6 >> 1) & ~7 : n6, j = t & 7;
            const int lo = (t >> 3) ? n2 : 0, len = (t >> 3) ? n6 - n2 : n2, full = len & ~7;
            const double* a = s_n + lo;
            double r = a[j < full ? j : 0];
#pragma unroll
            for (int i = 1; i < 16; ++i) r = r + (j + 8 * i < full ? a[j + 8 * i] : -0.0);  // (-0.0: adds nothing)
            r = r + __shfl_down(r, 1);
            r = r + __shfl_down(r, 2);
            r = r + __shfl_down(r, 4);
            if (len < 8) r = 0.0;  // numpy: n < 8 sums from 0, in order
#pragma unroll
            for (int u = 0; u < 7; ++u) r = r + (full + u < len ? a[full + u] : -0.0);
            const double right = __shfl_down(r, 8);
            if (t == 0) {
                const int64_t f = lv.full / kNpBuf * 64 + node;
                lv.ent[f] = n6 > 128 ? r + right : r;
                lv.cov[f] = s_q[0] + s_q[1] + s_q[2] + s_q[3];
                lv.nz[f] = s_q[4] + s_q[5] + s_q[6] + s_q[7];
            }
        }
    } else if (LEAVES && (int64_t)blockIdx.x * 256 + 256 <= lv.full) {  // (uniform) two whole leaves
        __shared__ double s_h[256];
        __shared__ long long s_r[8];
        const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
        s_h[t] = h;
        long long cs = cov, nzc = cov != 0;
        for (int o = 32; o > 0; o >>= 1) {
            cs += __shfl_down(cs, o);
            nzc += __shfl_down(nzc, o);
        }
        if (lane == 0) s_r[wave] = cs, s_r[4 + wave] = nzc;
        __syncthreads();
        if (t < 16) {  // leaf t >> 3, accumulator j = t & 7: r_j = a[j] + a[j + 8] + ... in order
            const double* a = s_h + 128 * (t >> 3) + (t & 7);
            double r = a[0];
#pragma unroll
            for (int i = 1; i < 16; ++i) r += a[8 * i];
            r = r + __shfl_down(r, 1);  // (r0+r1), (r2+r3), ...
            r = r + __shfl_down(r, 2);  // (r0+r1)+(r2+r3), (r4+r5)+(r6+r7)
            r = r + __shfl_down(r, 4);  // the leaf
            if ((t & 7) == 0) {
                const int64_t f = (int64_t)blockIdx.x * 2 + (t >> 3);
                lv.ent[f] = r;
                lv.cov[f] = s_r[2 * (t >> 3)] + s_r[2 * (t >> 3) + 1];
                lv.nz[f] = s_r[4 + 2 * (t >> 3)] + s_r[4 + 2 * (t >> 3) + 1];
            }
        }
    }
}

// Kernel 2 with eight lanes per position: lane j < K computes column j's percentage and its two
// entropy terms (one division and log2 each: dependent fp64 chains K times shorter than
// k_stats_lane's, over 8x the lanes), then the position's first lane adds the terms in column
// order, as position_stats does.  Every lane holds all K counts (K in-group shuffles), so cov,
// the maximum and np.argmax come from the same code as in position_stats; the results are those
// of k_stats / k_stats_lane bit for bit.  NULL cov / pc / ent / sec are skipped as there.
template <int K>
__global__ __launch_bounds__(256) void k_stats_oct(int32_t* __restrict__ hist, int64_t L, double nf, double nf2,
                                                   int32_t* __restrict__ counts_out, int32_t* __restrict__ cov_out,
                                                   double* __restrict__ pc, double* __restrict__ ent,
                                                   double* __restrict__ sec) {
    __shared__ __attribute__((aligned(16))) double tab[64][4];
    const int j = threadIdx.x & 7;
    const int64_t P = (int64_t)blockIdx.x * 32 + (threadIdx.x >> 3);
    const bool in = P < L, col = in && j < K;
    const uint32_t cj = col ? (uint32_t)hist[(int64_t)j * L + P] : 0u;
    if (threadIdx.x < 128)
        *(double2*)&tab[threadIdx.x >> 1][2 * (threadIdx.x & 1)] =
            *(const double2*)&log2d::kTab[threadIdx.x >> 1][2 * (threadIdx.x & 1)];
    __syncthreads();
    if (col && counts_out) {
        counts_out[(int64_t)j * L + P] = (int32_t)cj;
        hist[(int64_t)j * L + P] = 0;
    }
    uint32_t c[K];
#pragma unroll
    for (int i = 0; i < K; ++i) c[i] = (uint32_t)__shfl((int)cj, i, 8);
    int64_t cov = 0;
    int am = 0;
    uint32_t mx = c[0];
#pragma unroll
    for (int i = 0; i < K; ++i) {
        cov += c[i];
        if (c[i] > mx) mx = c[i], am = i;  // np.argmax: first maximum
    }
    const bool one = cov != 0 && cov == (int64_t)mx;  // one class only: the terms are exact constants
    const int64_t cov2 = cov - (int64_t)mx;
    double t = 0.0, u = 0.0;
    if (col && cov != 0) {
        if (one) {
            if (pc) pc[(int64_t)j * L + P] = j == am ? 100.0 : 0.0;
        } else {
            const double pj = (double)cj / (double)cov;
            if (pc) pc[(int64_t)j * L + P] = 100.0 * pj;
            if (cj != 0) t = -(pj * glibc_log2_t(pj, tab));
            if (sec && cov2 != 0 && j != am && cj != 0) {
                const double q = (double)cj / (double)cov2;
                u = -(q * glibc_log2_t(q, tab));
            }
        }
    } else if (col && pc) {
        pc[(int64_t)j * L + P] = -1.0;
    }
    double ts[K], us[K];
#pragma unroll
    for (int i = 0; i < K; ++i) {
        ts[i] = __shfl(t, i, 8);
        us[i] = __shfl(u, i, 8);
    }
    if (!in || j != 0) return;
    if (cov_out) cov_out[P] = (int32_t)cov;
    double h = 1.0, h2 = 1.0;
    if (one) {
        h = 0.0;
    } else if (cov != 0) {
        double s1 = 0.0;
#pragma unroll
        for (int i = 0; i < K; ++i)
            if (c[i] != 0) s1 = s1 + ts[i];
        h = nf * s1;
        if (cov2 != 0) {
            double s2 = 0.0;
#pragma unroll
            for (int i = 0; i < K; ++i)
                if (i != am && c[i] != 0) s2 = s2 + us[i];
            h2 = nf2 * s2;
        }
    }
    if (ent) ent[P] = h;
    if (sec) sec[P] = h2;
}

// ------------------------------------------------------------------------------ numpy sums
// numpy float64 add.reduce (numpy 2.2, verified against np.add.reduce / np.mean in
// test_summary_matches_numpy in tests/test_gpu_parity.py): the input is consumed in 8192-element buffers, s = 0; s += pw(buffer),
// where pw is numpy's pairwise_sum: n < 8 -> sequential from 0.0; n <= 128 -> eight strided
// accumulators combined ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) then the tail sequentially;
// else split at n2 = n/2 - (n/2)%8 and add the halves.

__device__ double pw_leaf(const double* a, int n) {
    if (n < 8) {
        double r = 0.0;
        for (int i = 0; i < n; ++i) r += a[i];
        return r;
    }
    double r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = a[j];
    int i = 8;
    for (; i < n - (n % 8); i += 8) {
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] += a[i + j];
    }
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += a[i];
    return res;
}

// Generic pairwise sum of a[0..m), m <= 8192, by one workgroup (any blockDim >= 128).  numpy's
// recursion (split at n2 = n/2 - (n/2)%8 down to leaves of <= 128) is laid out level by level in
// LDS, in parallel: node i of level l has children 2i, 2i+1 of level l+1; a leaf passes itself
// down as its left child (and an empty right one), so level kLv holds every leaf in order.  The
// leaves are summed in parallel, then every level adds its children bottom-up: the same sums in
// the same order as the recursion, with no per-thread stack (a private array there lives in
// scratch memory, one slow round trip per push).  Returns the value in thread 0 only.
__device__ double pw_block(const double* a, int m, int* s_off, int* s_len, double* s_val) {
    // s_off / s_len: (2^(kLv+1) - 1) nodes; s_val: 2 x 2^kLv values (ping-pong)
    const int t = threadIdx.x;
    if (t == 0) {
        s_off[0] = 0;
        s_len[0] = m;
    }
    __syncthreads();
    for (int l = 0; l < kLv; ++l) {  // top-down: split the nodes of level l
        const int base = (1 << l) - 1, nb = (1 << (l + 1)) - 1;
        for (int i = t; i < (1 << l); i += blockDim.x) {
            const int o = s_off[base + i], n = s_len[base + i];
            int n2 = n;
            if (n > 128) {
                n2 = n / 2;
                n2 -= n2 % 8;
            }
            s_off[nb + 2 * i] = o;
            s_len[nb + 2 * i] = n2;
            s_off[nb + 2 * i + 1] = o + n2;
            s_len[nb + 2 * i + 1] = n - n2;
        }
        __syncthreads();
    }
    const int leaves = 1 << kLv, lbase = leaves - 1;
    double* cur = s_val;
    double* nxt = s_val + leaves;
    for (int i = t; i < leaves; i += blockDim.x) {
        const int n = s_len[lbase + i];
        cur[i] = n > 0 ? pw_leaf(a + s_off[lbase + i], n) : 0.0;
    }
    __syncthreads();
    for (int l = kLv - 1; l >= 0; --l) {  // bottom-up: a split node adds its children, left + right
        const int base = (1 << l) - 1;
        for (int i = t; i < (1 << l); i += blockDim.x)
            nxt[i] = s_len[base + i] > 128 ? cur[2 * i] + cur[2 * i + 1] : cur[2 * i];
        __syncthreads();
        double* tmp = cur;
        cur = nxt;
        nxt = tmp;
    }
    const double r = t == 0 ? cur[0] : 0.0;
    __syncthreads();
    return r;
}

// The same sum, pw_block's tree, without its 14 barriers and one-thread leaves: every leaf slot
// (LV levels of numpy's split: a leaf passes itself down as the left child, an empty right one)
// is found by descending its bit path, its eight strided accumulators are eight threads'
// (every load issued together, unguarded: clamped, and the extra ones selected to -0.0, which
// adds exactly nothing to any double), combined by shuffles in numpy's order; then one wave adds
// the slots up the tree: node i of level d sits in lane i << (LV - 1 - d), its right child
// 2^(LV-2-d) lanes up (a shuffle down), and each lane's descent recorded which of its ancestors
// split.  LV = kLv covers m <= 8192; LV = 4 covers m <= 512 (checked against numpy for every
// such m) with 128 tasks, two waves, instead of 1024.  a: m doubles (LDS or global); s_leaf:
// 2^LV doubles of LDS; NT threads, all calling.  Returns the value in thread 0 only.
template <int NT, int LV = kLv>
__device__ __forceinline__ double pw_fast(const double* a, int m, double* s_leaf) {
    constexpr int kSlots = 1 << LV, kTasks = 8 * kSlots, R = kTasks >= NT ? kTasks / NT : 1;
    static_assert(kTasks % 64 == 0 && (kTasks < NT || R * NT == kTasks), "tasks: whole waves");
    const int t = threadIdx.x, j = t & 7;  // (NT is a multiple of 8: every task of a thread has accumulator j)
    if (kTasks >= NT || t < kTasks) {  // (wave-uniform)
        int len[R], full[R];
        double v[R][16], rem[R][7];
#pragma unroll
        for (int q = 0; q < R; ++q) {  // every task's loads issued first
            int off;
            pw_node(m, LV, (t + NT * q) >> 3, off, len[q]);
            full[q] = len[q] & ~7;
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                const int i = j + 8 * u;
                v[q][u] = a[off + (i < full[q] ? i : 0)];
            }
#pragma unroll
            for (int u = 0; u < 7; ++u) {  // the leaf's last len % 8 (or, below 8, all) elements
                const int i = full[q] + u;
                rem[q][u] = a[off + (i < len[q] ? i : 0)];
            }
        }
#pragma unroll
        for (int q = 0; q < R; ++q) {
            double x = v[q][0];
#pragma unroll
            for (int u = 1; u < 16; ++u) x = x + (j + 8 * u < full[q] ? v[q][u] : -0.0);
            x = x + __shfl_down(x, 1);  // (r0+r1), (r2+r3), ...
            x = x + __shfl_down(x, 2);
            x = x + __shfl_down(x, 4);  // ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7))
            if (len[q] < 8) x = 0.0;    // numpy: n < 8 sums from 0, in order
#pragma unroll
            for (int u = 0; u < 7; ++u) x = x + (full[q] + u < len[q] ? rem[q][u] : -0.0);
            if (((t + NT * q) & 7) == 0) s_leaf[(t + NT * q) >> 3] = x;
        }
    }
    __syncthreads();
    double res = 0.0;
    if (t < 64) {
        // lane tt's descent to node tt of level LV - 1, recording which ancestors split
        const int tt = t < (1 << (LV - 1)) ? t : 0;
        int n = m;
        unsigned split = 0;
#pragma unroll
        for (int l = 0; l < LV - 1; ++l) {
            split |= (unsigned)(n > 128) << l;
            const int n2 = n > 128 ? (n >> 1) & ~7 : n;
            n = ((tt >> (LV - 2 - l)) & 1) ? n - n2 : n2;
        }
        const double v0 = s_leaf[2 * tt], v1 = s_leaf[2 * tt + 1];
        double val = n > 128 ? v0 + v1 : v0;
#pragma unroll
        for (int d = LV - 2; d >= 0; --d) {
            const double c1 = __shfl_down(val, 1 << (LV - 2 - d));
            val = ((split >> d) & 1) ? val + c1 : val;
        }
        res = val;
    }
    __syncthreads();  // s_leaf reusable
    return res;
}

// Full 8192-element buffer with the fixed tree: 64 leaves of 128; 256 threads, thread t owns
// accumulators {2(t&3), 2(t&3)+1} of leaf t>>2.  Value valid in thread 0.
template <class F>
__device__ double pw_full8192(F&& val, double* s_wave) {
    const int t = threadIdx.x;
    const int leaf = t >> 2, s = t & 3;
    const int base = leaf * 128 + 2 * s;
    double ra = val(base), rb = val(base + 1);
#pragma unroll
    for (int i = 1; i < 16; ++i) {
        ra += val(base + 8 * i);
        rb += val(base + 8 * i + 1);
    }
    double v = ra + rb;              // (r0+r1), (r2+r3), (r4+r5), (r6+r7)
    v = v + __shfl_down(v, 1);       // lanes s=0: (r0+r1)+(r2+r3); s=2: (r4+r5)+(r6+r7)
    v = v + __shfl_down(v, 2);       // s=0: leaf value
    v = v + __shfl_down(v, 4);       // pairs of leaves
    v = v + __shfl_down(v, 8);
    v = v + __shfl_down(v, 16);
    v = v + __shfl_down(v, 32);      // lane 0: 16 leaves = pw(2048)
    if ((t & 63) == 0) s_wave[t >> 6] = v;
    __syncthreads();
    double r = 0.0;
    if (t == 0) r = (s_wave[0] + s_wave[1]) + (s_wave[2] + s_wave[3]);
    __syncthreads();
    return r;
}

__device__ __forceinline__ long long block_sum_i64(long long v, long long* s_red) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o);
    if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = v;
    __syncthreads();
    long long r = 0;
    if (threadIdx.x == 0)
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) r += s_red[w];
    __syncthreads();
    return r;
}

// The last, partial buffer of a reference (m < 8192 elements): numpy's generic pairwise tree
// (pw_block) over the entropies staged in LDS (dynamic, m doubles), so the leaves are summed from
// LDS instead of one dependent global load after another; every global load of the buffer is
// issued at once.
__device__ __forceinline__ void sum_tail_block(const int32_t* cov, const double* ent, int64_t L, double* part_ent,
                                               long long* part_cov, long long* part_nz, int64_t chunk) {
    extern __shared__ __attribute__((aligned(16))) unsigned char dyn[];
    double* s_ent = (double*)dyn;  // [m]
    __shared__ long long s_red[8];
    __shared__ int s_off[(2 << kLv) - 1], s_len[(2 << kLv) - 1];
    __shared__ double s_val[2 << kLv];
    const int64_t c0 = chunk * kNpBuf;
    const int m = (int)(L - c0);  // 0 < m < 8192
    const int t = threadIdx.x;
    int cv[32];
    double ev[32];
#pragma unroll
    for (int j = 0; j < 32; ++j) {
        const int i = t + 256 * j;
        cv[j] = i < m ? cov[c0 + i] : 0;
        ev[j] = i < m ? ent[c0 + i] : 0.0;
    }
    long long cs = 0, nz = 0;
#pragma unroll
    for (int j = 0; j < 32; ++j) {
        cs += cv[j];
        nz += cv[j] != 0;
        const int i = t + 256 * j;
        if (i < m) s_ent[i] = ev[j];
    }
    __syncthreads();
    const double e = pw_block(s_ent, m, s_off, s_len, s_val);
    for (int o = 32; o > 0; o >>= 1) {
        cs += __shfl_down(cs, o);
        nz += __shfl_down(nz, o);
    }
    if ((t & 63) == 0) {
        s_red[t >> 6] = cs;
        s_red[4 + (t >> 6)] = nz;
    }
    __syncthreads();
    if (t == 0) {
        part_ent[chunk] = e;
        part_cov[chunk] = (s_red[0] + s_red[1]) + (s_red[2] + s_red[3]);
        part_nz[chunk] = (s_red[4] + s_red[5]) + (s_red[6] + s_red[7]);
    }
}

__global__ __launch_bounds__(256) void k_sum_tail(const int32_t* cov, const double* ent, int64_t L,
                                                  double* part_ent, long long* part_cov, long long* part_nz,
                                                  int64_t chunk, int32_t* hdr, int32_t hval) {
    if (threadIdx.x == 0 && hdr) *hdr = hval;
    sum_tail_block(cov, ent, L, part_ent, part_cov, part_nz, chunk);
}

// one workgroup (256 threads) per 8192 buffer: entropy pairwise sum, exact coverage sum, nnz.
// A full buffer issues all its loads up front (8 x 16 B of coverage and 16 x 16 B of entropy per
// thread) before any reduction, so a workgroup has its whole 96 KiB in flight at once; the
// coverage sum and the non-zero count share one block reduction.
// (hdr: block 0 also writes the work header, the fold's count of quarter buffers: no memset launch;
// STAGE_TAIL: the last block is the reference's partial buffer, summed as k_sum_tail does, in
// the same launch — the dynamic LDS then holds its entropies)
template <bool STAGE_TAIL>
__global__ __launch_bounds__(256) void k_sum_chunks(const int32_t* cov, const double* ent, int64_t L,
                                                    double* part_ent, long long* part_cov, long long* part_nz,
                                                    int64_t first_chunk, int32_t* hdr, int32_t hval) {
    if (blockIdx.x == 0 && threadIdx.x == 0 && hdr) *hdr = hval;
    if (STAGE_TAIL && blockIdx.x == gridDim.x - 1) {  // (uniform)
        sum_tail_block(cov, ent, L, part_ent, part_cov, part_nz, first_chunk + blockIdx.x);
        return;
    }
    __shared__ double s_wave[4];
    __shared__ long long s_red[8];
    __shared__ int s_off[(2 << kLv) - 1], s_len[(2 << kLv) - 1];
    __shared__ double s_val[2 << kLv];
    const int64_t chunk = first_chunk + blockIdx.x;
    const int64_t c0 = chunk * kNpBuf;
    const int m = (int)((L - c0) < kNpBuf ? (L - c0) : kNpBuf);
    const int t = threadIdx.x;
    long long cs = 0, nz = 0;
    double e;
    if (m == kNpBuf && ((uintptr_t)(cov + c0) & 15u) == 0) {
        int4 cv[8];
        const int4* c4 = (const int4*)(cov + c0);
#pragma unroll
        for (int j = 0; j < 8; ++j) cv[j] = c4[t + 256 * j];
        e = pw_full8192([&](int i) { return ent[c0 + i]; }, s_wave);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            cs += (long long)cv[j].x + cv[j].y + cv[j].z + cv[j].w;
            nz += (cv[j].x != 0) + (cv[j].y != 0) + (cv[j].z != 0) + (cv[j].w != 0);
        }
    } else {
        for (int i = t; i < m; i += blockDim.x) {
            const long long v = cov[c0 + i];
            cs += v;
            nz += v != 0;
        }
        e = (m == kNpBuf) ? pw_full8192([&](int i) { return ent[c0 + i]; }, s_wave)
                          : pw_block(ent + c0, m, s_off, s_len, s_val);
    }
    for (int o = 32; o > 0; o >>= 1) {
        cs += __shfl_down(cs, o);
        nz += __shfl_down(nz, o);
    }
    if ((t & 63) == 0) {
        s_red[t >> 6] = cs;
        s_red[4 + (t >> 6)] = nz;
    }
    __syncthreads();
    if (t == 0) {
        part_ent[chunk] = e;
        part_cov[chunk] = (s_red[0] + s_red[1]) + (s_red[2] + s_red[3]);
        part_nz[chunk] = (s_red[4] + s_red[5]) + (s_red[6] + s_red[7]);
    }
}

// The float64 fold over the per-buffer partials stays sequential (numpy adds the buffers'
// pairwise sums in order), but it need not take one dependent add per buffer.  Buffer sums are
// >= 0, and most are integers (8192 positions whose entropies are 0.0 / 1.0: every buffer no two
// reads share a position of; exactly 8192.0 without reads).  Adding integers to s rounds only
// where s crosses into a binade whose ulp exceeds the granularity of its fraction, and then the
// final sum of the run is not representable either: so a run of integer buffers adds as ONE add
// of its exact integer total whenever that add is exact (TwoSum error 0), and only fractional
// buffers (and the rare run that crosses such a binade) take sequential adds.  One workgroup per
// reference, so the folds of several references (bc_summary_fold) run side by side.  The
// partials are double-buffered through LDS, 1024 per round: the block loads round r+1 into
// registers while round r is scanned (the integer buffers' exact prefix sums and the list of the
// fractional ones) and folded by thread 0 from LDS.  The integer sums reduce in parallel.
struct FoldRef {
    const double* pe;
    const long long* pc;
    const long long* pn;
    const double* qe;  // quarter partials of the buffers [0, *nquart)
    const long long* qc;
    const long long* qn;
    const int32_t* nquart;  // the work buffer's header (set by whoever produced the partials)
    int64_t nchunks;
    int64_t L;
    double* out;
};
constexpr int kFoldMax = 24;  // references per launch (kernel arguments by value)
struct FoldArgs {
    FoldRef ref[kFoldMax];
};

constexpr int kFoldThreads = 1024;
__global__ __launch_bounds__(kFoldThreads) void k_sum_final(FoldArgs FA) {
    constexpr int kR = 4 * kFoldThreads;  // buffers per round, 4 per thread
    constexpr int kW = kFoldThreads / 64;
    __shared__ double s_buf[kR];
    // The walk (rounds with at most kE fractional buffers): per fractional buffer, in order, its
    // index, the exclusive prefix of the round's integer buffer sums (<= 8192 each) before it, its
    // value, and the running sum s before its run (the optimistic chain's record)
    constexpr int kE = kR / 4;
    constexpr int kB = 8;  // events per batch of the chain
    __shared__ uint16_t s_fr[kE];
    __shared__ int s_fpre[kE + 1 + kB];   // (past the last event: the round's total, repeated)
    __shared__ double s_fv[kE + 1 + kB];  // (past the last fractional buffer: 0.0)
    __shared__ double s_rd[kE + 1 + kB];  // each event's integer run total, as a double (exact)
    __shared__ int s_total;  // the round's integer buffer sum
    __shared__ int s_wsum[kW], s_wfr[kW];
    __shared__ long long s_red[2 * kW];
    const FoldRef& R = FA.ref[blockIdx.x];
    const double* part_ent = R.pe;
    const long long* part_cov = R.pc;
    const long long* part_nz = R.pn;
    const int64_t nchunks = R.nchunks;
    const int64_t nq = *R.nquart;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    double s = 0.0;
    long long cs = 0, nz = 0;
    double v[4];
    long long vc[4], vn[4];
    auto load = [&](int64_t r0) {  // issue only: the values are consumed a round later
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int64_t c = r0 + t + kFoldThreads * j;
            if (c < nq) {  // a buffer's 4 quarters: (q0 + q1) + (q2 + q3), numpy's tree
                const double* q = R.qe + 4 * c;
                v[j] = (q[0] + q[1]) + (q[2] + q[3]);
                vc[j] = (R.qc[4 * c] + R.qc[4 * c + 1]) + (R.qc[4 * c + 2] + R.qc[4 * c + 3]);
                vn[j] = (R.qn[4 * c] + R.qn[4 * c + 1]) + (R.qn[4 * c + 2] + R.qn[4 * c + 3]);
            } else {
                const bool in = c < nchunks;
                v[j] = in ? part_ent[c] : 0.0;
                vc[j] = in ? part_cov[c] : 0;
                vn[j] = in ? part_nz[c] : 0;
            }
        }
    };
    auto stash = [&]() {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            s_buf[t + kFoldThreads * j] = v[j];
            cs += vc[j];
            nz += vn[j];
        }
    };
    // the round's scan: thread t takes buffers 4t .. 4t+3 (in order); integer sums as int (a
    // round's total <= 4096 * 8192), fractional buffers listed in order
    auto scan = [&](int m) {
        int isum = 0, nfr = 0, iv[4];
        bool fr[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int e = 4 * t + j;
            const double x = e < m ? s_buf[e] : 0.0;
            fr[j] = e < m && x != __builtin_floor(x);
            iv[j] = fr[j] ? 0 : (int)x;
            isum += iv[j];
            nfr += fr[j] ? 1 : 0;
        }
        int ps = isum, pf = nfr;  // inclusive wave scans
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int a = __shfl_up(ps, o), f = __shfl_up(pf, o);
            if (lane >= o) ps += a, pf += f;
        }
        if (lane == 63) s_wsum[wave] = ps, s_wfr[wave] = pf;
        __syncthreads();
        int bs = 0, bf = 0, tf = 0;
        for (int w = 0; w < kW; ++w) {
            if (w < wave) bs += s_wsum[w], bf += s_wfr[w];
            tf += s_wfr[w];
        }
        int xs = bs + ps - isum, xf = bf + pf - nfr;  // exclusive
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int e = 4 * t + j;
            if (fr[j]) {
                if (xf < kE) {
                    s_fr[xf] = (uint16_t)e;
                    s_fpre[xf] = xs;
                    s_fv[xf] = s_buf[e];
                }
                ++xf;
            }
            xs += iv[j];
        }
        if (t == kFoldThreads - 1) s_total = xs;
        __syncthreads();
        return tf;
    };
    load(0);
    stash();
    __syncthreads();
    for (int64_t r0 = 0; r0 < nchunks; r0 += kR) {
        const bool more = r0 + kR < nchunks;
        if (more) load(r0 + kR);  // in flight while this round is scanned and folded
        const int m = (int)((nchunks - r0) < kR ? (nchunks - r0) : kR);
        const int nfr = scan(m);
        const bool walk = nfr <= kE && 4 * nfr <= m;  // (uniform) few fractional buffers: the event walk
        if (!walk) {
            if (t == 0) {  // mostly fractional: plain sequential adds
                const double* b = s_buf;
                int i = 0;
                for (; i + 8 <= m; i += 8) {
                    double w[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u) w[u] = b[i + u];
#pragma unroll
                    for (int u = 0; u < 8; ++u) s += w[u];
                }
                for (; i < m; ++i) s += b[i];
            }
        } else {
            // Each fractional buffer f ends an integer run of exact total R_f (prefix difference;
            // event nfr: the round's last run): s = (s + R_f) + v_f, two adds per event, by thread
            // 0 alone.  The run's add (and every partial sum inside it, all smaller) is exact when
            // s + R_f lies in the binade of s (multiples of ulp(s) <= 1): checked with integer ops
            // on the exponent bits, off the add chain, per batch of kB events (loads of the next
            // batch in flight); a batch with a run leaving its binade (a few per reference) is
            // redone buffer by buffer from the s before it.
            if (t <= kB) {  // the last run and the batch padding: x unchanged past it
                s_fpre[nfr + t] = s_total;
                s_fv[nfr + t] = 0.0;
            }
            __syncthreads();
            for (int f = t; f <= nfr + kB; f += kFoldThreads)
                s_rd[f] = (double)(s_fpre[f] - (f ? s_fpre[f - 1] : 0));
            __syncthreads();
            if (t == 0) {
                auto hi = [](double v) { return (uint32_t)((unsigned long long)__double_as_longlong(v) >> 32); };
                double x = s, rdA[kB], fvA[kB];
#pragma unroll
                for (int u = 0; u < kB; ++u) rdA[u] = s_rd[u], fvA[u] = s_fv[u];
                for (int f0 = 0; f0 <= nfr; f0 += kB) {
                    double rdB[kB], fvB[kB];
                    const int fn = f0 + kB <= nfr ? f0 + kB : f0;  // (the next batch, or a reload)
#pragma unroll
                    for (int u = 0; u < kB; ++u) rdB[u] = s_rd[fn + u], fvB[u] = s_fv[fn + u];
                    const double x0 = x;
                    uint32_t moved = 0;
#pragma unroll
                    for (int u = 0; u < kB; ++u) {
                        const double tt = x + rdA[u];
                        moved |= (hi(x) ^ hi(tt)) & 0xFFF00000u;  // the exponent changed
                        x = tt + fvA[u];  // (past the last event: + 0.0 + 0.0, exact)
                    }
                    // (a batch of integer buffers only, from an integer-valued s: exact below 2^53)
                    if (moved && !(f0 == nfr && x0 == __builtin_floor(x0) && x < 9007199254740992.0)) {
                        // redo the batch's buffers one by one, loaded 8 at a time
                        const int last = f0 + kB - 1 < nfr ? f0 + kB - 1 : nfr;
                        const int i0 = f0 == 0 ? 0 : (int)s_fr[f0 - 1] + 1;
                        const int i1 = last < nfr ? (int)s_fr[last] + 1 : m;
                        x = x0;
                        int i = i0;
                        for (; i + 8 <= i1; i += 8) {
                            double w[8];
#pragma unroll
                            for (int u = 0; u < 8; ++u) w[u] = s_buf[i + u];
#pragma unroll
                            for (int u = 0; u < 8; ++u) x += w[u];
                        }
                        for (; i < i1; ++i) x += s_buf[i];
                    }
#pragma unroll
                    for (int u = 0; u < kB; ++u) rdA[u] = rdB[u], fvA[u] = fvB[u];
                }
                s = x;
            }
        }
        __syncthreads();  // s_buf read by thread 0
        if (more) stash();
        __syncthreads();
    }
    for (int o = 32; o > 0; o >>= 1) {
        cs += __shfl_down(cs, o);
        nz += __shfl_down(nz, o);
    }
    if (lane == 0) {
        s_red[wave] = cs;
        s_red[kW + wave] = nz;
    }
    __syncthreads();
    if (t == 0) {
        cs = 0;
        nz = 0;
        for (int w = 0; w < kW; ++w) cs += s_red[w], nz += s_red[kW + w];
        const double n = (double)R.L;
        R.out[0] = (double)cs / n;  // integer sum is exact in float64 below 2^53: np.mean == sum / n
        R.out[1] = s / n;
        R.out[2] = (double)nz;
        R.out[3] = (double)cs;
    }
}

// ------------------------------------------------------------------------------ amplicons
// k-th smallest (0-based) of n non-negative keys by 8-bit radix select (exact; np.median
// takes the middle element(s) of the sorted values).
template <class KeyF>
__device__ unsigned long long radix_select(KeyF&& key, int64_t n, int64_t k, int bits, unsigned* s_hist,
                                           unsigned long long* s_sel) {
    unsigned long long prefix = 0, mask = 0;
    for (int shift = bits - 8; shift >= 0; shift -= 8) {
        for (int b = threadIdx.x; b < 256; b += blockDim.x) s_hist[b] = 0;
        __syncthreads();
        for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
            const unsigned long long v = key(i);
            if ((v & mask) == prefix) atomicAdd(&s_hist[(v >> shift) & 255u], 1u);
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            int64_t acc = 0;
            int b = 0;
            for (; b < 256; ++b) {
                if (acc + s_hist[b] > k) break;
                acc += s_hist[b];
            }
            s_sel[0] = (unsigned long long)b;
            s_sel[1] = (unsigned long long)(k - acc);
        }
        __syncthreads();
        prefix |= s_sel[0] << shift;
        mask |= 255ull << shift;
        k = (int64_t)s_sel[1];
        __syncthreads();
    }
    return prefix;
}

__device__ double np_mean_block(const double* a, int64_t n, int* s_off, int* s_len, double* s_val) {
    // s = 0; s += pw(buffer) per 8192 buffer; mean = s / n   (value valid in thread 0)
    double s = 0.0;
    for (int64_t c0 = 0; c0 < n; c0 += kNpBuf) {
        const int m = (int)((n - c0) < kNpBuf ? (n - c0) : kNpBuf);
        const double v = pw_block(a + c0, m, s_off, s_len, s_val);
        s += v;
    }
    return s / (double)n;
}

// Ascending bitonic sort of 64 * E unsigned 64-bit keys by ONE wave, E per lane (element
// lane * E + r in register r), no barriers: pairs less than E apart are in one lane's registers,
// the others E * m apart are lanes m apart (one 64-bit shuffle per key).  Fully unrolled.
template <int E, typename T = unsigned long long>
__device__ __forceinline__ void wave_bitonic(T (&v)[E]) {
    const int lane = threadIdx.x & 63;
    constexpr int N = 64 * E;
#pragma unroll
    for (int k = 2; k <= N; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            if (j >= E) {
                const int m = j / E;
                const bool lower = (lane & m) == 0;
#pragma unroll
                for (int r = 0; r < E; ++r) {
                    const T p = __shfl_xor(v[r], m);
                    const bool up = ((lane * E + r) & k) == 0;
                    const T lo = v[r] < p ? v[r] : p, hi = v[r] < p ? p : v[r];
                    v[r] = (up == lower) ? lo : hi;
                }
            } else {
#pragma unroll
                for (int r = 0; r < E; ++r) {
                    if (r & j) continue;
                    const bool up = ((lane * E + r) & k) == 0;
                    const T a = v[r], b = v[r ^ j];
                    const T lo = a < b ? a : b, hi = a < b ? b : a;
                    v[r] = up ? lo : hi;
                    v[r ^ j] = up ? hi : lo;
                }
            }
        }
    }
}
// The k-th smallest of a wave's sorted keys (k < 64 * E, wave-uniform)
template <int E>
__device__ __forceinline__ unsigned long long wave_kth(const unsigned long long (&v)[E], int64_t k) {
    const int r = (int)(k % E), l = (int)(k / E);
    unsigned long long x = v[0];
#pragma unroll
    for (int i = 1; i < E; ++i) x = r == i ? v[i] : x;
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), l);
    return ((unsigned long long)hi << 32) | lo;
}
constexpr int kAmpSortE = 8;  // windows of <= 512 positions: medians by one wave's bitonic sort

__global__ __launch_bounds__(256) void k_amplicon(const int32_t* cov, const double* ent, const double* sec, int64_t L,
                                                  const int64_t* lo_a, const int64_t* hi_a, double* out) {
    __shared__ unsigned s_hist[256];
    __shared__ unsigned long long s_sel[2];
    __shared__ long long s_red[4];
    __shared__ int s_off[(2 << kLv) - 1], s_len[(2 << kLv) - 1];
    __shared__ double s_val[2 << kLv];
    const int t = blockIdx.x;
    int64_t lo = lo_a[t], hi = hi_a[t];
    if (lo < 0) lo = 0;
    if (hi > L - 1) hi = L - 1;
    double* o = out + (int64_t)t * 6;
    if (lo > hi) {
        if (threadIdx.x == 0)
            for (int j = 0; j < 6; ++j) o[j] = -1.0;
        return;
    }
    const int64_t n = hi - lo + 1;
    const int64_t k1 = (n - 1) / 2, k2 = n / 2;
    __shared__ unsigned long long s_med[3][2];
    constexpr int kWin = 64 * kAmpSortE;
    // windows of amplicon size (C4: ~300 positions): the three arrays staged in LDS once (every
    // load issued at once), then the sorts, the sums and numpy's pairwise means read LDS only
    __shared__ int32_t s_c[kWin];
    __shared__ double s_e[kWin], s_s[kWin];
    const bool sorted = n <= kWin;  // (uniform)
    if (sorted) {
        for (int i = threadIdx.x; i < n; i += blockDim.x) {
            s_c[i] = cov[lo + i];
            s_e[i] = ent[lo + i];
            s_s[i] = sec[lo + i];
        }
        __syncthreads();
        // waves 0-2 each sort one array's keys in registers (the doubles are >= 0, so their bit
        // patterns order like their values)
        const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
        if (wave < 3) {
            unsigned long long v[kAmpSortE];
#pragma unroll
            for (int r = 0; r < kAmpSortE; ++r) {  // (the input order does not matter)
                const int i = r * 64 + lane;
                v[r] = ~0ull;
                if (i < n)
                    v[r] = wave == 0 ? (unsigned long long)(uint32_t)s_c[i]
                                     : (unsigned long long)__double_as_longlong((wave == 1 ? s_e : s_s)[i]);
            }
            wave_bitonic<kAmpSortE>(v);
            const unsigned long long a = wave_kth<kAmpSortE>(v, k1), b = wave_kth<kAmpSortE>(v, k2);
            if (lane == 0) {
                s_med[wave][0] = a;
                s_med[wave][1] = b;
            }
        }
        __syncthreads();
    }
    // coverage: exact integer mean, median via 32-bit select
    long long cs = 0;
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) cs += sorted ? s_c[i] : cov[lo + i];
    cs = block_sum_i64(cs, s_red);
    auto ckey = [&](int64_t i) { return (unsigned long long)(uint32_t)cov[lo + i]; };
    const double c_a = sorted ? (double)s_med[0][0] : (double)radix_select(ckey, n, k1, 32, s_hist, s_sel);
    const double c_b = sorted ? (double)s_med[0][1]
                              : (k2 != k1) ? (double)radix_select(ckey, n, k2, 32, s_hist, s_sel) : c_a;
    const double* vals[2] = {sorted ? s_e : ent + lo, sorted ? s_s : sec + lo};
    double means[2], meds[2];
    for (int q = 0; q < 2; ++q) {
        const double* a = vals[q];
        means[q] = np_mean_block(a, n, s_off, s_len, s_val);
        auto dkey = [&](int64_t i) { return (unsigned long long)__double_as_longlong(a[i]); };
        const double va = __longlong_as_double(
            (long long)(sorted ? s_med[1 + q][0] : radix_select(dkey, n, k1, 64, s_hist, s_sel)));
        const double vb = __longlong_as_double(
            (long long)(sorted ? s_med[1 + q][1]
                               : (k2 != k1) ? radix_select(dkey, n, k2, 64, s_hist, s_sel)
                                            : (unsigned long long)__double_as_longlong(va)));
        meds[q] = (k2 != k1) ? ((0.0 + va) + vb) / 2.0 : (0.0 + va) / 1.0;
    }
    if (threadIdx.x == 0) {
        o[0] = (double)cs / (double)n;
        o[1] = (k2 != k1) ? ((0.0 + c_a) + c_b) / 2.0 : c_a;
        o[2] = means[0];
        o[3] = meds[0];
        o[4] = means[1];
        o[5] = meds[1];
    }
}

// ---- the fused --summarise-with-bed tail (main.py:469-551) after kernel 1 + 2 -------------------
// One launch: blocks 1 .. 3 n_tiles take one (amplicon window, array) each -- array 0 coverage,
// 1 entropy, 2 secondary entropy: its numpy mean and np.median -- and block 0 the summary:
// every buffer's 64 partials (k_stats_lane<LEAVES>: a whole buffer's 128-position leaves, the
// partial buffer's nodes one level above its leaves) added up numpy's tree by a wave, the
// buffers folded in order, the exact coverage sum and non-zero count.  The windows' medians: a
// window of <= 320 positions (kTailWin) is loaded one element per thread, each wave sorts its 64 keys
// (shuffles), and each thread counts the keys smaller than its own by a binary search in every
// wave's sorted run: the k-th smallest value is the largest one with at most k smaller keys (a
// wave max, then an LDS atomic max); longer windows take the radix select.  The means: numpy's
// pairwise sum (pw_fast) over the window in LDS.  Same values as k_amplicon + k_sum_chunks +
// k_sum_final.
#ifdef BC_TAIL_TRACE  // diagnostic: block 1's phase stamps (s_memtime; the first window's entropy) after the windows' outputs
#define TAIL_STAMP(k) \
    do { if (blockIdx.x == 1 && threadIdx.x == 0) amp[6 * n_tiles + (k)] = (double)__builtin_amdgcn_s_memtime(); } while (0)
#else
#define TAIL_STAMP(k) do {} while (0)
#endif
// Keys below x in NR sorted runs of 64 (LDS): NR branchless binary searches, interleaved
template <int NR, typename T>
__device__ __forceinline__ int runs_below(const T* run, T x) {
    int p[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) p[r] = 0;
#pragma unroll
    for (int st = 32; st > 0; st >>= 1)
#pragma unroll
        for (int r = 0; r < NR; ++r) p[r] += run[64 * r + p[r] + st - 1] < x ? st : 0;
    int lt = 0;
#pragma unroll
    for (int r = 0; r < NR; ++r) lt += p[r] + (run[64 * r + p[r]] < x ? 1 : 0);
    return lt;
}
// The k1-th and k2-th smallest of a window's n <= 512 keys, one per thread (pads ~0: never
// smaller than a key): each wave sorts its 64 keys by shuffles, each thread counts the keys
// below its own by a binary search in every wave's sorted run (by the waves that hold keys, in
// the runs that hold keys: a guard per run inside one unrolled loop compiled to a branch and a
// wait per read); x <= (k-th smallest) iff at most k keys are below x, so the k-th smallest is
// the largest such x: a wave max (shuffles), then one LDS max per wave (an atomicMax of every
// lane compiled to a scalar loop over the lanes, ~10 us per window) into s_sel (zeroed, read
// after the caller's next barrier).  T: the coverage's 32 bits (half the shuffles and compares)
// or an entropy's 64.  An all-pairs compare loop cost 10k cycles per window.
template <typename T, int NWM>
__device__ __forceinline__ void window_kth(T x, bool in, int64_t n, int64_t k1, int64_t k2, T* s_run,
                                           unsigned long long* s_sel) {
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    T v[1] = {x};
    wave_bitonic<1, T>(v);
    s_run[t] = v[0];
    __syncthreads();
    const int nr = (int)((n + 63) / 64);
    int lt = 0;
    if (wave < nr) {
        // (uniform; the search of nr runs unrolled at compile time; nr <= NWM, and the runs
        // past n hold pads only, which count 0)
        switch (nr) {
            case 1: lt = runs_below<1, T>(s_run, x); break;
            case 2: lt = runs_below<2, T>(s_run, x); break;
            case 3: lt = runs_below<3, T>(s_run, x); break;
            case 4: lt = runs_below<4, T>(s_run, x); break;
            default: lt = runs_below<NWM, T>(s_run, x); break;
        }
    }
    T c1 = (in && lt <= k1) ? x : (T)0, c2 = (in && lt <= k2) ? x : (T)0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const T d1 = __shfl_xor(c1, o), d2 = __shfl_xor(c2, o);
        c1 = d1 > c1 ? d1 : c1;
        c2 = d2 > c2 ? d2 : c2;
    }
    if (lane == 0) {
        atomicMax(&s_sel[0], (unsigned long long)c1);
        atomicMax(&s_sel[1], (unsigned long long)c2);
    }
}
constexpr int kTailThreads = 320;  // five waves: amplicon windows (C4: 201-279 positions) in one pass
constexpr int kTailWin = kTailThreads;  // one position per thread
__global__ __launch_bounds__(kTailThreads) void k_tail(const int32_t* cov, const double* ent, const double* sec, int64_t L,
                                              const int64_t* lo_a, const int64_t* hi_a, int n_tiles, double* amp,
                                              Leaves lv, double* out) {
    __shared__ unsigned s_hist[256];
    __shared__ unsigned long long s_sel[2];
    __shared__ long long s_red[kTailThreads / 64];
    __shared__ int s_off[(2 << kLv) - 1], s_len[(2 << kLv) - 1];
    __shared__ double s_val[2 << kLv];
    __shared__ unsigned long long s_key[kTailWin];  // the window's values in order (numpy's mean)
    __shared__ unsigned long long s_run[kTailWin];  // ... and each wave's 64 of them sorted
    constexpr int NW = kTailThreads / 64;
    __shared__ double s_buf[NW];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    // block 0 the summary (dispatched first: the longest chain), then the entropy blocks of every
    // window, then the coverage ones (no pairwise mean: the lightest, so the blocks past one per
    // CU that share a CU with another are these)
    if (blockIdx.x == 0) {  // (uniform) the summary
        TAIL_STAMP(0);
        // the partial buffer's tree above its 64 nodes: which of lane's ancestors split
        const int m = (int)(L - lv.full);
        unsigned split = 0;
        {
            int n = m;
#pragma unroll
            for (int l = 0; l < kLv - 1; ++l) {
                split |= (unsigned)(n > 128) << l;
                const int n2 = n > 128 ? (n >> 1) & ~7 : n;
                n = ((lane >> (kLv - 2 - l)) & 1) ? n - n2 : n2;
            }
        }
        const int64_t nfull = lv.full / kNpBuf, nbuf = nfull + (m > 0);
        double s = 0.0;
        long long cs = 0, nz = 0;
        for (int64_t b0 = 0; b0 < nbuf; b0 += NW) {
            const int64_t b = b0 + wave;
            double v = 0.0;
            if (b < nbuf) {
                const int64_t f = b * 64 + lane;
                v = lv.ent[f];
                cs += lv.cov[f];
                nz += lv.nz[f];
            }
            // numpy's tree over a buffer's 64 nodes: node i of level d in lane i << (6 - d), its
            // right child 2^(5-d) lanes up; a whole buffer splits everywhere (pw_full8192's order)
            const unsigned sp = b < nfull ? ~0u : split;
#pragma unroll
            for (int d = kLv - 2; d >= 0; --d) {
                const double c1 = __shfl_down(v, 1 << (kLv - 2 - d));
                v = ((sp >> d) & 1) ? v + c1 : v;
            }
            if (lane == 0) s_buf[wave] = v;
            __syncthreads();
            if (t == 0)
                for (int w = 0; w < NW && b0 + w < nbuf; ++w) s += s_buf[w];  // buffers in order
            __syncthreads();
        }
        TAIL_STAMP(1);
        cs = block_sum_i64(cs, s_red);
        nz = block_sum_i64(nz, s_red);
        if (t == 0) {
            const double n = (double)L;
            out[0] = (double)cs / n;  // integer sum exact in float64 below 2^53: np.mean == sum / n
            out[1] = s / n;
            out[2] = (double)nz;
            out[3] = (double)cs;
        }
        return;
    }
    TAIL_STAMP(0);
    const int bq = (int)blockIdx.x - 1;
    const int w = bq < 2 * n_tiles ? bq >> 1 : bq - 2 * n_tiles, q = bq < 2 * n_tiles ? 1 + (bq & 1) : 0;
    int64_t lo = lo_a[w], hi = hi_a[w];
    if (lo < 0) lo = 0;
    if (hi > L - 1) hi = L - 1;
    double* o = amp + (int64_t)w * 6 + 2 * q;
    if (lo > hi) {
        if (t == 0) o[0] = o[1] = -1.0;
        return;
    }
    const int64_t n = hi - lo + 1;
    const int64_t k1 = (n - 1) / 2, k2 = n / 2;
    // keys that order like the values: the coverage as an unsigned int, the entropies (>= 0) by
    // their bit patterns
    auto key = [&](int64_t i) -> unsigned long long {
        return q == 0 ? (unsigned long long)(uint32_t)cov[lo + i]
                      : (unsigned long long)__double_as_longlong((q == 1 ? ent : sec)[lo + i]);
    };
    unsigned long long a, b;
    double mean;
    if (n <= kTailWin) {  // (uniform)
        const bool in = t < n;
        if (t < 2) s_sel[t] = 0ull;  // (read after window_kth's and the mean's barriers)
        if (q == 0) {  // (uniform) coverage: 32-bit keys; the exact integer sum
            const uint32_t x = in ? (uint32_t)cov[lo + t] : ~0u;
            window_kth<uint32_t, NW>(x, in, n, k1, k2, (uint32_t*)s_run, s_sel);
            TAIL_STAMP(1);
            const long long cs = block_sum_i64(in ? (long long)x : 0, s_red);  // (its barriers order s_sel)
            mean = (double)cs / (double)n;
        } else {  // the entropies' bit patterns; numpy's pairwise mean over the window in LDS
            const unsigned long long x = in ? key(t) : ~0ull;
            s_key[t] = x;
            window_kth<unsigned long long, NW>(x, in, n, k1, k2, s_run, s_sel);
            TAIL_STAMP(1);
            __syncthreads();
            mean = pw_fast<kTailThreads, 4>((const double*)s_key, (int)n, s_val) / (double)n;  // (n <= kTailWin)
        }
        TAIL_STAMP(2);
        a = s_sel[0];
        b = s_sel[1];
        TAIL_STAMP(3);
    } else {  // a long window: radix selects
        const int bits = q == 0 ? 32 : 64;
        a = radix_select(key, n, k1, bits, s_hist, s_sel);
        b = k2 != k1 ? radix_select(key, n, k2, bits, s_hist, s_sel) : a;
        if (q == 0) {
            long long cs = 0;
            for (int64_t i = t; i < n; i += kTailThreads) cs += (long long)(uint32_t)cov[lo + i];
            cs = block_sum_i64(cs, s_red);
            mean = (double)cs / (double)n;
        } else {
            mean = np_mean_block((q == 1 ? ent : sec) + lo, n, s_off, s_len, s_val);
        }
    }
    if (t == 0) {
        o[0] = mean;
        if (q == 0) {
            const double ca = (double)a, cb = (double)b;
            o[1] = (k2 != k1) ? ((0.0 + ca) + cb) / 2.0 : ca;
        } else {
            const double va = __longlong_as_double((long long)a), vb = __longlong_as_double((long long)b);
            o[1] = (k2 != k1) ? ((0.0 + va) + vb) / 2.0 : (0.0 + va) / 1.0;
        }
    }
}

}  // namespace

// ------------------------------------------------------------------------------ launchers
hipError_t launch_count(hipStream_t s, const bc_reads& r, int64_t ref_len, uint32_t mbq, int ncols,
                        int32_t* hist, int rpb, unsigned long long* d_err) {
    if (r.n_reads <= 0) return hipSuccess;
    CountArgs A;
    A.pos = r.pos;
    A.cig_beg = r.cig_beg;
    A.cig_n = r.cig_n;
    A.seq_nib = r.seq_nib;
    A.cigar = r.cigar;
    A.seq = r.seq;
    A.qual = r.qual;
    A.n = r.n_reads;
    A.ref_len = ref_len;
    A.mbq = mbq;
    A.ncols = ncols;
    A.rpb = rpb;
    A.max_span = r.max_span;
    A.sorted = r.sorted;
    A.layout = r.seq_layout;
    A.hist = hist;
    A.err = d_err;
    const int64_t nblk = (r.n_reads + rpb - 1) / rpb;
    if (mbq > 0)
        hipLaunchKernelGGL(k_count<true>, dim3((unsigned)nblk), dim3(kCountThreads), 0, s, A);
    else
        hipLaunchKernelGGL(k_count<false>, dim3((unsigned)nblk), dim3(kCountThreads), 0, s, A);
    return hipGetLastError();
}

size_t seq_event_bytes(int64_t seq_bytes) {
    return (size_t)((seq_bytes > 0 ? seq_bytes : 0) + 15) / 16 * 16 + 16;
}

hipError_t launch_seq_event(hipStream_t s, const uint8_t* src, int64_t nbytes, uint8_t* dst) {
    const int64_t out = (int64_t)seq_event_bytes(nbytes);
    int64_t blocks = (out / 16 + 255) / 256;
    if (blocks > 256 * 32) blocks = 256 * 32;
    hipLaunchKernelGGL(k_seq_event, dim3((unsigned)blocks), dim3(256), 0, s, src, nbytes, dst, out);
    return hipGetLastError();
}

hipError_t launch_span(hipStream_t s, const bc_reads& r, int* d_max_span) {
    if (r.n_reads <= 0) return hipSuccess;
    int64_t blocks = (r.n_reads + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(k_span, dim3((unsigned)blocks), dim3(256), 0, s, r.cig_beg, r.cig_n, r.cigar, r.n_reads,
                       d_max_span);
    return hipGetLastError();
}

// kernel 2's shape: 1 = k_stats_lane (one lane per position), 2 = k_stats_oct (eight lanes per
// position: 6.8 vs 7.1 us per launch by event pairs, but the C3 step 37.2-38.3 vs 36.5-37.1 us,
// A/B x2), 0 = k_stats (one wave per column); -DBC_STATS_LANE=<n> builds the A/B variants
#ifndef BC_STATS_LANE
#define BC_STATS_LANE 1
#endif
constexpr int kStatsShape = BC_STATS_LANE;

hipError_t launch_stats(hipStream_t s, const int32_t* hist, int64_t L, int k, double nf, double nf2, int32_t* cov,
                        double* pc, double* ent, double* sec, int32_t* scratch_counts_out) {
    if (L <= 0) return hipSuccess;
    int64_t blocks = (L + 63) / 64;  // one 64-position tile per block
    if (blocks > 256 * 8 * 8) blocks = 256 * 8 * 8;
    int32_t* h = const_cast<int32_t*>(hist);  // written only in scratch mode (scratch_counts_out)
    if (kStatsShape == 2) {
        const unsigned ob = (unsigned)((L + 31) / 32);
        if (k == 5)
            hipLaunchKernelGGL(k_stats_oct<5>, dim3(ob), dim3(256), 0, s, h, L, nf, nf2, scratch_counts_out, cov, pc,
                               ent, sec);
        else
            hipLaunchKernelGGL(k_stats_oct<6>, dim3(ob), dim3(256), 0, s, h, L, nf, nf2, scratch_counts_out, cov, pc,
                               ent, sec);
        return hipGetLastError();
    }
    if (kStatsShape == 1) {
        const unsigned lb = (unsigned)((L + 255) / 256);
        if (k == 5)
            hipLaunchKernelGGL(k_stats_lane<5>, dim3(lb), dim3(256), 0, s, h, L, nf, nf2, scratch_counts_out, cov, pc,
                               ent, sec);
        else
            hipLaunchKernelGGL(k_stats_lane<6>, dim3(lb), dim3(256), 0, s, h, L, nf, nf2, scratch_counts_out, cov, pc,
                               ent, sec);
        return hipGetLastError();
    }
    if (k == 5)
        hipLaunchKernelGGL(k_stats<5>, dim3((unsigned)blocks), dim3(64 * 5), 0, s, h, L, nf, nf2,
                           scratch_counts_out, cov, pc, ent, sec);
    else
        hipLaunchKernelGGL(k_stats<6>, dim3((unsigned)blocks), dim3(64 * 6), 0, s, h, L, nf, nf2,
                           scratch_counts_out, cov, pc, ent, sec);
    return hipGetLastError();
}

size_t summary_work_bytes(int64_t L) {
    const int64_t nc = (L + kNpBuf - 1) / kNpBuf;
    // header; per buffer: its partials + its 4 quarters', and its 64 leaves' (the fused tail)
    return 16 + (size_t)(nc > 0 ? nc : 1) * (24 * 5 + 24 * 64);
}

// the leaf partials inside a summary work buffer (after the buffer and quarter partials)
static Leaves summary_leaves(void* work, int64_t L) {
    const int64_t nc = (L + kNpBuf - 1) / kNpBuf, m = nc > 0 ? nc : 1;
    Leaves lv;
    lv.ent = (double*)((uint8_t*)work + 16 + (size_t)m * 24 * 5);
    lv.cov = (long long*)(lv.ent + 64 * m);
    lv.nz = lv.cov + 64 * m;
    lv.full = (L / kNpBuf) * kNpBuf;
    return lv;
}

hipError_t launch_stats_leaves(hipStream_t s, int32_t* hist, int64_t L, int k, double nf, double nf2, int32_t* cov,
                               double* ent, double* sec, int32_t* counts_out, void* work) {
    if (L <= 0) return hipSuccess;
    const Leaves lv = summary_leaves(work, L);
    const unsigned lb = (unsigned)(lv.full / 256 + (L > lv.full ? 64 : 0));  // + the partial buffer's nodes
    if (k == 5)
        hipLaunchKernelGGL((k_stats_lane<5, true>), dim3(lb), dim3(256), 0, s, hist, L, nf, nf2, counts_out, cov,
                           nullptr, ent, sec, lv);
    else
        hipLaunchKernelGGL((k_stats_lane<6, true>), dim3(lb), dim3(256), 0, s, hist, L, nf, nf2, counts_out, cov,
                           nullptr, ent, sec, lv);
    return hipGetLastError();
}

hipError_t launch_tail(hipStream_t s, const int32_t* cov, const double* ent, const double* sec, int64_t L, void* work,
                       double* out, const int64_t* lo, const int64_t* hi, int n_tiles, double* amp) {
    if (L <= 0) return hipSuccess;
    const Leaves lv = summary_leaves(work, L);
    hipLaunchKernelGGL(k_tail, dim3((unsigned)(3 * n_tiles + 1)), dim3(kTailThreads), 0, s, cov, ent, sec, L, lo, hi,
                       n_tiles, amp, lv, out);
    return hipGetLastError();
}

SumParts summary_parts(void* work, int64_t L) {
    const int64_t nc = (L + kNpBuf - 1) / kNpBuf;
    const int64_t m = nc > 0 ? nc : 1;
    SumParts P;
    P.hdr = (int32_t*)work;  // [0]: buffers whose partials are in the quarter arrays
    P.ent = (double*)((uint8_t*)work + 16);
    P.cov = (long long*)(P.ent + m);
    P.nz = P.cov + m;
    P.sub_ent = (double*)(P.nz + m);
    P.sub_cov = (long long*)(P.sub_ent + 4 * m);
    P.sub_nz = P.sub_cov + 4 * m;
    P.fused = false;
    P.full_chunks = 0;
    return P;
}

// first_chunk > 0: the partials of the buffers before it are already in the work buffer (written
// by the sparse pileup sweep, bc_pileup_summary); only the rest are computed here
hipError_t launch_summary_partials(hipStream_t s, const int32_t* cov, const double* ent, int64_t L, void* work,
                                   int64_t first_chunk, bool quarters) {
    const int64_t nc = (L + kNpBuf - 1) / kNpBuf;
    const SumParts P = summary_parts(work, L);
    // the header tells the fold how many leading buffers come as quarters (stream-ordered): written
    // by the first launch below, or by a memset when there is none
    const int32_t hval = quarters ? (int32_t)first_chunk : 0;
    const int64_t nfull = L / kNpBuf;  // whole buffers: k_sum_chunks; the partial one: k_sum_tail
    const bool chunks = nfull > first_chunk, tail = nc > nfull && nfull >= first_chunk;
    if (!chunks && !tail) return hipMemsetD32Async((hipDeviceptr_t)P.hdr, hval, 1, s);
    const size_t tail_lds = (size_t)(L - nfull * kNpBuf) * sizeof(double);
    if (chunks && tail && nfull - first_chunk <= 64) {  // a short reference: whole buffers and tail in one launch
        hipLaunchKernelGGL(k_sum_chunks<true>, dim3((unsigned)(nfull - first_chunk + 1)), dim3(256), tail_lds, s, cov,
                           ent, L, P.ent, P.cov, P.nz, first_chunk, P.hdr, hval);
        return hipGetLastError();
    }
    if (chunks)
        hipLaunchKernelGGL(k_sum_chunks<false>, dim3((unsigned)(nfull - first_chunk)), dim3(256), 0, s, cov, ent, L,
                           P.ent, P.cov, P.nz, first_chunk, P.hdr, hval);
    if (tail)
        hipLaunchKernelGGL(k_sum_tail, dim3(1), dim3(256), (size_t)(L - nfull * kNpBuf) * sizeof(double), s, cov, ent,
                           L, P.ent, P.cov, P.nz, nfull, chunks ? nullptr : P.hdr, hval);
    return hipGetLastError();
}

hipError_t launch_summary_fold(hipStream_t s, int n, const int64_t* L, void* const* work, double* const* out) {
    for (int i0 = 0; i0 < n; i0 += kFoldMax) {
        FoldArgs FA;
        std::memset(&FA, 0, sizeof FA);
        const int m = n - i0 < kFoldMax ? n - i0 : kFoldMax;
        for (int i = 0; i < m; ++i) {
            const SumParts P = summary_parts(work[i0 + i], L[i0 + i]);
            FA.ref[i] = FoldRef{P.ent,    P.cov,  P.nz, P.sub_ent, P.sub_cov, P.sub_nz,
                                P.hdr,    (L[i0 + i] + kNpBuf - 1) / kNpBuf, L[i0 + i], out[i0 + i]};
        }
        hipLaunchKernelGGL(k_sum_final, dim3((unsigned)m), dim3(kFoldThreads), 0, s, FA);
    }
    return hipGetLastError();
}

hipError_t launch_summary(hipStream_t s, const int32_t* cov, const double* ent, int64_t L, void* work, double* out,
                          int64_t first_chunk) {
    hipError_t e = launch_summary_partials(s, cov, ent, L, work, first_chunk);
    if (e != hipSuccess) return e;
    return launch_summary_fold(s, 1, &L, &work, &out);
}

hipError_t launch_amplicons(hipStream_t s, const int32_t* cov, const double* ent, const double* sec, int64_t L,
                            const int64_t* lo, const int64_t* hi, int n_tiles, double* out) {
    if (n_tiles <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_amplicon, dim3((unsigned)n_tiles), dim3(256), 0, s, cov, ent, sec, L, lo, hi, out);
    return hipGetLastError();
}

}  // namespace bc
