// bc_sum.hip — summary only (main.py:469-499) for sparse sorted batches: the read-parallel
// summary, see below.
#include "bc_tile.h"

namespace bc {
namespace {

// ---- summary only, sparse batches: the read-parallel summary (main.py:469-499) ------------------
//
// numpy's mean of the entropies is a pairwise sum whose leaves are 128 consecutive positions.  A
// position no read covers has entropy 1 (int), one that a single read covers with a counted event
// has 0.0 (one class: position_entropy), so a leaf in which no position is covered by two reads
// holds integers only and sums exactly to 128 - (its positions with a counted event), in any
// order.  Only a leaf some position of which two reads cover can hold a fractional entropy, and
// only such a leaf needs the exact per-position walk in numpy's order.  Reads are sorted by start,
// so read i shares a position with a later read only inside [pos[i + 1], end_i): those intervals
// cover every position of coverage >= 2.
//   k_sum_reads    one lane per read: its counted positions added per leaf (leaf_cnt, <= 3 atomics
//                  per 150 bp read), the leaves of [pos[i + 1], end_i) listed once each (dlist),
//                  and the reference's out_of_range check for reads reaching past L;
//   k_sum_exact    one wave per listed leaf: its two tiles walked like k_pileup_solo, the leaf's
//                  exact pairwise sum, coverage and non-zero count; first the tiles of the last
//                  partial buffer, whose per-position coverage / entropy the fold's tail reads;
//   k_sum_buffers  numpy's pairwise tree over the 64 leaves of every whole 8192-position buffer
//                  (the per-buffer partials the fold adds in order), re-zeroing the leaf arrays.
// The same numbers as k_pileup_solo<STORE = false> bit for bit, with ~10x fewer tile walks at
// C5's depth (every non-empty tile there, only the overlapping ones here).

// Counted events (K = 5: A C G T, one bit per nibble; K = 6: N 0011 too) among the aligned bases
// at nibble indices [q0, q0 + len) of the BC_SEQ_EVENT buffer, with the quality test.
template <bool QUAL, int K>
__device__ __forceinline__ int count_counted(const PileArgs& A, int64_t q0, int64_t len, bool qual_vec) {
    const uint32_t* sw = (const uint32_t*)A.seq;
    const int64_t q1 = q0 + len;
    int c = 0;
    for (int64_t w = q0 >> 3; w <= (q1 - 1) >> 3; ++w) {
        const int64_t b = w * 8;
        const int kl = q0 > b ? (int)(q0 - b) : 0, kh = q1 - b < 8 ? (int)(q1 - b) : 8;
        uint32_t x = sw[w] & nib_range(kl, kh);
        if (QUAL) {
            if (qual_vec && b + 8 <= A.qual_bytes) {
                const uint2 q = *(const uint2*)(A.qual + b);
                x &= qual_nibmask(q.x, q.y, A.mbq);
            } else {
                x &= qual_mask_at(SeqSrc{sw, A.seq_words, A.qual, A.qual_bytes, A.mbq}, b);
            }
        }
        uint32_t nz = (x | (x >> 1) | (x >> 2) | (x >> 3)) & kM1;
        if (K == 5) nz &= ~(x & (x >> 1));  // N (0011) is not coverage
        c += __popc(nz);
    }
    return c;
}

// Does a run reach a position >= L with an event the reference would count (count.cpp:60-65,85:
// counts.at(refPos) on a base in A C G T N passing the quality test, or on a deletion)?
template <bool QUAL>
__device__ __forceinline__ bool run_beyond(const PileArgs& A, bool mrun, int64_t r0, int64_t r1, int64_t q0) {
    const int64_t a = r0 > A.L ? r0 : A.L;
    if (a >= r1) return false;
    if (!mrun) return true;
    for (int64_t r = a; r < r1; ++r) {
        const int64_t q = q0 + (r - r0);
        const uint32_t nib = (A.seq[q >> 1] >> ((q & 1) * 4)) & 15u;
        if (nib && (!QUAL || (q < A.qual_bytes && (uint32_t)A.qual[q] >= A.mbq))) return true;
    }
    return false;
}

template <bool QUAL, int K>
__global__ __launch_bounds__(256) void k_sum_reads(PileArgs A) {
    const int64_t n = A.n;
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;  // no barriers in this kernel
    const int64_t p = A.pos[i];
    const uint32_t cb = A.cig_beg[i], cn = A.cig_n[i];
    const int64_t sn = A.seq_nib[i];
    const int64_t nxt = i + 1 < n ? (int64_t)A.pos[i + 1] : INT64_MAX;
    const int64_t lim = A.nleaf * 128;  // positions of the whole buffers
    const bool qual_vec = ((uintptr_t)A.qual & 7u) == 0;
    int64_t leaf = -1;
    int acc = 0;
    bool bad = false;
    int64_t rc = 0, qc = 0;
    for (uint32_t k = 0; k < cn; ++k) {
        const uint32_t w = A.cigar[cb + k], op = w & 15u, len = w >> 4;
        const bool m = mlike(op);
        if (m || dlike(op)) {
            const int64_t r0 = p + rc, r1 = r0 + len, q0 = sn + qc;
            const int64_t rl = r1 < lim ? r1 : lim;
            for (int64_t r = r0; r < rl;) {  // leaf by leaf
                const int64_t e = ((r | 127) + 1) < rl ? ((r | 127) + 1) : rl;
                const int c = m ? count_counted<QUAL, K>(A, q0 + (r - r0), e - r, qual_vec) : (int)(e - r);
                if ((r >> 7) != leaf) {
                    if (acc) atomicAdd(&A.leaf_cnt[leaf], acc);
                    leaf = r >> 7;
                    acc = 0;
                }
                acc += c;
                r = e;
            }
            if (r1 > A.L && !bad) bad = run_beyond<QUAL>(A, m, r0, r1, q0);
            rc += len;
        }
        if (qcons(op)) qc += len;
    }
    if (acc) atomicAdd(&A.leaf_cnt[leaf], acc);
    if (bad) atomicMin(A.err, (unsigned long long)i);
    // positions this read shares with later reads: [pos[i + 1], end), listed leaf by leaf
    const int64_t end = p + rc;
    const int64_t ol = nxt > 0 ? nxt : 0, oh = end < lim ? end : lim;
    for (int64_t l = ol >> 7; ol < oh && l <= (oh - 1) >> 7; ++l) {
        if (atomicCAS(&A.leaf_mark[l], 0, -1) == 0) {
            const int s = atomicAdd(A.ndirty, 1);
            A.dlist[s] = (int32_t)l;
            A.leaf_mark[l] = s + 1;  // (read after this launch)
        }
    }
}

// The counts of the lane's position in tile t (k_pileup_solo's walk of one tile) from its reads
// [lo, hi) (lo < 0: found by one search here).
template <bool QUAL, int K>
__device__ __forceinline__ void tile_counts(const PileArgs& A, int64_t t, int lane, uint4* myrec, uint8_t* mystage,
                                            bool qual_vec, uint32_t (&cnt)[6], int64_t lo = -1, int64_t hi = -1) {
    const int64_t t0 = t * kTile, P = t0 + lane, L = A.L;
    const int gb = (int)t0 + 8 * (lane >> 3);
    const int s8 = lane & 7;
#pragma unroll
    for (int c = 0; c < 6; ++c) cnt[c] = 0;
    if (lo < 0) lower_bound_pair(A.pos, A.n, t0 - A.max_span + 1, t0 + kTile, lane, lo, hi);
    if (hi <= lo) return;
    int64_t bad = INT64_MAX;
    const bool edge = t0 + kTile > L;
    const bool beyond = P >= L;
    uint32_t bmask = 0;
    if (edge) {
        int64_t kL = L - gb;
        kL = kL < 0 ? 0 : (kL > 8 ? 8 : kL);
        bmask = ~(lo32_bit(4 * (int)kL) - 1u);
    }
    unsigned long long acc = 0;
    int pending = 0;
    Swar W;
#pragma unroll
    for (int c = 0; c < 6; ++c) W.a4[c] = 0;
    int it4 = 0;
    auto chunk_nr = [&](int64_t b) { return b < hi ? (int)((hi - b) < 64 ? (hi - b) : 64) : 0; };
    ReadFields F = load_fields(A, lo, chunk_nr(lo), lane);
    for (int64_t base = lo; base < hi; base += 64) {
        process_chunk<QUAL, K>(A, base, chunk_nr(base), F, base + 64, chunk_nr(base + 64), lane, s8, gb, t0, P, edge,
                               beyond, bmask, myrec, mystage, qual_vec, W, it4, cnt, acc, pending, bad);
        __builtin_amdgcn_wave_barrier();
    }
    flush_acc(acc, cnt);
    if (it4) swar_fold<K>(W, cnt, s8);
    if (edge) {
        for (int o = 32; o > 0; o >>= 1) {
            const int64_t b2 = __shfl_down(bad, o);
            bad = b2 < bad ? b2 : bad;
        }
        if (lane == 0 && bad != INT64_MAX) atomicMin(A.err, (unsigned long long)bad);
    }
}

constexpr int kSumTr = 64;  // doubles of leaf transposition scratch per wave
template <bool QUAL, int K>
__global__ __launch_bounds__(256, 2) void k_sum_exact(PileArgs A) {
    extern __shared__ __attribute__((aligned(16))) unsigned char dyn[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nw = blockDim.x >> 6;
    uint4* myrec = (uint4*)dyn + wave * kTile * 3;
    uint8_t* mystage = dyn + (size_t)nw * kRecBytes + (size_t)wave * kStageRegion + 16;
    double* tr = (double*)(dyn + (size_t)nw * (kRecBytes + kStageRegion)) + kSumTr * wave;
    const bool qual_vec = ((uintptr_t)A.qual & 15u) == 0;
    const int64_t tail0 = A.full_chunks * kNpBuf;
    const int64_t items = A.n_tail_tiles + (int64_t)__builtin_amdgcn_readfirstlane(*A.ndirty);
    const int64_t stride = (int64_t)gridDim.x * nw;
    uint32_t cnt[6];
    for (int64_t it = (int64_t)blockIdx.x * nw + wave; it < items; it += stride) {
        if (it < A.n_tail_tiles) {  // the last partial buffer: per-position coverage / entropy
            const int64_t t = tail0 / kTile + it;
            tile_counts<QUAL, K>(A, t, lane, myrec, mystage, qual_vec, cnt);
            const int64_t P = t * kTile + lane;
            if (P < A.L) {
                uint32_t cov;
                const double h = position_entropy<K>(cnt, A.nf, cov);
                A.cov_tail[P - tail0] = (int32_t)cov;
                A.ent_tail[P - tail0] = h;
            }
            continue;
        }
        const int64_t s = it - A.n_tail_tiles;
        const int64_t l = A.dlist[s];
        uint32_t cov0, cov1;
        // both tiles' read ranges in one search (a quarter-wave per bound), not one search per tile
        const int64_t t0 = 2 * l * kTile;
        const int64_t keys[4] = {t0 - A.max_span + 1, t0 + kTile, t0 + kTile - A.max_span + 1, t0 + 2 * kTile};
        int64_t rg[4];
        lower_bound_quad(A.pos, A.n, keys, lane, rg);
        tile_counts<QUAL, K>(A, 2 * l, lane, myrec, mystage, qual_vec, cnt, rg[0], rg[1]);
        const double h0 = position_entropy<K>(cnt, A.nf, cov0);
        const double half = leaf_half(h0, lane, tr);
        tile_counts<QUAL, K>(A, 2 * l + 1, lane, myrec, mystage, qual_vec, cnt, rg[2], rg[3]);
        const double h1 = position_entropy<K>(cnt, A.nf, cov1);
        const double leaf = leaf_finish(half, h1, lane, tr);
        const long long cs = wave_sum_i64((long long)cov0 + cov1);
        const long long nz = wave_sum_i64((long long)(cov0 != 0) + (cov1 != 0));
        if (lane == 0) {
            A.dval[s] = leaf;
            A.dcov[s] = cs;
            A.leaf_cnt[l] = (int32_t)nz;
        }
    }
}

// numpy's pairwise tree over the 64 leaves of every whole 8192-position buffer (one wave per
// buffer, lane = leaf; left + right at every level: the quarters' 16-leaf trees, then
// (q0 + q1) + (q2 + q3)), the leaves of single-read coverage as 128 - counted positions, into the
// per-buffer partials the fold adds in order; the leaf arrays are zeroed again for the next launch.
__global__ __launch_bounds__(256) void k_sum_buffers(PileArgs A) {
    const int lane = threadIdx.x & 63;
    const int64_t buf = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
    double v = 0.0;
    long long cs = 0, nz = 0;
    if (buf < A.full_chunks) {
        const int64_t l = buf * 64 + lane;
        const int32_t c = A.leaf_cnt[l], m = A.leaf_mark[l];
        if (m) {
            v = A.dval[m - 1];
            cs = A.dcov[m - 1];
            A.leaf_mark[l] = 0;
        } else {
            v = 128.0 - (double)c;
            cs = c;
        }
        nz = c;
        if (c) A.leaf_cnt[l] = 0;
    }
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const double w = __shfl_down(v, o);
        if ((lane & (2 * o - 1)) == 0) v = v + w;
        cs += __shfl_xor(cs, o);
        nz += __shfl_xor(nz, o);
    }
    if (lane == 0 && buf < A.full_chunks) {
        A.sub_ent[buf] = v;
        A.sub_cov[buf] = cs;
        A.sub_nz[buf] = nz;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) *A.ndirty = 0;  // k_sum_exact of this launch is done
}

}  // namespace

// scratch of the read-parallel summary: [ndirty, padded to 256 B][leaf_cnt][leaf_mark][dlist] int32
// per leaf, then [dval] f64 and [dcov] i64 per leaf (slots); zero when allocated, and kept zero
size_t sum_sparse_bytes(int64_t L) {
    const int64_t nleaf = (L > 0 ? L / kNpBuf : 0) * (kNpBuf / 128);
    return 256 + (size_t)nleaf * (4 + 4 + 4 + 8 + 8);
}

hipError_t launch_sum_sparse(hipStream_t s, const bc_reads& r, int64_t L, uint32_t mbq, int k, double nf,
                             unsigned long long* d_err, SumParts& parts, void* scratch, size_t scratch_bytes) {
    PileArgs A = make_args(r, L, mbq);
    A.nf = nf;
    A.err = d_err;
    A.full_chunks = L / kNpBuf;
    A.nleaf = A.full_chunks * (kNpBuf / 128);
    // the arrays sit at offsets fixed by the scratch's capacity, not by L: the zeroed leaf_cnt /
    // leaf_mark of one call are the zeroed arrays of the next call of any length (the slots,
    // dlist / dval / dcov, hold stale values that are never read unlisted)
    const int64_t cap = scratch_bytes > 256 ? (int64_t)((scratch_bytes - 256) / 28) & ~(int64_t)1 : 0;
    if (A.nleaf > cap) return hipErrorInvalidValue;
    uint8_t* p = (uint8_t*)scratch;
    A.ndirty = (int32_t*)p;
    p += 256;
    A.leaf_cnt = (int32_t*)p;
    A.leaf_mark = A.leaf_cnt + cap;
    A.dlist = A.leaf_mark + cap;
    A.dval = (double*)(A.dlist + cap);  // (cap even: 8-byte aligned)
    A.dcov = (long long*)(A.dval + cap);
    A.sub_ent = parts.ent;  // (k_sum_buffers: whole-buffer partials)
    A.sub_cov = parts.cov;
    A.sub_nz = parts.nz;
    parts.whole_buffers = true;
    A.cov_tail = parts.cov_tail;
    A.ent_tail = parts.ent_tail;
    A.n_tail_tiles = (L - A.full_chunks * kNpBuf + kTile - 1) / kTile;
    parts.fused = true;
    parts.full_chunks = A.full_chunks;
    const int nw = 4;
    const size_t lds = (size_t)nw * (kRecBytes + kStageRegion + kSumTr * 8);
    int64_t xb = (A.n_tail_tiles + A.nleaf + nw - 1) / nw;
    xb = xb < 1024 ? (xb < 1 ? 1 : xb) : 1024;
    const unsigned rb = (unsigned)((A.n + 255) / 256), qb = (unsigned)((A.full_chunks + 3) / 4);
#define BC_SUMS(Q, KK)                                                                                   \
    do {                                                                                                 \
        if (rb) hipLaunchKernelGGL((k_sum_reads<Q, KK>), dim3(rb), dim3(256), 0, s, A);                 \
        hipLaunchKernelGGL((k_sum_exact<Q, KK>), dim3((unsigned)xb), dim3(64 * nw), lds, s, A);          \
        if (qb) hipLaunchKernelGGL(k_sum_buffers, dim3(qb), dim3(256), 0, s, A);                        \
    } while (0)
    if (mbq > 0) {
        if (k == 5) BC_SUMS(true, 5); else BC_SUMS(true, 6);
    } else {
        if (k == 5) BC_SUMS(false, 5); else BC_SUMS(false, 6);
    }
#undef BC_SUMS
    return hipGetLastError();
}

}  // namespace bc