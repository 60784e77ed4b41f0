// bc_pileup.hip — the fused, position-tiled pileup kernel (kernel 1 + kernel 2 in ONE launch).
//
// Layout: the reference is cut into 64-position tiles; a tile is owned by a group of S waves.
// Reads are coordinate-sorted, so the reads overlapping a tile form one contiguous index range,
// read from the batch's tile index (bc_reads.tile_reads) or found by a 64-ary search over pos[].  They are processed in chunks of 64: each lane
// loads one read and decodes its CIGAR into a run table (count.cpp:40-96 semantics), the chunk's
// packed sequence is staged into LDS, and then the chunk is walked with
//     lane = (window g = lane >> 3, read slot s = lane & 7):
// the lane assembles the 8 event classes its read has in reference window [t0+8g, t0+8g+8) as
// ONE 32-bit word (a funnel shift of the BC_SEQ_EVENT sequence per CIGAR run, deletions as class
// 1100) and counts all 8 positions x 6 columns with SWAR nibble counters: ~30 VALU per 8 bases.
// No atomics and no histogram memset: the 8 read slots are reduced with DPP, the S waves of a
// group through LDS, the tile's counts are written once with coalesced stores (count.cpp's
// baseCounts), and the per-position statistics of main.py:29-53 are computed in the same launch
// (kernel 2 fused).  Reads with more than 8 CIGAR ops / 4 runs take a per-position walk.
//
// Positions >= L (the last, partial tile and "edge" tiles past the reference end, up to the
// furthest read end) do not count: a counted event there is the reference's std::out_of_range
// (count.cpp:60-65,85) and is recorded as the first offending read index.
#include "bc_tile.h"

namespace bc {
namespace {

template <bool QUAL, int K, bool STATS, typename IT>
__global__ __launch_bounds__(512, 4) void k_pileup(PileArgs A) {
    extern __shared__ __attribute__((aligned(16))) unsigned char dyn[];
    __shared__ IT rng[8][2];  // per group: the tile's read range
    if (BC_ABL(A) & 64) return;
    trace_stamp(A, 0);
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nw = blockDim.x >> 6;
    const int S = A.S;
    const int g = wave / S, ws = wave - g * S;
    const int groups = nw / S;
    uint4* rec_all = (uint4*)dyn;
    uint8_t* stage_all = dyn + (size_t)nw * kRecBytes;
    uint32_t(*fin)[6][kTile] = (uint32_t(*)[6][kTile])(stage_all + (size_t)nw * kStageRegion);
    // aliases of the stage regions, live only after the walk (see pileup_lds_bytes)
    double* terms_g = (double*)(stage_all + (size_t)(g * S) * kStageRegion);
    // IT: the index type of reads, tiles and positions (int32_t when they fit: scalar math)
    const IT n_tiles = (IT)A.n_tiles;
    const IT nblk_tiles = (n_tiles + groups - 1) / groups;
    const IT L = (IT)A.L;
    const int s8 = lane & 7;
    const bool qual_vec = ((uintptr_t)A.qual & 15u) == 0;

    // XCD-aware: workgroups are dispatched round-robin over the 8 XCDs; give each XCD a
    // contiguous run of tiles so neighbouring tiles (which share ~2/3 of their reads) hit the
    // same L2 instead of fetching the reads' CIGAR / sequence from HBM once per tile
    const IT G = gridDim.x;
    const IT lb = (G % 8 == 0) ? (IT)(blockIdx.x % 8) * (G / 8) + (IT)(blockIdx.x / 8) : (IT)blockIdx.x;
    for (IT bt = lb; bt < nblk_tiles; bt += G) {
        const IT t = bt * groups + g;
        const IT t0 = t * kTile;
        const IT P = t0 + lane;
        const int gb = (int)t0 + 8 * (lane >> 3);  // this lane's window [gb, gb + 8)
        uint32_t cnt[6] = {0, 0, 0, 0, 0, 0};
        int64_t bad = INT64_MAX;
        // the tile's reads [lo, hi): searched by the group's first wave (the S waves would all
        // find the same range), handed to the others through LDS
        IT lo = 0, hi = 0;
        if (ws == 0 && t < n_tiles && !(BC_ABL(A) & 2)) {
#ifdef BC_PHASE_TRACE
            if (A.trace) {  // diagnostic: latency of one dependent global load from here
                const int32_t probe = A.pos[(lane * 1543) % (int)A.n];
                if (probe == 0x7FFFFFFF) A.trace[0] = 1;
                trace_stamp(A, 8);
                const int32_t probe2 = A.pos[(lane * 977 + 5 + (probe & 1)) % (int)A.n];
                if (probe2 == 0x7FFFFFFF) A.trace[0] = 1;
                trace_stamp(A, 10);
                const int32_t probe3 = A.cigar[(lane * 977 + 11 + (probe2 & 1)) % (int)A.n];
                if (probe3 == 0x7FFFFFFF) A.trace[0] = 1;
                trace_stamp(A, 11);
            }
#endif
            if (t < A.n_trange) {  // the upload's tile index: one load instead of a search
                const int2 rg = A.trange[t];
                lo = rg.x;
                hi = rg.y;
            } else {
                int64_t l64, h64;
                lower_bound_pair(A.pos, A.n, (int64_t)t0 - A.max_span + 1, (int64_t)t0 + kTile, lane, l64, h64);
                lo = (IT)l64;
                hi = (IT)h64;
            }
            trace_stamp(A, 9);
        }
        if (S > 1) {
            if (ws == 0 && lane == 0) rng[g][0] = lo, rng[g][1] = hi;
            if (ws == 0) {  // the S waves add their counts here after the walk
#pragma unroll
                for (int c = 0; c < K; ++c) fin[g][c][lane] = 0u;
            }
            __syncthreads();
            trace_stamp(A, 1);
            lo = rng[g][0];
            hi = rng[g][1];
        }
        if (t < n_tiles) {
            if (BC_ABL(A) & 1) hi = lo;
            const bool edge = t0 + kTile > L;  // uniform
            const bool beyond = P >= L;
            uint32_t bmask = 0;                // window nibbles at positions >= L
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
            uint4* myrec = rec_all + wave * kTile * 3;
            uint8_t* mystage = stage_all + (size_t)wave * kStageRegion + 16;
            auto chunk_nr = [&](IT b) { return b < hi ? (int)((hi - b) < 64 ? (hi - b) : 64) : 0; };
            IT base = lo + (IT)ws * 64;
            ReadFields F = load_fields(A, base, chunk_nr(base), lane);
#ifdef BC_PHASE_TRACE
            int nch = 0;
#endif
            for (; base < hi; base += (IT)S * 64) {
                const IT nb = base + (IT)S * 64;
                process_chunk<QUAL, K>(A, base, chunk_nr(base), F, nb, chunk_nr(nb), lane, s8, gb, t0, P, edge,
                                       beyond, bmask, myrec, mystage, qual_vec, W, it4, cnt, acc, pending, bad);
                __builtin_amdgcn_wave_barrier();
#ifdef BC_PHASE_TRACE
                if (nch < 2) trace_stamp(A, 2 + nch);
                ++nch;
#endif
            }
            flush_acc(acc, cnt);
            if (it4) swar_fold<K>(W, cnt, s8);
            if (edge) {  // first offending read of this tile (std::out_of_range in the reference)
                for (int o = 32; o > 0; o >>= 1) {
                    const int64_t b2 = __shfl_down(bad, o);
                    bad = b2 < bad ? b2 : bad;
                }
                if (lane == 0 && bad != INT64_MAX) atomicMin(A.err, (unsigned long long)bad);
            }
        }
        // ---- reduce the S waves of the group: LDS atomics into fin (zeroed before the range
        // barrier), so every wave reads the totals after one barrier
        if (S > 1) {
#pragma unroll
            for (int c = 0; c < K; ++c) atomicAdd(&fin[g][c][lane], cnt[c]);
            __syncthreads();
            trace_stamp(A, 4);
            if (ws == 0) {
#pragma unroll
                for (int c = 0; c < K; ++c) cnt[c] = fin[g][c][lane];
            }
        }
        const bool own = t < n_tiles && t0 < L && !(BC_ABL(A) & 16);  // tile holds real positions
        if (ws == 0) {
#pragma unroll
            for (int c = 0; c < K; ++c) {
                if (own && P < L) {
                    int32_t* dst = A.counts + (int64_t)c * L + P;
                    if (A.accumulate) cnt[c] += (uint32_t)*dst;
                    *dst = (int32_t)cnt[c];
                }
                if (S == 1 || A.accumulate) fin[g][c][lane] = cnt[c];
            }
        }
        if (!STATS || (BC_ABL(A) & 8)) {
            if (S > 1) __syncthreads();
            continue;
        }
        if (S == 1 || A.accumulate) __syncthreads();  // (uniform) fin written by wave 0 above
        trace_stamp(A, 5);
        // ---- fused kernel 2: per-lane fp64 terms, then ordered sums per position
        if (own) tile_terms<K>(A, &fin[g][0][0], terms_g, t0, ws * 64 + lane, S * 64);
        __syncthreads();
        trace_stamp(A, 6);
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
                    if (cnt[j] != 0) s = s + terms_g[j * kTile + lane];
                h = A.nf * s;
                if (cov - (int64_t)mx != 0) {
                    double s2 = 0.0;
#pragma unroll
                    for (int j = 0; j < K; ++j) {
                        const double tj = terms_g[(K + j) * kTile + lane];
                        if (tj != 0.0) s2 = s2 + tj;
                    }
                    h2 = A.nf2 * s2;
                }
            }
            A.ent[P] = h;
            A.sec[P] = h2;
        }
        __syncthreads();
        trace_stamp(A, 7);
    }
}

// ---- sparse batches (at most ~48 reads per tile): one wave per tile, tiles swept in order ----

// Kernel 2 for one position from its counts (bc_stats.h: the same arithmetic as tile_terms + the
// ordered sums of k_pileup), written by the position's lane.
template <int K>
__device__ __forceinline__ double pos_stats(const PileArgs& A, const uint32_t* c, int64_t P) {
    return position_stats<K>(c, A.L, P, A.nf, A.nf2, A.cov, A.pc, A.ent, A.sec);
}

// Move a read cursor forward to the first index >= cur whose pos >= key (pos is sorted and the
// keys of successive tiles increase).  `win` holds pos[wbase + lane]: the 64 reads after the
// cursor are looked at with one ballot, refilled only when the cursor leaves them.
// IT: the index type of reads and positions (int32_t when both fit, so the cursor arithmetic
// stays on the scalar unit; int64_t otherwise).
template <typename IT>
__device__ __forceinline__ void advance_cursor(const int32_t* pos, IT n, IT& cur, IT key, int32_t& win, IT& wbase,
                                               int lane) {
    for (;;) {
        if (cur >= n) return;
        if (cur >= wbase + 64) {
            wbase = cur;
            const IT i = wbase + lane;
            win = i < n ? pos[i] : INT32_MAX;
        }
        const int below = __popcll(__ballot((IT)win < key));  // a prefix of the window
        IT end = wbase + below;
        end = end < n ? end : n;
        if (end > cur) cur = end;
        if (below < 64 || cur >= n) return;
        cur = wbase + 64;
    }
}

// Sparse batches: every wave owns a contiguous run of tiles and sweeps it with two read cursors
// (no per-tile search), walks the few reads of each tile alone, and computes the statistics of
// its own positions in registers: no block barriers at all.  Empty tiles only store.
// STORE = false (with STATS and SUMP; bc_pileup_partials with no outputs, the summary of
// main.py:469-499): no per-position output at all but the last partial buffer's coverage and
// entropy; the summary partials alone are written, and a quarter buffer with no reads is one
// constant store (its 16 leaves are 128.0 each: 2048.0, exactly).
// per wave: a quarter's 16 leaves, then the 64-double transposition scratch (80 doubles: four
// 4-wave workgroups with their records and stages fit a CU's 160 KiB of LDS)
constexpr int kLeafDoubles = 16 + 64;
static_assert(4 * (4 * (kRecBytes + kStageRegion) + 4 * kLeafDoubles * 8) <= 160 * 1024, "4 workgroups per CU");
template <bool QUAL, int K, bool STATS, bool SUMP, typename IT, bool STORE = true>
__global__ __launch_bounds__(256, 4) void k_pileup_solo(PileArgs A) {
    static_assert(STORE || (STATS && SUMP), "the summary-only sweep computes the summary partials");
    extern __shared__ __attribute__((aligned(16))) unsigned char dyn[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nw = blockDim.x >> 6;
    uint4* myrec = (uint4*)dyn + wave * kTile * 3;
    uint8_t* mystage = dyn + (size_t)nw * kRecBytes + (size_t)wave * kStageRegion + 16;
    const IT L = (IT)A.L, n = (IT)A.n;
    const int s8 = lane & 7;
    const bool qual_vec = ((uintptr_t)A.qual & 15u) == 0;
    const IT G = gridDim.x;
    const IT lb = (G % 8 == 0) ? (IT)(blockIdx.x % 8) * (G / 8) + (IT)(blockIdx.x / 8) : (IT)blockIdx.x;
    const IT tpw = (IT)A.tiles_per_wave;
    const IT t_begin = (lb * nw + wave) * tpw;
    const IT t_end = t_begin + tpw < (IT)A.n_tiles ? t_begin + tpw : (IT)A.n_tiles;
    if (t_begin >= t_end) return;  // no barriers in this kernel
    IT lo, hi;
    {
        int64_t l64, h64;
        lower_bound_pair(A.pos, A.n, (int64_t)t_begin * kTile - A.max_span + 1, (int64_t)t_begin * kTile + kTile, lane,
                         l64, h64);
        lo = (IT)l64;
        hi = (IT)h64;
    }
    IT wlo_base = lo, whi_base = hi;
    int32_t wlo = lo + lane < n ? A.pos[lo + lane] : INT32_MAX;
    int32_t whi = hi + lane < n ? A.pos[hi + lane] : INT32_MAX;
    const IT max_span = (IT)A.max_span;
    // SUMP: the wave's tiles start on a quarter-buffer boundary (tiles_per_wave is a multiple of
    // 32), so it sees whole 2048-position quarters, each a subtree of numpy's pairwise tree over
    // an 8192 buffer (split evenly down to 128-element leaves): leaves of two tiles wait in LDS (16
    // per quarter) and are added pairwise across the lanes once the quarter is complete; the fold
    // kernel joins the 4 quarters of a buffer
    double e_prev = 0.0;
    bool prev_empty = false;
    double* myleaves = (double*)(dyn + (size_t)nw * (kRecBytes + kStageRegion)) + kLeafDoubles * wave;
    double* mytr = myleaves + 16;  // transposition scratch of the leaf sums (64 doubles)
    long long sum_cov = 0, sum_nz = 0;
    // SUMP: tile t's share of numpy's pairwise leaves (h: its entropies; an empty tile's are 1.0)
    auto leaf_step = [&](IT t, bool empty, double h) {
        if (t & 1) {
            const double lf = (prev_empty && empty) ? 128.0
                              : empty                 ? leaf_finish_ones(prev_empty ? 8.0 : e_prev, lane, mytr)
                                                      : leaf_finish(prev_empty ? 8.0 : e_prev, h, lane, mytr);
            const int leaf = (int)((t >> 1) & 15);
            if (lane == 0) myleaves[leaf] = lf;
            if (leaf == 15) {  // the quarter is complete: its 16 leaves, pairwise
                __builtin_amdgcn_wave_barrier();
                double v = myleaves[lane & 15];
#pragma unroll
                for (int l = 1; l < 16; l <<= 1) {  // left (lower lanes) + right
                    const double w = __shfl_down(v, l);
                    if ((lane & (2 * l - 1)) == 0) v = v + w;
                }
                const long long cs = wave_sum_i64(sum_cov), nz = wave_sum_i64(sum_nz);
                if (lane == 0) {
                    const int64_t q = t >> 5;
                    A.sub_ent[q] = v;
                    A.sub_cov[q] = cs;
                    A.sub_nz[q] = nz;
                }
                sum_cov = sum_nz = 0;
            }
        } else {
            prev_empty = empty;  // an empty first tile's half is 8.0 (leaf_finish_ones)
            if (!empty) e_prev = leaf_half(h, lane, mytr);  // its half of the chains
        }
    };
    for (IT t = t_begin; t < t_end; ++t) {
        const IT t0 = t * kTile;
        const IT P = t0 + lane;
        const int gb = (int)t0 + 8 * (lane >> 3);
        if (t > t_begin) {
            advance_cursor<IT>(A.pos, n, lo, t0 - max_span + 1, wlo, wlo_base, lane);
            advance_cursor<IT>(A.pos, n, hi, t0 + kTile, whi, whi_base, lane);
        }
        if (STATS && lo >= hi && !A.accumulate && !(BC_ABL(A) & 16)) {
            // No read overlaps this tile, nor any tile before the next read's start tile: write
            // that run of full tiles' constant outputs (main.py:29-53 at zero coverage) without
            // per-tile cursor work.  The next tile with reads resumes the normal path.
            IT nxt = t_end;
            if (hi < n) {
                const IT d = hi - whi_base;  // in [0, 64]: the window holds pos[whi_base ..]
                const int32_t ph = d < 64 ? (int32_t)__builtin_amdgcn_readlane(whi, (int)d) : A.pos[hi];
                nxt = (IT)(ph >> 6);
            }
            IT stop = nxt < t_end ? nxt : t_end;
            const IT full = L / kTile;  // tiles entirely below L
            stop = stop < full ? stop : full;
            if (stop > t + 1) {
                for (; t < stop; ++t) {
                    const IT tz = t * kTile;
                    const bool whole = SUMP && (int64_t)(tz >> 13) < A.full_chunks;  // in a whole buffer
                    if (STORE) {
#pragma unroll
                        for (int c = 0; c < K; ++c) (A.counts + ((int64_t)c * L + tz))[lane] = 0;
                        (A.cov + tz)[lane] = 0;
                        if (A.pc) {
#pragma unroll
                            for (int j = 0; j < K; ++j) (A.pc + ((int64_t)j * L + tz))[lane] = -1.0;
                        }
                        (A.ent + tz)[lane] = 1.0;
                        (A.sec + tz)[lane] = 1.0;
                    } else if (!whole) {  // the last partial buffer: coverage 0, entropy 1
                        const int64_t i = (int64_t)tz - A.full_chunks * kNpBuf + lane;
                        A.cov_tail[i] = 0;
                        A.ent_tail[i] = 1.0;
                        continue;
                    } else if ((t & 31) == 0 && t + 32 <= stop) {
                        // a whole quarter without reads (32 tiles, one subtree of numpy's tree;
                        // the quarters before it left the coverage sums at 0)
                        if (lane == 0) {
                            const int64_t q = (int64_t)(t >> 5);
                            A.sub_ent[q] = 2048.0;
                            A.sub_cov[q] = 0;
                            A.sub_nz[q] = 0;
                        }
                        t += 31;
                        continue;
                    }
                    if (whole) leaf_step(t, true, 1.0);
                }
                --t;  // the loop's increment moves to `stop`
                continue;
            }
        }
        uint32_t cnt[6] = {0, 0, 0, 0, 0, 0};
        if (hi > lo) {
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
            for (int64_t base = lo; base < (int64_t)hi; base += 64) {
                process_chunk<QUAL, K>(A, base, chunk_nr(base), F, base + 64, chunk_nr(base + 64), lane, s8, gb, t0, P,
                                       edge, beyond, bmask, myrec, mystage, qual_vec, W, it4, cnt, acc, pending, bad);
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
        const bool empty = hi <= lo;  // (uniform) no read overlaps the tile: all counts zero
        if (!STORE && t0 < L && P < L) {  // summary only: coverage and entropy, no stores
            uint32_t cov;
            const double h = position_entropy<K>(cnt, A.nf, cov);
            if ((int64_t)(t0 >> 13) < A.full_chunks) {
                if (!empty) {
                    sum_cov += cov;
                    sum_nz += cov != 0;
                }
                leaf_step(t, empty, h);
            } else {
                const int64_t i = (int64_t)P - A.full_chunks * kNpBuf;
                A.cov_tail[i] = (int32_t)cov;
                A.ent_tail[i] = h;
            }
        } else if (STORE && t0 < L && P < L && !(BC_ABL(A) & 16)) {
#pragma unroll
            for (int c = 0; c < K; ++c) {
                int32_t* cb = A.counts + ((int64_t)c * L + t0);  // (uniform)
                if (A.accumulate) cnt[c] += (uint32_t)cb[lane];
                cb[lane] = (int32_t)cnt[c];
            }
            if (STATS) {
                // (an explicit zero-coverage branch here costs registers: the kernel spills)
                const double h = pos_stats<K>(A, cnt, P);
                if (SUMP) {
                    static_assert(kNpBuf == 8192 && kNpBuf == 128 * kTile, "buffers of 128 tiles");
                    const int64_t ch = t0 >> 13;  // 8192-position buffer
                    if (ch < A.full_chunks) {
                        if (!empty) {
                            const uint32_t cov = cnt[0] + cnt[1] + cnt[2] + cnt[3] + cnt[4] + (K == 6 ? cnt[5] : 0u);
                            sum_cov += cov;
                            sum_nz += cov != 0;
                        }
                        leaf_step(t, empty, h);
                    }
                }
            }
        }
    }
}

}  // namespace


int pileup_waves(const bc_reads& r, int64_t L, int64_t max_end, int tile_waves) {
    if (tile_waves == 1 || tile_waves == 2 || tile_waves == 4 || tile_waves == 8) return tile_waves;
    // waves per tile from the mean number of reads a tile walks
    // reads overlapping a tile ~ density * (span + 63); aim for ~48 reads per wave
    const int64_t reach = max_end > L ? max_end : L;
    const double per_tile = reach > 0 ? (double)r.n_reads * (double)(r.max_span + kTile - 1) / (double)reach : 0.0;
    int S = 1;
    while (S < 8 && per_tile > 48.0 * S) S *= 2;
    return S;
}

hipError_t launch_pileup_tiles(hipStream_t s, const bc_reads& r, int64_t L, int64_t max_end, uint32_t mbq, int k,
                               bool stats, bool accumulate, double nf, double nf2, int32_t* counts, int32_t* cov,
                               double* pc, double* ent, double* sec, unsigned long long* d_err, int shape,
                               int tile_waves, SumParts* parts) {
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
#ifdef BC_DIAG
    if (const char* ab = std::getenv("BC_ABLATE")) A.ablate = std::atoi(ab);
#endif
    const int S = pileup_waves(r, L, max_end, tile_waves);
    A.S = S;
    if (parts) parts->fused = false;
    if (S == 1 && shape != BC_SHAPE_TILE_NO_SOLO) {
        // sparse: waves sweep contiguous tile runs; ~8 rounds of resident waves (256 CUs x 16): shorter
        // runs shorten the last round's tail (C5: 31.6 ms at 2 rounds, 30.2-30.6 at 4-8, 30.4-30.8 at 16-32)
        const int nw = 4;
        const int64_t target_waves = 256 * 16 * 8;
        A.tiles_per_wave = (A.n_tiles + target_waves - 1) / target_waves;
        if (A.tiles_per_wave < 1) A.tiles_per_wave = 1;
        const bool sump = parts && stats && L >= kNpBuf;
        const bool nostore = sump && parts->no_store;
        if (sump) {  // whole quarter buffers per wave: the summary partials come for free
            A.tiles_per_wave = (A.tiles_per_wave + 31) / 32 * 32;
            A.sub_ent = parts->sub_ent;
            A.sub_cov = parts->sub_cov;
            A.sub_nz = parts->sub_nz;
            A.full_chunks = L / kNpBuf;
            parts->fused = true;
            parts->full_chunks = A.full_chunks;
            A.cov_tail = parts->cov_tail;
            A.ent_tail = parts->ent_tail;
        }
        const int64_t waves = (A.n_tiles + A.tiles_per_wave - 1) / A.tiles_per_wave;
        int64_t blocks = (waves + nw - 1) / nw;
        blocks = (blocks + 7) / 8 * 8;  // a multiple of the XCD count (see the kernel's tile mapping)
        const dim3 grid((unsigned)blocks), block(64 * nw);
        const size_t lds = (size_t)nw * (kRecBytes + kStageRegion) + (sump ? (size_t)nw * kLeafDoubles * 8 : 0);
        // 32-bit reads and positions when they fit (the cursor loop then stays on the scalar unit)
        const bool i32 = A.n < (int64_t)0x7FFFFF00 && A.n_tiles * kTile + A.max_span + 2 * kTile < (int64_t)0x7FFFFF00;
#define BC_SOLO(Q, KK, ST)                                                                                       \
    do {                                                                                                         \
        if (nostore && i32)                                                                                      \
            hipLaunchKernelGGL((k_pileup_solo<Q, KK, true, true, int32_t, false>), grid, block, lds, s, A);      \
        else if (nostore) hipLaunchKernelGGL((k_pileup_solo<Q, KK, true, true, int64_t, false>), grid, block, lds, s, A); \
        else if (sump && i32) hipLaunchKernelGGL((k_pileup_solo<Q, KK, true, true, int32_t>), grid, block, lds, s, A); \
        else if (sump) hipLaunchKernelGGL((k_pileup_solo<Q, KK, true, true, int64_t>), grid, block, lds, s, A);   \
        else if (i32) hipLaunchKernelGGL((k_pileup_solo<Q, KK, ST, false, int32_t>), grid, block, lds, s, A);     \
        else hipLaunchKernelGGL((k_pileup_solo<Q, KK, ST, false, int64_t>), grid, block, lds, s, A);              \
    } while (0)
        if (mbq > 0) {
            if (k == 5) {
                if (stats) BC_SOLO(true, 5, true); else BC_SOLO(true, 5, false);
            } else {
                if (stats) BC_SOLO(true, 6, true); else BC_SOLO(true, 6, false);
            }
        } else {
            if (k == 5) {
                if (stats) BC_SOLO(false, 5, true); else BC_SOLO(false, 5, false);
            } else {
                if (stats) BC_SOLO(false, 6, true); else BC_SOLO(false, 6, false);
            }
        }
#undef BC_SOLO
        return hipGetLastError();
    }
    const int nw = S >= 4 ? S : 4;
    const int groups = nw / S;
    int64_t blocks = (A.n_tiles + groups - 1) / groups;
    const int64_t cap = 256 * 64;
    if (blocks > cap) blocks = cap;
    blocks = (blocks + 7) / 8 * 8;  // a multiple of the XCD count (see the kernel's tile mapping)
    const dim3 grid((unsigned)blocks), block(64 * nw);
    const size_t lds = pileup_lds_bytes(nw, groups);
    // diagnostic only: BC_TRACE=<file> dumps the per-wave phase stamps of the 20th launch
    static unsigned long long* tbuf = nullptr;
    static int tcalls = 0;
#ifdef BC_PHASE_TRACE
    const char* tpath = std::getenv("BC_TRACE");
#else
    const char* tpath = nullptr;
#endif
    const size_t tn = (size_t)blocks * nw * kTracePhases;
    if (tpath) {
        if (!tbuf && hipMallocManaged((void**)&tbuf, 8 * (size_t)256 * 64 * 16 * kTracePhases) != hipSuccess) tbuf = nullptr;
        if (tn <= (size_t)256 * 64 * 16 * kTracePhases) A.trace = tbuf;
    }
    // 32-bit reads, tiles and positions when they fit
    const bool i32 = A.n < (int64_t)0x7FFFFF00 && A.n_tiles * kTile + A.max_span + 2 * kTile < (int64_t)0x7FFFFF00;
    // > 64 KiB of dynamic LDS must be allowed per kernel (160 KiB per CU on gfx950)
#define BC_PILE(Q, KK, ST)                                                                                   \
    do {                                                                                                     \
        static bool attr_set = false;                                                                        \
        if (!attr_set) {                                                                                     \
            (void)hipFuncSetAttribute((const void*)k_pileup<Q, KK, ST, int32_t>,                             \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - 1024);        \
            (void)hipFuncSetAttribute((const void*)k_pileup<Q, KK, ST, int64_t>,                             \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - 1024);        \
            attr_set = true;                                                                                 \
        }                                                                                                    \
        if (i32) hipLaunchKernelGGL((k_pileup<Q, KK, ST, int32_t>), grid, block, lds, s, A);                 \
        else hipLaunchKernelGGL((k_pileup<Q, KK, ST, int64_t>), grid, block, lds, s, A);                     \
        if (A.trace && ++tcalls == 20) {                                                                     \
            (void)hipStreamSynchronize(s);                                                                   \
            if (FILE* f = std::fopen(tpath, "wb")) {                                                         \
                std::fwrite(A.trace, 8, tn, f);                                                              \
                std::fclose(f);                                                                              \
            }                                                                                                \
        }                                                                                                    \
    } while (0)
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
