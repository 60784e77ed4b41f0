// bc_sort.hip — a coordinate-sorted copy of an unsorted batch, built on the device.
//
// The reference consumes reads in file order (main.py:127); counts do not depend on the order
// (count.cpp:22-97 adds one per event), but the fast kernels do: the tiled k_pileup walks a
// contiguous range of reads per tile and the read-chunked k_rc stages a chunk's contiguous
// sequence.  An unsorted batch (reads of one reference in any order) is therefore put in start
// order here, with no host round trip: bc_reads_sort only enqueues (stream-ordered, graph-
// capturable), every decision about the layout is taken on the device.  The default is the
// bucketed sort (k_bkt_*, below): no global atomics, per-block LDS histograms of the starts' high
// bits, one block per bucket sorting by the low bits, the sequence copied in destination order.
// References with more than 2^24 starts take the counting sort (one global atomic per read on its
// start's bin, k_sort_count + scan_u32 + k_sort_relay).
//
// The copy (both sorts): every read gets a slot of the same size, the batch's longest read's
// bytes, when those slots fit the copy's buffer (T = 1.5 x the batch's bytes); otherwise (reads of
// very different lengths) the slots shrink to half the batch's mean and a read longer than its
// slot takes its bytes from a bump allocator past the slots (one global atomic per such read).
// Either way everything fits T, so there is nothing to fall back to and nothing for the host to
// wait for.  Caller errors (a start outside [0, max_end], reads whose sequences overlap so the
// copy overflows) are flagged in a device word (bc_reads_sort_check reads it); the sorted copy is
// still safe to count (such reads are clamped to start 0 / given no CIGAR).
// Measured and dropped: one bin per 128-byte line (the count's atomics took as long), rocPRIM's
// radix sort of the (start, index) pairs (155 us for C3's 1 M pairs over 15 bits); the round-5
// exact fallback (gather + scanned offsets), which needed a blocking host read of the flags.
#include "bc_internal.h"

namespace bc {
namespace {

#include "bc_walk.h"

constexpr int kScanTile = 1024;  // elements per scan block (256 threads x 4)

__global__ __launch_bounds__(256) void k_scan_tiles(uint32_t* a, int64_t m, uint32_t* sums) {
    __shared__ uint32_t ws[4];
    const int64_t base = (int64_t)blockIdx.x * kScanTile + 4 * threadIdx.x;
    uint32_t v[4], t = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        v[k] = base + k < m ? a[base + k] : 0u;
        t += v[k];
    }
    // inclusive scan of the thread totals: wave (DPP-free shuffles), then across the 4 waves
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t inc = t;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(inc, o);
        if (lane >= o) inc += y;
    }
    if (lane == 63) ws[wave] = inc;
    __syncthreads();
    uint32_t before = 0;
    for (int w = 0; w < wave; ++w) before += ws[w];
    uint32_t run = before + inc - t;  // exclusive prefix of this thread's first element
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (base + k < m) a[base + k] = run;
        run += v[k];
    }
    if (threadIdx.x == 255) sums[blockIdx.x] = before + inc;
}

// one block: exclusive scan of the tile sums in place (any count, 1024 per pass with a carry)
__global__ __launch_bounds__(256) void k_scan_sums(uint32_t* sums, int64_t n, uint32_t* total) {
    __shared__ uint32_t ws[4];
    __shared__ uint32_t carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int64_t b0 = 0; b0 < n; b0 += kScanTile) {
        const int64_t base = b0 + 4 * threadIdx.x;
        uint32_t v[4], t = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            v[k] = base + k < n ? sums[base + k] : 0u;
            t += v[k];
        }
        uint32_t inc = t;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(inc, o);
            if (lane >= o) inc += y;
        }
        if (lane == 63) ws[wave] = inc;
        __syncthreads();
        uint32_t before = carry;
        for (int w = 0; w < wave; ++w) before += ws[w];
        uint32_t run = before + inc - t;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (base + k < n) sums[base + k] = run;
            run += v[k];
        }
        __syncthreads();
        if (threadIdx.x == 255) carry = before + inc;
        __syncthreads();
    }
    if (threadIdx.x == 0 && total) *total = carry;
}

__global__ __launch_bounds__(256) void k_scan_add(uint32_t* a, int64_t m, const uint32_t* sums) {
    const int64_t base = (int64_t)blockIdx.x * kScanTile + 4 * threadIdx.x;
    const uint32_t add = sums[blockIdx.x];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (base + k < m) a[base + k] += add;
}

// exclusive prefix sum of a[0, m) in place; tmp holds scan_tmp_words(m) words; *total (device,
// may be NULL) = the sum of all elements
size_t scan_tmp_words(int64_t m) { return (size_t)((m + kScanTile - 1) / kScanTile) + 1; }

hipError_t scan_u32(hipStream_t s, uint32_t* a, int64_t m, uint32_t* tmp, uint32_t* total) {
    const int64_t tiles = (m + kScanTile - 1) / kScanTile;
    if (tiles == 0) return total ? hipMemsetAsync(total, 0, 4, s) : hipSuccess;
    hipLaunchKernelGGL(k_scan_tiles, dim3((unsigned)tiles), dim3(256), 0, s, a, m, tmp);
    hipLaunchKernelGGL(k_scan_sums, dim3(1), dim3(256), 0, s, tmp, tiles, total);
    hipLaunchKernelGGL(k_scan_add, dim3((unsigned)tiles), dim3(256), 0, s, a, m, (const uint32_t*)tmp);
    return hipGetLastError();
}

struct SortArgs {
    const int32_t* pos;
    const uint32_t* cig_beg;
    const uint32_t* cig_n;
    const uint32_t* seq_nib;
    const uint32_t* cigar;
    const uint8_t* seq;
    const uint8_t* qual;
    int64_t n;
    uint32_t* bins;   // [nbins] counts, then offsets (counting sort)
    uint4* rec;       // counting sort: [2n] read i: {pos, cig_beg, cig_n, seq_nib}, {qlen, rank in its bin, 0, 0}
    int32_t* o_pos;
    uint32_t* o_cig_beg;
    uint32_t* o_cig_n;
    uint32_t* o_seq_nib;
    uint32_t* bump;     // bytes handed out past the fixed slots (device word, zeroed before the copy)
    uint32_t* overflow; // caller errors: bit 0 the copy overflowed (overlapping sequences), bit 1 a bad start
    uint32_t* qmax;     // the batch's largest query length (device word)
    uint8_t* o_seq;
    uint8_t* o_qual;
    uint32_t cap;       // the batch's bytes bound: seq_bytes + 5 n + 16 (every read's slot bytes sum to less)
    uint32_t room;      // bytes of o_seq (o_qual: twice as many): cap + cap / 2
    int64_t qual_bytes;
    int64_t nbins;      // bins: starts in [0, nbins - 1)
    // the bucketed variant (k_bkt_*): buckets of 2^wbits starts, nbkt of them; block b of the
    // count and scatter passes takes reads [b * chunk, (b + 1) * chunk)
    uint32_t* mat;      // [nblk][nbkt]: reads of bucket h in block b
    uint32_t* bbase;    // [nbkt + 1]: the first sorted slot of bucket h
    uint32_t* bstat;    // [nblk][2]: block b's largest query length, its flags
    uint4* brec;        // [n] {pos, cig_beg, seq_nib, cig_n | qlen << 16} in bucket order
    uint4* srec;        // [n] the same in start order
    // fields-only sorts (no sequence copy): each read's run record (bc_runs.h pack_runs) in bucket
    // order, and the sorted batch's run records
    uint4* brun;
    uint4* o_runs;
    int64_t chunk;
    int nblk, nbkt, wbits;
};

// read i: its rank inside its start's bin (one atomic on the bin), its query length from the
// CIGAR (M/I/=/X), and its fields packed into one 32-byte record (written coalesced); the batch's
// largest query length (one guarded atomic per block)
__global__ __launch_bounds__(256) void k_sort_count(SortArgs A) {
    __shared__ uint32_t wmax[4];
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    uint32_t q = 0;
    if (i < A.n) {
        int32_t pos = A.pos[i];
        if (pos < 0 || (int64_t)pos >= A.nbins - 1) {  // a start outside [0, max_end]: the caller's batch is wrong
            atomicOr(A.overflow, 2u);                     // (bc_reads_sort_check reports it)
            pos = 0;
        }
        const uint32_t cb = A.cig_beg[i], cn = A.cig_n[i], sn = A.seq_nib[i];
        const uint32_t rank = atomicAdd(&A.bins[pos], 1u);
        const uint32_t* cg = A.cigar + cb;
        uint32_t w[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) w[k] = (uint32_t)k < cn ? cg[k] : 0u;  // the loads issued together
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (qcons(w[k] & 15u)) q += w[k] >> 4;
        for (uint32_t k = 8; k < cn; ++k) {
            const uint32_t x = cg[k];
            if (qcons(x & 15u)) q += x >> 4;
        }
        A.rec[2 * i] = make_uint4((uint32_t)pos, cb, cn, sn);
        A.rec[2 * i + 1] = make_uint4(q, rank, 0u, 0u);
    }
    uint32_t m = q;
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t y = __shfl_xor(m, o);
        m = y > m ? y : m;
    }
    if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t a = wmax[0] > wmax[1] ? wmax[0] : wmax[1], b = wmax[2] > wmax[3] ? wmax[2] : wmax[3];
        const uint32_t bm = a > b ? a : b;
        if (bm > __hip_atomic_load(A.qmax, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(A.qmax, bm);
    }
}

// bytes of a read's copy: its aligned bases at its nibble parity, rounded up to whole words
__device__ __forceinline__ uint32_t read_words(uint32_t sn, uint32_t q) { return ((((sn & 1u) + q + 1u) >> 1) + 3u) >> 2; }

// The copy's slot size, the same in every thread: the longest read's bytes (at either nibble
// parity, in words) when n such slots fit the buffer -- then no read is longer than its slot --
// else half the batch's mean bytes per read, n slots taking at most cap / 2 and the longer reads
// at most cap (their bytes sum to less) from the bump allocator past them: room = 1.5 cap.
__device__ __forceinline__ uint32_t copy_slot(const SortArgs& A, uint32_t qmax) {
    const uint64_t full = (((uint64_t)qmax + 2u) / 2u + 3u) & ~3ull;
    if (full * (uint64_t)A.n <= (uint64_t)A.room) return (uint32_t)full;
    return (uint32_t)(((uint64_t)A.cap / (2u * (uint64_t)A.n)) & ~3ull);
}

// R sorted reads per 4-lane group (lane `sub` of the group): read r has start pos[r], CIGAR
// (cb[r], cn[r]), source nibble index sn[r], query length q[r] and sorted slot jj[r] (ok[r]:
// uniform in the group).  Its destination: slot jj[r] of the fixed slots, or (longer than a slot)
// bytes from the bump allocator; a destination past the buffer (the caller's reads overlap) is
// flagged and the read written with no CIGAR.  Fields (lane r & 3 writes read r's), the aligned
// sequence (two source words and a funnel shift per output word; every source word of the
// unrolled part requested first) and the qualities; the new nibble index keeps the old parity.
constexpr int kRelayWords = 5;  // words per lane per read in the unrolled part (20 per read: 160 bases)
template <int R>
__device__ __forceinline__ void copy_reads(const SortArgs& A, const uint32_t (&pos)[R], const uint32_t (&cb)[R],
                                           const uint32_t (&cn)[R], const uint32_t (&sn)[R], const uint32_t (&q)[R],
                                           const uint32_t (&jj)[R], const bool (&ok)[R], uint32_t sub, uint32_t slot) {
    uint32_t dst[R];
    bool keep[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint32_t bytes = 4u * read_words(sn[r], q[r]);
        dst[r] = slot * jj[r];
        keep[r] = true;
        if (ok[r] && bytes > slot) {  // (uniform in the lane group; only when the slots were shrunk)
            uint32_t at = 0;
            if (sub == 0) at = atomicAdd(A.bump, bytes);
            at = __shfl(at, 0, 4);
            const uint64_t end = (uint64_t)slot * (uint64_t)A.n + at + bytes;
            dst[r] = slot * (uint32_t)A.n + at;
            if (end > (uint64_t)A.room) {  // the reads' bytes exceed cap: overlapping sequences
                keep[r] = false;
                if (sub == 0) atomicOr(A.overflow, 1u);
            }
        }
    }
#pragma unroll
    for (int r = 0; r < R; ++r)
        if (ok[r] && sub == ((uint32_t)r & 3u)) {
            const uint32_t j = jj[r];
            A.o_pos[j] = (int32_t)pos[r];
            A.o_cig_beg[j] = cb[r];
            A.o_cig_n[j] = keep[r] ? cn[r] : 0u;
            A.o_seq_nib[j] = keep[r] ? 2u * dst[r] + (sn[r] & 1u) : 0u;
        }
    uint32_t x[R][kRelayWords + 1];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint32_t words = read_words(sn[r], q[r]);
        const uint32_t* s32 = (const uint32_t*)(A.seq + ((sn[r] >> 1) & ~3u));
#pragma unroll
        for (int k = 0; k <= kRelayWords; ++k) {
            const uint32_t w = sub + 4u * (uint32_t)k;
            x[r][k] = (ok[r] && keep[r] && w <= words) ? s32[w] : 0u;  // (word `words`: the last shift's upper half)
        }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if (!ok[r] || !keep[r]) continue;  // (uniform in the lane group)
        const uint32_t from = sn[r] >> 1, words = read_words(sn[r], q[r]);
        const uint32_t sh = (from & 3u) * 8u;
        const uint32_t* s32 = (const uint32_t*)(A.seq + (from & ~3u));
        uint32_t* d32 = (uint32_t*)(A.o_seq + dst[r]);
        // word w needs source words w and w + 1: w + 1 is the next lane's (lane 3: lane 0's next)
#pragma unroll
        for (int k = 0; k < kRelayWords; ++k) {
            const uint32_t w = sub + 4u * (uint32_t)k;
            const uint32_t nxt = __shfl_down(x[r][k], 1, 4), wrap = __shfl(x[r][k + 1], 0, 4);
            if (w < words) d32[w] = __builtin_amdgcn_alignbit(sub == 3u ? wrap : nxt, x[r][k], sh);
        }
        for (uint32_t w = sub + 4u * kRelayWords; w < words; w += 4)  // words past the unrolled part
            d32[w] = __builtin_amdgcn_alignbit(s32[w + 1], s32[w], sh);
        if (A.qual) {
            const uint64_t qf = 2 * (uint64_t)from;
            const uint32_t* q32 = (const uint32_t*)(A.qual + (qf & ~3ull));
            const uint32_t qsh = (uint32_t)(qf & 3u) * 8u;
            uint32_t* dq = (uint32_t*)(A.o_qual + 2 * (uint64_t)dst[r]);
            const uint64_t q0 = qf & ~3ull;
            for (uint32_t w = sub; w < 2 * words; w += 4) {
                if (q0 + 4ull * w + 8 <= (uint64_t)A.qual_bytes) {
                    dq[w] = __builtin_amdgcn_alignbit(q32[w + 1], q32[w], qsh);
                } else {  // the buffer's last bytes (the quality buffer has no padding)
                    uint32_t v = 0;
                    for (uint32_t bb = 0; bb < 4; ++bb) {
                        const uint64_t at = qf + 4ull * w + bb;
                        if (at < (uint64_t)A.qual_bytes) v |= (uint32_t)A.qual[at] << (8 * bb);
                    }
                    dq[w] = v;
                }
            }
        }
    }
}

// Counting sort's copy: reads i in SOURCE order (4 lanes per read, kRelayReads consecutive reads
// per lane group, their loads batched), read i's 32-byte record (coalesced), its sorted slot j =
// scanned bin of its start + its rank in the bin (no permutation array), then copy_reads.
constexpr int kRelayReads = 4;
__global__ __launch_bounds__(256) void k_sort_relay(SortArgs A) {
    const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const uint32_t sub = (uint32_t)g & 3u;
    const int64_t j0 = (g >> 2) * kRelayReads;
    if (j0 >= A.n) return;
    const uint32_t slot = copy_slot(A, *A.qmax);
    uint32_t pos[kRelayReads], cb[kRelayReads], cn[kRelayReads], sn[kRelayReads], q[kRelayReads], jj[kRelayReads];
    bool ok[kRelayReads];
#pragma unroll
    for (int r = 0; r < kRelayReads; ++r) {
        ok[r] = j0 + r < A.n;
        const size_t i = (size_t)(ok[r] ? j0 + r : j0);  // source read
        const uint4 a = A.rec[2 * i], b = A.rec[2 * i + 1];  // {pos, cig_beg, cig_n, seq_nib}, {qlen, rank}
        pos[r] = a.x, cb[r] = a.y, cn[r] = a.z, sn[r] = a.w, q[r] = b.x, jj[r] = b.y;
    }
#pragma unroll
    for (int r = 0; r < kRelayReads; ++r) jj[r] += A.bins[pos[r]];  // the read's sorted slot
    copy_reads<kRelayReads>(A, pos, cb, cn, sn, q, jj, ok, sub, slot);
}

// ---- the bucketed sort (no global atomics): starts binned by their high bits with per-block
// LDS histograms, each bucket then sorted by its low bits in one block, the sequence copied in
// start order.
//   k_bkt_count    block b: its reads' bucket histogram in LDS (the starts alone) -> row b of mat
//                  (every entry written);
//   k_bkt_scatter  block b: every bucket's total and the count of blocks before b from the rows
//                  (coalesced, L2-resident), their scan in LDS, then each read's slot in (bucket,
//                  block) from an LDS atomic with return; its 16-byte record (with the query
//                  length from its CIGAR) written there (a read whose CIGAR count or query
//                  length does not fit 16 bits: its source index instead, re-read by the copy);
//                  the block's largest query length and flags; block 0 also writes every
//                  bucket's first slot;
//   k_bkt_rank     one block per bucket, the bucket's records in registers: LDS counting sort by
//                  the low bits (histogram, scan, ranks), the records written in start order;
//                  block 0 folds the block stats into the batch's largest query length and the
//                  flags word, and zeroes the bump allocator;
//   k_bkt_copy     4 lanes per sorted slot: fields, sequence and qualities (copy_reads: fixed
//                  slots, so a wave writes whole lines of the copy, in destination order).
// 256 buckets of ~4,096 reads and 4,096-read blocks (C3: 245 of them, every CU busy) beat 512 buckets
// and 8,192-read blocks (123 CUs, the scatter's CIGAR decode VALU-bound on them): 88 vs 94 us.
// Measured and dropped: the scatter's first fields requested before the count rows are summed (no
// change, 25 us); rank and copy fused (one block per bucket staging its records in LDS and
// copying them): 79 us against 10 + 53; the matrix scanned by scan_u32 (3 launches, 14 us)
// instead of each scatter block summing the rows itself.
constexpr int kBktThreads = 1024;  // count / scatter blocks
constexpr int kBktGroup = 8;       // scatter: buckets per lane and rows per wave whose count loads
constexpr int kBktRows = 4;        // are in flight together
constexpr int kRankThreads = 1024;
constexpr int kRankRegs = 8;       // records per rank thread held in registers
constexpr int kBktMax = 4096;      // buckets (LDS words of the count / scatter passes)
constexpr int kBktTarget = 256;    // buckets aimed at (fewer starts per bucket: larger buckets)
constexpr int kBktChunk = 4096;    // reads per count / scatter block aimed at
constexpr int kBktLowMax = 4096;   // low-bit bins of one bucket (2^12)
constexpr uint32_t kQlenMax = 0xFFFFu;  // query lengths packed in 16 bits
constexpr int64_t kSortCapMax = 0x55555550;  // room = 1.5 cap < 2^31: nibble indices 2 * room fit 32 bits
// fields-only sorts: run records from the scatter's CIGAR loads (k_rc then loads a record per read
// instead of the read's CIGAR, which in a sorted view of an unsorted batch lies anywhere);
// off by default (no CIGAR loads in the sort at all): the unsorted C3 step measured faster without
// them (sort 34 vs 46 us, k_rc slower by less); -DBC_SORT_RUNS=1 builds the A/B variant
#ifndef BC_SORT_RUNS
#define BC_SORT_RUNS 0
#endif
constexpr bool kSortRuns = BC_SORT_RUNS != 0;
constexpr uint32_t kBigRec = 0xFFFFFFFFu;  // record word 3 of a read whose fields need 32 bits: word 2 = its index

__device__ __forceinline__ uint32_t bkt_pos(const SortArgs& A, int64_t i, bool& bad) {
    int32_t p = A.pos[i];
    bad = p < 0 || (int64_t)p >= A.nbins - 1;
    return bad ? 0u : (uint32_t)p;
}

// exclusive scan of s[0, m) in LDS by an NT-thread block (m <= NT * E); ws: NT / 64 words
template <int NT, int E>
__device__ __forceinline__ void lds_scan_excl(uint32_t* s, int m, uint32_t* ws) {
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    uint32_t v[E], tot = 0;
#pragma unroll
    for (int k = 0; k < E; ++k) {
        const int at = t * E + k;
        v[k] = at < m ? s[at] : 0u;
        tot += v[k];
    }
    uint32_t inc = tot;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(inc, o);
        if (lane >= o) inc += y;
    }
    if (lane == 63) ws[wave] = inc;
    __syncthreads();
    uint32_t run = inc - tot;
    for (int w = 0; w < wave; ++w) run += ws[w];
#pragma unroll
    for (int k = 0; k < E; ++k) {
        const int at = t * E + k;
        if (at < m) s[at] = run;
        run += v[k];
    }
    __syncthreads();
}

__global__ __launch_bounds__(kBktThreads) void k_bkt_count(SortArgs A) {
    __shared__ uint32_t hist[kBktMax];
    const int H = A.nbkt;
    const int64_t beg = (int64_t)blockIdx.x * A.chunk;
    const int64_t end = beg + A.chunk < A.n ? beg + A.chunk : A.n;
    constexpr int B = 8;  // reads per thread whose loads are in flight together
    uint32_t p[B];
    bool in[B];
    int64_t i0 = beg + threadIdx.x;
#pragma unroll
    for (int u = 0; u < B; ++u) {  // the first round's starts requested before the histogram is cleared
        const int64_t i = i0 + (int64_t)u * kBktThreads;
        bool bad;
        in[u] = i < end;
        p[u] = in[u] ? bkt_pos(A, i, bad) : 0u;
    }
    for (int h = threadIdx.x; h < H; h += kBktThreads) hist[h] = 0u;
    __syncthreads();
    for (;;) {
#pragma unroll
        for (int u = 0; u < B; ++u)
            if (in[u]) atomicAdd(&hist[p[u] >> A.wbits], 1u);
        i0 += (int64_t)B * kBktThreads;
        if (i0 - threadIdx.x >= end) break;  // (uniform)
#pragma unroll
        for (int u = 0; u < B; ++u) {
            const int64_t i = i0 + (int64_t)u * kBktThreads;
            bool bad;
            in[u] = i < end;
            p[u] = in[u] ? bkt_pos(A, i, bad) : 0u;
        }
    }
    __syncthreads();
    for (int h = threadIdx.x; h < H; h += kBktThreads) A.mat[(int64_t)blockIdx.x * H + h] = hist[h];
}

// Every bucket's total and its reads in blocks before b, added into next / pre (LDS, zeroed):
// wave v takes rows v, v + 16, ..., R of them per round, lane the buckets lane + 64 m, m < G
// (every load of a round issued before its adds); the 16 waves' partial sums meet in LDS.  The
// rows were written by blocks on every XCD, so each round is a trip past this XCD's L2.
template <int G, int R>
__device__ __forceinline__ void count_rows(const SortArgs& A, int b, uint32_t* next, uint32_t* pre) {
    const int H = A.nbkt, nb = A.nblk;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    constexpr int NW = kBktThreads / 64;
    for (int h0 = 0; h0 < H; h0 += 64 * G) {
        uint32_t tot[G], before[G];
#pragma unroll
        for (int m = 0; m < G; ++m) tot[m] = 0u, before[m] = 0u;
        for (int r0 = wave; r0 < nb; r0 += NW * R) {
            uint32_t v[R][G];
#pragma unroll
            for (int u = 0; u < R; ++u)
#pragma unroll
                for (int m = 0; m < G; ++m) {
                    const int r = r0 + u * NW, h = h0 + 64 * m + lane;
                    v[u][m] = r < nb && h < H ? A.mat[(int64_t)r * H + h] : 0u;
                }
#pragma unroll
            for (int u = 0; u < R; ++u)
#pragma unroll
                for (int m = 0; m < G; ++m) {
                    tot[m] += v[u][m];
                    before[m] += r0 + u * NW < b ? v[u][m] : 0u;
                }
        }
#pragma unroll
        for (int m = 0; m < G; ++m) {
            const int h = h0 + 64 * m + lane;
            if (h < H && tot[m]) atomicAdd(&next[h], tot[m]);
            if (h < H && before[m]) atomicAdd(&pre[h], before[m]);
        }
    }
}

template <bool FIELDS>
__global__ __launch_bounds__(kBktThreads) void k_bkt_scatter(SortArgs A) {
    __shared__ uint32_t next[kBktMax], pre[kBktMax];
    __shared__ __attribute__((aligned(16))) uint32_t dscr[(FIELDS && kSortRuns) ? 8 * kBktThreads : 4];
    __shared__ uint32_t lcnt[(FIELDS && kSortRuns) ? 1 : kBktMax];  // a round's bucket counts, scanned
    __shared__ uint4 stage[(FIELDS && kSortRuns) ? 1 : 4 * kBktThreads];  // a round's records by bucket
    __shared__ uint32_t ws[kBktThreads / 64];
    __shared__ uint32_t rq, rf;
    const int H = A.nbkt, b = blockIdx.x;
    if (threadIdx.x == 0) rq = 0u, rf = 0u;  // the block's largest query length and flags
    const int64_t beg = (int64_t)b * A.chunk;
    const int64_t end = beg + A.chunk < A.n ? beg + A.chunk : A.n;
    constexpr int B = 4;  // reads per thread whose loads are in flight together
    constexpr bool kStaged = !(FIELDS && kSortRuns);
    uint32_t qm = 0, fl = 0;
    const int t = threadIdx.x;
    uint32_t p[B], cb[B], cn[B], sn[B];
    bool in[B];
    auto load_round = [&](int64_t r0) {  // the fields of a round's reads
#pragma unroll
        for (int u = 0; u < B; ++u) {
            const int64_t i = r0 + t + (int64_t)u * kBktThreads;
            in[u] = i < end;
            p[u] = 0u, cb[u] = 0u, cn[u] = 0u, sn[u] = 0u;
            if (in[u]) {
                bool bad;
                p[u] = bkt_pos(A, i, bad);
                fl |= bad ? 2u : 0u;
                cb[u] = A.cig_beg[i];
                cn[u] = A.cig_n[i];
                sn[u] = A.seq_nib[i];
            }
        }
    };
    // bucket h's total and its reads in blocks before b, from the count rows (count_rows)
    for (int h = threadIdx.x; h < H; h += kBktThreads) next[h] = 0u, pre[h] = 0u;
    __syncthreads();
    if (H <= 256)  // (uniform) C3's 234 buckets x 245 rows: every load of a lane in one round trip
        count_rows<4, 16>(A, b, next, pre);
    else
        count_rows<kBktGroup, kBktRows>(A, b, next, pre);
    __syncthreads();
    lds_scan_excl<kBktThreads, kBktMax / kBktThreads>(next, H, ws);
    if (b == 0) {  // every bucket's first slot, for the rank pass
        for (int h = threadIdx.x; h < H; h += kBktThreads) A.bbase[h] = next[h];
        if (threadIdx.x == 0) A.bbase[H] = (uint32_t)A.n;
    }
    for (int h = threadIdx.x; h < H; h += kBktThreads) next[h] += pre[h];
    __syncthreads();
    if constexpr (kStaged) {
        // Rounds of B x kBktThreads reads: each read's record placed in LDS by bucket (the round's
        // counts, scanned), then the block writes the round bucket run by bucket run, neighbouring
        // slots from neighbouring lanes.  (A store per record straight to its slot scattered the
        // 16-byte records over every bucket: 18.5 us at C3.)
        // (the first round's loads issued before the count rows' instead: 19.7 vs 17.1 us)
        for (int64_t r0 = beg; r0 < end; r0 += (int64_t)B * kBktThreads) {
            load_round(r0);
            uint4 rec[B];
            if (FIELDS) {
#pragma unroll
                for (int u = 0; u < B; ++u) rec[u] = make_uint4(p[u], cb[u], sn[u], cn[u]);
            } else {
                uint32_t w[B][8];
#pragma unroll
                for (int u = 0; u < B; ++u)
#pragma unroll
                    for (int k = 0; k < 8; ++k) w[u][k] = (uint32_t)k < cn[u] ? A.cigar[cb[u] + k] : 0u;
#pragma unroll
                for (int u = 0; u < B; ++u) {
                    uint32_t q = 0;  // query length (M/I/=/X)
#pragma unroll
                    for (int k = 0; k < 8; ++k)
                        if (qcons(w[u][k] & 15u)) q += w[u][k] >> 4;
                    for (uint32_t k = 8; k < cn[u]; ++k) {
                        const uint32_t x = A.cigar[cb[u] + k];
                        if (qcons(x & 15u)) q += x >> 4;
                    }
                    qm = (in[u] && q > qm) ? q : qm;
                    // cig_n and the query length packed in 16 bits each; a read that needs more
                    // (only a caller's batch: BAM's n_cigar_op is 16 bits) keeps its source
                    // index for the copy
                    const bool small = cn[u] <= 0xFFFFu && q < kQlenMax;
                    const int64_t i = r0 + t + (int64_t)u * kBktThreads;
                    rec[u] = make_uint4(p[u], cb[u], small ? sn[u] : (uint32_t)i, small ? cn[u] | q << 16 : kBigRec);
                }
            }
            uint32_t bk[B];
            bool inr[B];
#pragma unroll
            for (int u = 0; u < B; ++u) bk[u] = p[u] >> A.wbits, inr[u] = in[u];
            for (int h = t; h < H; h += kBktThreads) lcnt[h] = 0u;
            __syncthreads();
            uint32_t rk[B];
#pragma unroll
            for (int u = 0; u < B; ++u) rk[u] = inr[u] ? atomicAdd(&lcnt[bk[u]], 1u) : 0u;
            __syncthreads();
            lds_scan_excl<kBktThreads, kBktMax / kBktThreads>(lcnt, H, ws);
#pragma unroll
            for (int u = 0; u < B; ++u)
                if (inr[u]) stage[lcnt[bk[u]] + rk[u]] = rec[u];
            __syncthreads();
            const int nr = (int)(end - r0 < (int64_t)B * kBktThreads ? end - r0 : (int64_t)B * kBktThreads);
            for (int i = t; i < nr; i += kBktThreads) {
                const uint4 x = stage[i];
                const uint32_t h = x.x >> A.wbits;
                A.brec[next[h] + (uint32_t)i - lcnt[h]] = x;
            }
            __syncthreads();
            for (int h = t; h < H; h += kBktThreads) next[h] += (h + 1 < H ? lcnt[h + 1] : (uint32_t)nr) - lcnt[h];
            __syncthreads();
        }
    } else {
        for (int64_t i0 = beg + threadIdx.x; i0 < end; i0 += (int64_t)B * kBktThreads) {
            uint32_t p[B], cb[B], cn[B], sn[B];
#pragma unroll
            for (int u = 0; u < B; ++u) {
                const int64_t i = i0 + (int64_t)u * kBktThreads;
                p[u] = 0u, cb[u] = 0u, cn[u] = 0u, sn[u] = 0u;
                if (i < end) {
                    bool bad;
                    p[u] = bkt_pos(A, i, bad);
                    fl |= bad ? 2u : 0u;
                    cb[u] = A.cig_beg[i];
                    cn[u] = A.cig_n[i];
                    sn[u] = A.seq_nib[i];
                }
            }
            uint32_t w[B][8];
#pragma unroll
            for (int u = 0; u < B; ++u)
#pragma unroll
                for (int k = 0; k < 8; ++k) w[u][k] = (uint32_t)k < cn[u] ? A.cigar[cb[u] + k] : 0u;
            // no copy: the record and the read's run record (k_rc then decodes nothing)
            int cm[B];
#pragma unroll
            for (int u = 0; u < B; ++u)  // ops decoded: the wave's longest CIGAR (up to kPre), outside the tail's branch
                cm[u] = (int)(uint32_t)__builtin_amdgcn_readfirstlane(
                    (int)wave_reduce<true>(i0 + (int64_t)u * kBktThreads < end ? (cn[u] < (uint32_t)kPre ? cn[u] : (uint32_t)kPre) : 0u));
#pragma unroll
            for (int u = 0; u < B; ++u) {
                const bool in = i0 + (int64_t)u * kBktThreads < end;
                // decode_fast2 (k_rc's own image decode, ~12 VALU per op; the lane's 8 scratch
                // words in LDS), decode_runs for a wave with a read it declines
                RunTable T;
                const bool ok = in ? decode_fast2(w[u], cn[u], cm[u], dscr + 8 * threadIdx.x, T) : true;
                if (__ballot(!ok) && in) T = decode_runs<2>(w[u], cn[u], cm[u]);
                if (!in) continue;
                uint32_t rr[4];
                pack_runs(T, rr);
                const uint32_t j = atomicAdd(&next[p[u] >> A.wbits], 1u);
                A.brec[j] = make_uint4(p[u], cb[u], sn[u], cn[u]);
                A.brun[j] = make_uint4(rr[0], rr[1], rr[2], rr[3]);
            }
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t y = __shfl_xor(qm, o), f = __shfl_xor(fl, o);
        qm = y > qm ? y : qm;
        fl |= f;
    }
    if ((threadIdx.x & 63) == 0) {
        atomicMax(&rq, qm);
        atomicOr(&rf, fl);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        A.bstat[2 * b] = rq;
        A.bstat[2 * b + 1] = rf;
    }
}

constexpr int kPermSlots = kSortRuns ? 1024 : 4096;  // fields-only rank: sorted slots per LDS pass (16 B each, + 16 B of run)
template <bool FIELDS>
__global__ __launch_bounds__(kRankThreads) void k_bkt_rank(SortArgs A) {
    __shared__ uint32_t cnt[kBktLowMax];
    __shared__ uint4 perm_rec[FIELDS ? kPermSlots : 1], perm_run[(FIELDS && kSortRuns) ? kPermSlots : 1];
    __shared__ uint32_t ws[kRankThreads / 64];
    __shared__ uint32_t rq, rf;
    const int h = blockIdx.x, t = threadIdx.x;
    if (t == 0) rq = 0u, rf = 0u;
    const uint32_t bs = A.bbase[h], be = A.bbase[h + 1];
    const int W = 1 << A.wbits;
    const uint32_t lo_mask = (uint32_t)W - 1u;
    uint4 rec[kRankRegs];  // the bucket's first kRankRegs * kRankThreads records
    uint4 run[FIELDS ? kRankRegs : 1];
#pragma unroll
    for (int k = 0; k < kRankRegs; ++k) {
        const uint32_t r = bs + t + k * kRankThreads;
        rec[k] = r < be ? A.brec[r] : make_uint4(0u, 0u, 0u, 0u);
        if (FIELDS && kSortRuns) run[k] = r < be ? A.brun[r] : make_uint4(0u, 0u, 0u, 0u);
    }
    // the record of sorted slot j: its start-ordered copy (srec), or with FIELDS the sorted
    // batch's own arrays (the sequence stays where it is: seq_nib is the source's)
    auto put = [&](uint32_t j, const uint4& x, const uint4& y) {
        if (FIELDS) {
            A.o_pos[j] = (int32_t)x.x;
            A.o_cig_beg[j] = x.y;
            A.o_seq_nib[j] = x.z;
            A.o_cig_n[j] = x.w;
            if (kSortRuns) A.o_runs[j] = y;
        } else {
            A.srec[j] = x;
        }
    };
    if (h == 0) {  // the batch's largest query length and flags; the copy's zero padding
        uint32_t qm = 0, fl = 0;
        for (int b = t; b < A.nblk; b += kRankThreads) {
            qm = A.bstat[2 * b] > qm ? A.bstat[2 * b] : qm;
            fl |= A.bstat[2 * b + 1];
        }
        for (int o = 32; o > 0; o >>= 1) {
            const uint32_t y = __shfl_xor(qm, o), f = __shfl_xor(fl, o);
            qm = y > qm ? y : qm;
            fl |= f;
        }
        if ((t & 63) == 0) {
            atomicMax(&rq, qm);
            atomicOr(&rf, fl);
        }
        __syncthreads();  // (uniform: h == 0 for the whole block)
        if (t == 0) {
            *A.qmax = rq;
            *A.overflow = rf;  // (bit 1: a bad start; the copy may add bit 0)
            *A.bump = 0u;
        }
        if (!FIELDS) {
            const size_t pad0 = A.room, pad1 = ((size_t)A.room + 15) / 16 * 16 + 16;  // seq_event_bytes(room): zero
            for (size_t at = pad0 + t; at < pad1; at += kRankThreads) A.o_seq[at] = 0;
        }
    }
    for (int k = t; k < W; k += kRankThreads) cnt[k] = 0u;
    __syncthreads();
    const uint32_t more = bs + kRankRegs * kRankThreads;  // records past the registers (large buckets)
#pragma unroll
    for (int k = 0; k < kRankRegs; ++k)
        if (bs + t + k * kRankThreads < be) atomicAdd(&cnt[rec[k].x & lo_mask], 1u);
    for (uint32_t r = more + t; r < be; r += kRankThreads) atomicAdd(&cnt[A.brec[r].x & lo_mask], 1u);
    __syncthreads();
    lds_scan_excl<kRankThreads, kBktLowMax / kRankThreads>(cnt, W, ws);
    if (FIELDS && be - bs <= (uint32_t)(kRankRegs * kRankThreads)) {  // (uniform) the bucket in registers
        // The sorted bucket written through LDS, kPermSlots slots per pass: every record goes to
        // its slot's LDS entry, then the block writes the slots' five arrays with coalesced
        // stores (a direct store per record and array scatters 4-byte words: 35 vs ~12 us at C3)
        uint32_t lr[kRankRegs];
#pragma unroll
        for (int k = 0; k < kRankRegs; ++k)
            lr[k] = bs + t + k * kRankThreads < be ? atomicAdd(&cnt[rec[k].x & lo_mask], 1u) : 0xFFFFFFFFu;
        for (uint32_t p0 = 0; p0 < be - bs; p0 += kPermSlots) {
#pragma unroll
            for (int k = 0; k < kRankRegs; ++k)
                if (lr[k] - p0 < (uint32_t)kPermSlots) {
                    perm_rec[lr[k] - p0] = rec[k];
                    if constexpr (kSortRuns) perm_run[lr[k] - p0] = run[FIELDS ? k : 0];
                }
            __syncthreads();
            for (uint32_t q = t; q < kPermSlots && p0 + q < be - bs; q += kRankThreads)
                put(bs + p0 + q, perm_rec[q], perm_run[kSortRuns ? q : 0]);
            __syncthreads();
        }
        return;
    }
#pragma unroll
    for (int k = 0; k < kRankRegs; ++k)
        if (bs + t + k * kRankThreads < be) put(bs + atomicAdd(&cnt[rec[k].x & lo_mask], 1u), rec[k], run[FIELDS ? k : 0]);
    for (uint32_t r = more + t; r < be; r += kRankThreads) {
        const uint4 x = A.brec[r];
        put(bs + atomicAdd(&cnt[x.x & lo_mask], 1u), x, (FIELDS && kSortRuns) ? A.brun[r] : x);
    }
}

// 4 lanes per sorted slot, R slots per lane group, over every slot (after k_bkt_rank; R = 1):
// the start-ordered records unpacked (a read with 32-bit fields re-read from the source arrays,
// its query length from its CIGAR) and copied by copy_reads
template <int R>
__global__ __launch_bounds__(256) void k_bkt_copy(SortArgs A) {
    const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const uint32_t sub = (uint32_t)g & 3u;
    // a wave's 16 lane groups take 16 R consecutive slots: group q of the wave, step r -> slot
    // base + 16 r + q, so each store instruction writes 16 neighbouring slots
    const int64_t wbase = (g >> 6) * 16 * R, qg = (g & 63) >> 2;
    if (wbase >= A.n) return;
    const uint32_t slot = copy_slot(A, *A.qmax);
    uint32_t pos[R], cb[R], cn[R], sn[R], q[R], jj[R];
    bool ok[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int64_t j = wbase + 16 * r + qg;
        ok[r] = j < A.n;
        jj[r] = (uint32_t)j;
        const uint4 a = ok[r] ? A.srec[j] : make_uint4(0u, 0u, 0u, 0u);
        pos[r] = a.x, cb[r] = a.y, sn[r] = a.z, cn[r] = a.w & 0xFFFFu, q[r] = a.w >> 16;
        if (a.w == kBigRec) {  // (rare: uniform in the lane group)
            const uint32_t i = a.z;
            sn[r] = A.seq_nib[i];
            cn[r] = A.cig_n[i];
            uint32_t qq = 0;
            for (uint32_t k = 0; k < cn[r]; ++k) {
                const uint32_t x = A.cigar[cb[r] + k];
                if (qcons(x & 15u)) qq += x >> 4;
            }
            q[r] = qq;
        }
    }
    copy_reads<R>(A, pos, cb, cn, sn, q, jj, ok, sub, slot);
}

// The bucketed sort's shape: buckets of 2^wbits starts (at most 256 of them, or 4096 of 4096),
// blocks of ~4,096 reads, so that the count rows (blocks x buckets) stay within 65,536 words:
// each scatter block reads them all.  ok = false: the counting sort with global atomics.
struct BktPlan {
    bool ok;
    int wbits, nbkt, nblk;
    int64_t chunk;
};

BktPlan bkt_plan(const bc_reads& r) {
    BktPlan P{};
    const int64_t n = r.n_reads, nbins = r.max_end + 2;
    if (n <= 0 || n >= (int64_t)0xFFFFFFFFll || nbins <= 0) return P;
    int w = 0;
    while (w < 12 && (nbins + (1ll << w) - 1) >> w > kBktTarget) ++w;
    const int64_t H = (nbins + (1ll << w) - 1) >> w;
    if (H > kBktMax) return P;
    P.wbits = w;
    P.nbkt = (int)H;
    const int64_t nblk = std::max<int64_t>(1, std::min<int64_t>((n + kBktChunk - 1) / kBktChunk, 65536 / H));
    P.chunk = (n + nblk - 1) / nblk;
    P.nblk = (int)((n + P.chunk - 1) / P.chunk);
    P.ok = true;
    return P;
}

struct SortLayout {
    size_t bins, rec, o_pos, o_cb, o_cn, o_sn, o_runs, tmp, words, o_seq, o_qual, mat, bstat, bbase, total;
    int64_t nbins;
    uint32_t cap, room;
    BktPlan bkt;
};

// fields: the bucketed sort without the sequence copy (sort_fields_only)
SortLayout sort_layout(const bc_reads& r, bool fields) {
    SortLayout L{};
    const int64_t n = r.n_reads;
    L.bkt = bkt_plan(r);
    fields = fields && L.bkt.ok;
    const int64_t mat_words = L.bkt.ok ? (int64_t)L.bkt.nbkt * L.bkt.nblk : 0;
    L.nbins = r.max_end + 2;  // every start <= max_end
    // every read takes its aligned bases' bytes rounded up to 4 (+ 1 for an odd start); the copy's
    // buffer has half as much again (copy_slot), nibble indices stay below 2^32 (sort_fits)
    L.cap = (uint32_t)std::min<int64_t>(r.seq_bytes + 5 * n + 16, kSortCapMax);
    L.room = (uint32_t)((L.cap + L.cap / 2 + 15) / 16 * 16);
    size_t off = 0;
    auto take = [&](size_t bytes) {
        const size_t at = off;
        off += (bytes + 255) / 256 * 256;
        return at;
    };
    L.words = take(16);  // bump, flags, qmax: first, at the same offset in every layout
    L.bins = L.bkt.ok ? 0 : take(4 * (size_t)L.nbins);
    L.rec = take(32 * (size_t)n);
    L.o_pos = take(4 * (size_t)n);
    L.o_cb = take(4 * (size_t)n);
    L.o_cn = take(4 * (size_t)n);
    L.o_sn = take(4 * (size_t)n);
    L.o_runs = fields ? take(16 * (size_t)n) : 0;
    L.tmp = L.bkt.ok ? 0 : take(4 * scan_tmp_words(L.nbins));
    L.o_seq = fields ? 0 : take(seq_event_bytes(L.room));
    L.o_qual = (r.qual && !fields) ? take(2 * (size_t)L.room + 32) : 0;
    L.mat = take(4 * (size_t)mat_words);
    L.bstat = take(8 * (size_t)(L.bkt.ok ? L.bkt.nblk : 0));
    L.bbase = take(4 * (size_t)(L.bkt.ok ? L.bkt.nbkt + 1 : 0));
    L.total = off;
    return L;
}

}  // namespace

size_t sort_bytes(const bc_reads& r, bool fields) {
    if (r.n_reads <= 0) return 0;
    return sort_layout(r, fields).total;
}

bool sort_fits(const bc_reads& r) { return r.seq_bytes + 5 * r.n_reads + 16 <= kSortCapMax; }

hipError_t launch_sort(hipStream_t s, const bc_reads& r, bc_reads& out, void* mem, bool fields) {
    const SortLayout L = sort_layout(r, fields);
    fields = fields && L.bkt.ok;
    uint8_t* b = (uint8_t*)mem;
    SortArgs A{};
    A.pos = r.pos;
    A.cig_beg = r.cig_beg;
    A.cig_n = r.cig_n;
    A.seq_nib = r.seq_nib;
    A.cigar = r.cigar;
    A.seq = r.seq;
    A.qual = r.qual;
    A.n = r.n_reads;
    A.rec = (uint4*)(b + L.rec);
    A.o_pos = (int32_t*)(b + L.o_pos);
    A.o_cig_beg = (uint32_t*)(b + L.o_cb);
    A.o_cig_n = (uint32_t*)(b + L.o_cn);
    A.o_seq_nib = (uint32_t*)(b + L.o_sn);
    A.bump = (uint32_t*)(b + L.words);
    A.overflow = A.bump + 1;
    A.qmax = A.bump + 2;
    A.o_seq = b + L.o_seq;
    A.o_qual = r.qual ? b + L.o_qual : nullptr;
    A.cap = L.cap;
    A.room = L.room;
    A.qual_bytes = r.qual ? r.qual_bytes : 0;
    A.nbins = L.nbins;
    const unsigned blocks = (unsigned)((r.n_reads + 255) / 256);
    hipError_t e = hipSuccess;
    if (L.bkt.ok) {
        A.mat = (uint32_t*)(b + L.mat);
        A.bstat = (uint32_t*)(b + L.bstat);
        A.bbase = (uint32_t*)(b + L.bbase);
        A.brec = A.rec;
        A.srec = A.rec + r.n_reads;
        A.chunk = L.bkt.chunk;
        A.nblk = L.bkt.nblk;
        A.nbkt = L.bkt.nbkt;
        A.wbits = L.bkt.wbits;
        hipLaunchKernelGGL(k_bkt_count, dim3((unsigned)A.nblk), dim3(kBktThreads), 0, s, A);
        if (fields) {  // the sorted fields and run records; the sequence stays where it is
            A.brun = A.rec + r.n_reads;
            A.o_runs = (uint4*)(b + L.o_runs);
            hipLaunchKernelGGL(k_bkt_scatter<true>, dim3((unsigned)A.nblk), dim3(kBktThreads), 0, s, A);
            hipLaunchKernelGGL(k_bkt_rank<true>, dim3((unsigned)A.nbkt), dim3(kRankThreads), 0, s, A);
        } else {
            hipLaunchKernelGGL(k_bkt_scatter<false>, dim3((unsigned)A.nblk), dim3(kBktThreads), 0, s, A);
            hipLaunchKernelGGL(k_bkt_rank<false>, dim3((unsigned)A.nbkt), dim3(kRankThreads), 0, s, A);
            // one slot per lane group (a wave: 16 slots): 93 us against 95 / 98 / 101 at 2 / 4 / 8
            const int64_t waves = (r.n_reads + 15) / 16;
            hipLaunchKernelGGL(k_bkt_copy<1>, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, s, A);
        }
    } else {  // more than 2^24 starts: the counting sort with one global atomic per read
        A.bins = (uint32_t*)(b + L.bins);
        uint32_t* tmp = (uint32_t*)(b + L.tmp);
        e = hipMemsetAsync(A.bins, 0, 4 * (size_t)L.nbins, s);
        if (e == hipSuccess) e = hipMemsetAsync(A.bump, 0, 16, s);  // bump, flags, qmax
        // the sorted sequence's padding past room (BC_SEQ_EVENT) is zero
        if (e == hipSuccess) e = hipMemsetAsync(A.o_seq + L.room, 0, seq_event_bytes(L.room) - L.room, s);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(k_sort_count, dim3(blocks), dim3(256), 0, s, A);
        if ((e = scan_u32(s, A.bins, L.nbins, tmp, nullptr)) != hipSuccess) return e;
        const int64_t groups = (r.n_reads + kRelayReads - 1) / kRelayReads;
        hipLaunchKernelGGL(k_sort_relay, dim3((unsigned)((groups * 4 + 255) / 256)), dim3(256), 0, s, A);
    }
    if ((e = hipGetLastError()) != hipSuccess) return e;
    out = r;
    if (fields) {  // the source's sequence, CIGARs and (no) qualities; run records, no summaries
        out.pos = A.o_pos;
        out.cig_beg = A.o_cig_beg;
        out.cig_n = A.o_cig_n;
        out.seq_nib = A.o_seq_nib;
        out.sorted = 1;
        out.seq_layout = BC_SEQ_EVENT;
        out.read_runs = kSortRuns ? (const uint32_t*)A.o_runs : nullptr;
        out.run_chunks = 0;
        out.tile_reads = nullptr;
        out.n_tiles = 0;
        out.index_tag = kSortRuns ? index_tag(out) : 0;
        return hipSuccess;
    }
    out.pos = A.o_pos;
    out.cig_beg = A.o_cig_beg;
    out.cig_n = A.o_cig_n;
    out.seq_nib = A.o_seq_nib;
    out.seq = A.o_seq;
    out.seq_bytes = L.room;
    out.qual = A.o_qual;
    out.qual_bytes = r.qual ? 2 * (int64_t)L.room : 0;
    out.sorted = 1;
    out.seq_layout = BC_SEQ_EVENT;
    out.read_runs = nullptr;
    out.run_chunks = 0;
    out.tile_reads = nullptr;
    out.n_tiles = 0;
    out.index_tag = 0;
    return hipSuccess;
}

const uint32_t* sort_flags_word(const bc_reads& r, const void* mem) {
    return (const uint32_t*)((const uint8_t*)mem + sort_layout(r, false).words) + 1;  // (offset 0 in every layout)
}

}  // namespace bc
