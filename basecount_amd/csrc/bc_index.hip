// bc_index.hip — the device index of a coordinate-sorted batch (bc_reads.read_runs, run_chunks,
// tile_reads), built on the device from the batch itself: pos[], the CIGAR words and seq_nib[].
//
// The index holds nothing the reference computes: it is the CIGAR walk of count.cpp:40-96 done
// ahead of the kernels, in the layout they consume.
//   * run records (16 B per read, bc_runs.h: pack_runs): each read's CIGAR decoded once by the
//     kernels' own decode_runs, so the read-chunked k_rc loads a record instead of decoding on
//     its chunk's critical path;
//   * chunk summaries (8 words per 256-read k_rc chunk, bc_runs.h: chunk order of run_shape /
//     full_span): the bounds a k_rc block would otherwise reduce at the start of each chunk;
//   * the tile index (2 x int32 per 64-position tile): the reads [lo, hi) that can overlap tile t,
//     which the tiled k_pileup would otherwise search for.
// One launch per part, each a plain streaming pass with full parallelism (a block per 256-read
// chunk, a thread per tile), stream-ordered and capturable: no allocation, no synchronisation.
#include "bc_internal.h"

namespace bc {
namespace {

#include "bc_walk.h"

constexpr int kCigStage = 2048;  // CIGAR words a k_index_runs block stages (8 KiB: 8 per read)

struct IdxArgs {
    const int32_t* pos;
    const uint32_t* cig_beg;
    const uint32_t* cig_n;
    const uint32_t* seq_nib;
    const uint32_t* cigar;
    int64_t n;
    uint4* runs;  // [n] records
    uint4* sums;  // [2 * n_chunks] chunk summaries, or NULL
};

// One 256-thread block per k_rc chunk: thread t decodes read chunk * 256 + t into its record,
// then the block reduces the chunk's summary (the same values bc_capi.hip's host chunk_summary
// computed from the records: complex reads contribute only their full span to the bounds).
__global__ __launch_bounds__(kRcChunkReads) void k_index_runs(IdxArgs A) {
    constexpr int NT = kRcChunkReads, NW = NT / 64;
    __shared__ __attribute__((aligned(16))) uint32_t red[NW][8];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t i = (int64_t)blockIdx.x * NT + tid;
    const bool valid = i < A.n;
    __shared__ uint32_t cig[kCigStage];
    __shared__ uint32_t seg[2];
    uint32_t pos = 0, cb = 0, cn = 0, sn = 0;
    if (valid) {
        pos = (uint32_t)A.pos[i];
        cb = A.cig_beg[i];
        cn = A.cig_n[i];
        sn = A.seq_nib[i];
    }
    // The chunk's CIGAR words usually lie in one contiguous segment (reads in file order): it is
    // staged with coalesced loads, each thread then reads its words from LDS (per-thread loads of
    // scattered 4-byte words cost ~10 cache lines per wave instruction, eight times over)
    const int64_t last = ((int64_t)blockIdx.x + 1) * NT < A.n ? ((int64_t)blockIdx.x + 1) * NT - 1 : A.n - 1;
    if (tid == 0) seg[0] = cb;
    if (i == last) seg[1] = cb + (cn < (uint32_t)kPre ? cn : (uint32_t)kPre);
    __syncthreads();
    const uint32_t s0 = seg[0], s1 = seg[1];
    const bool staged = s1 >= s0 && s1 - s0 <= (uint32_t)kCigStage;
    if (staged)
        for (uint32_t k = tid; k < s1 - s0; k += NT) cig[k] = A.cigar[s0 + k];
    __syncthreads();
    const bool mine_in = staged && cb >= s0 && cb + (cn < (uint32_t)kPre ? cn : (uint32_t)kPre) <= s1;
    uint32_t w[kPre];
#pragma unroll
    for (int k = 0; k < kPre; ++k)
        w[k] = (valid && (uint32_t)k < cn) ? (mine_in ? cig[cb - s0 + k] : A.cigar[cb + k]) : 0u;
    // ops decoded: the wave's longest CIGAR (up to kPre; the decode's per-op select chain is
    // the kernel's VALU cost, and most waves' reads have far fewer ops)
    const int cmax = (int)(uint32_t)__builtin_amdgcn_readfirstlane(
        (int)wave_reduce<true>(valid ? (cn < (uint32_t)kPre ? cn : (uint32_t)kPre) : 0u));
    uint32_t q[4];
    pack_runs(decode_runs<2>(w, cn, cmax), q);
    if (valid) A.runs[i] = make_uint4(q[0], q[1], q[2], q[3]);
    if (!A.sums) return;  // (uniform)
    // the summary from the record, as the kernel will read it (pack_runs may mark a read complex)
    const RunTable T = unpack_runs(q[0], q[1], q[2], q[3]);
    const bool simple = valid && !T.complex;
    const uint32_t span = (valid && T.complex) ? full_span(A.cigar + cb, cn) : T.span;
    uint32_t v[7];
    v[0] = valid ? pos : 0xFFFFFFFFu;
    v[1] = valid ? pos + span : 0u;
    v[2] = (simple && T.qlen) ? (sn >> 1) : 0xFFFFFFFFu;
    v[3] = (simple && T.qlen) ? ((sn + T.qlen + 1) >> 1) : 0u;
    v[4] = simple ? T.span : 0u;
    v[5] = simple ? run_shape(T) : 0u;
    v[6] = (simple && T.gap) ? 1u : 0u;
    constexpr bool is_max[7] = {false, true, false, true, true, true, true};
    uint32_t mine = 0;
#pragma unroll
    for (int k = 0; k < 7; ++k) {
        const uint32_t r = is_max[k] ? wave_reduce<true>(v[k]) : wave_reduce<false>(v[k]);
        mine = lane == k ? r : mine;
    }
    if (lane < 8) red[wave][lane] = lane < 7 ? mine : 0u;
    __syncthreads();
    if (tid < 8) {
        uint32_t r = red[0][tid];
#pragma unroll
        for (int q2 = 1; q2 < NW; ++q2) {
            const uint32_t o = red[q2][tid];
            r = (tid == 0 || tid == 2) ? (o < r ? o : r) : (o > r ? o : r);
        }
        ((uint32_t*)A.sums)[(size_t)blockIdx.x * 8 + tid] = r;
    }
}

// floor(x / 64) for any sign
__device__ __forceinline__ int64_t fdiv64(int64_t x) { return x >> 6; }

// Thread per read i (and one past the last): the tiles whose range starts or ends at read i.
// With v increasing in t, "first i with pos[i] >= v(t)" is read i exactly for the t with
// pos[i-1] < v(t) <= pos[i] (pos[-1] = -inf, pos[n] = +inf), so every tile entry is written by
// one thread, and no thread searches:
//   lo: v(t) = 64t - max_span + 1  ->  t in (fdiv64(pos[i-1] + max_span - 1), fdiv64(pos[i] + max_span - 1)]
//   hi: v(t) = 64t + 64            ->  t in [fdiv64(pos[i-1]), fdiv64(pos[i]) - 1]
__global__ __launch_bounds__(256) void k_index_tiles(const int32_t* pos, int64_t n, int64_t tiles, int64_t max_span,
                                                     int32_t* out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i > n) return;
    const bool first = i == 0, last = i == n;
    const int64_t p1 = last ? 0 : (int64_t)pos[i], p0 = first ? 0 : (int64_t)pos[i - 1];
    int64_t a = first ? 0 : fdiv64(p0 + max_span - 1) + 1;
    int64_t b = last ? tiles - 1 : fdiv64(p1 + max_span - 1);
    a = a < 0 ? 0 : a;
    b = b > tiles - 1 ? tiles - 1 : b;
    for (int64_t t = a; t <= b; ++t) out[2 * t] = (int32_t)i;
    a = first ? 0 : fdiv64(p0);
    b = last ? tiles - 1 : fdiv64(p1) - 1;
    a = a < 0 ? 0 : a;
    b = b > tiles - 1 ? tiles - 1 : b;
    for (int64_t t = a; t <= b; ++t) out[2 * t + 1] = (int32_t)i;
}

}  // namespace

IndexPlan index_plan(const bc_reads& r, int what) {
    IndexPlan p{};
    const int64_t n = r.n_reads;
    if (!r.sorted || n <= 0) return p;
    if (what & BC_INDEX_RUNS) {
        p.runs_bytes = (size_t)n * 16;
        p.n_chunks = (n + kRcChunkReads - 1) / kRcChunkReads;
        if (p.n_chunks < (int64_t)0x7FFFFFFF) p.sums_bytes = (size_t)p.n_chunks * 32;
    }
    const int64_t tiles = (r.max_end + 63) / 64;
    if ((what & BC_INDEX_TILES) && n < (int64_t)0x7FFFFFC0 && tiles > 0 && tiles <= n / 16) {
        p.n_tiles = tiles;
        p.tiles_bytes = (size_t)tiles * 8;
    }
    p.total = (p.runs_bytes + p.sums_bytes + 15) / 16 * 16 + p.tiles_bytes;
    return p;
}

hipError_t launch_index(hipStream_t s, bc_reads& r, const IndexPlan& p, void* mem) {
    uint8_t* base = (uint8_t*)mem;
    r.read_runs = nullptr;
    r.run_chunks = 0;
    r.tile_reads = nullptr;
    r.n_tiles = 0;
    if (p.runs_bytes) {
        IdxArgs A;
        A.pos = r.pos;
        A.cig_beg = r.cig_beg;
        A.cig_n = r.cig_n;
        A.seq_nib = r.seq_nib;
        A.cigar = r.cigar;
        A.n = r.n_reads;
        A.runs = (uint4*)base;
        A.sums = p.sums_bytes ? (uint4*)(base + p.runs_bytes) : nullptr;
        hipLaunchKernelGGL(k_index_runs, dim3((unsigned)p.n_chunks), dim3(kRcChunkReads), 0, s, A);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        r.read_runs = (const uint32_t*)base;
        r.run_chunks = p.sums_bytes ? (int32_t)p.n_chunks : 0;
    }
    if (p.tiles_bytes) {
        int32_t* out = (int32_t*)(base + (p.runs_bytes + p.sums_bytes + 15) / 16 * 16);
        const int64_t blocks = (r.n_reads + 1 + 255) / 256;
        hipLaunchKernelGGL(k_index_tiles, dim3((unsigned)blocks), dim3(256), 0, s, r.pos, r.n_reads, p.n_tiles,
                           (int64_t)r.max_span, out);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        r.tile_reads = out;
        r.n_tiles = p.n_tiles;
    }
    r.index_tag = index_tag(r);
    return hipSuccess;
}

}  // namespace bc
