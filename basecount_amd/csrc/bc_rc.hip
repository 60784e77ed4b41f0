// bc_rc.hip — read-chunked kernel 1 for deep, coordinate-sorted batches (count.cpp:22-97).
//
// The position-tiled k_pileup decodes and stages every read once per 64-position tile it
// overlaps (~(span + 63) / 64 times: 3.3x for 150 bp reads).  At high depth that repeated setup
// and its HBM traffic dominate.  Here a 256-thread block takes 256 CONSECUTIVE reads of the
// sorted batch (a chunk), so each read is loaded, CIGAR-decoded and staged exactly once:
//
//   1. thread i: read c0 + i -> its CIGAR's first two runs (decode_fast2, or the upload's run
//      records) ; the chunk's packed sequence (BC_SEQ_EVENT, bases below min_base_quality
//      cleared) is staged into LDS (one segment by LDS-DMA, or per-read slots: gather staging);
//   2. event image (chunks of reads with <= 2 runs): thread i writes its read's 8-position window
//      words into column i of an LDS image [read][row]; the transposed sum counts each row's 32
//      reads bit-sliced (carry-save trees + an 8x8 bit transpose) into per-position class counts;
//      other chunks walk run tables: (window, 64-read slice) items over the 4 waves, SWAR nibble
//      counters folded by DPP into an LDS histogram;
//   3. the chunk's counts are flushed into the int32 counts with coalesced global atomics (a
//      position receives one add per chunk overlapping it), an image chunk's by wave 3 during
//      the next chunk's sum.
//
// Reads with more than 8 CIGAR ops / 4 runs / huge spans are walked separately with global
// atomics.  Counted events at positions >= L are the reference's std::out_of_range
// (count.cpp:60-65,85): the first offending read index is kept (atomicMin), nothing is counted
// there.  Kernel 2 (k_stats) runs afterwards on the counts.
#include <cstdio>
#include <cstring>
#include <type_traits>

#include "bc_internal.h"

namespace bc {
namespace {

// Chunk geometry: NT threads = NT reads per chunk (one per thread at setup), 78 staged sequence
// bytes per read (150 bp reads fit with room).  Bigger chunks amortize the per-chunk setup
// (barriers, reductions, window tables, flush atomics) and give every window more 64-read
// slices, so a wave folds its counters less often.
template <int NT>
struct RcGeo {
    static constexpr int kThreads = NT;
    static constexpr int kReads = NT;
    static constexpr int kStage = 78 * NT;
    static constexpr int kWaves = NT / 64;
};
constexpr int kRcChunk = 256;
constexpr int kImgRows = 23;  // windows an imaged chunk may cover (odd: the image's read stride)
constexpr int kPadW = 24;     // stage pad words on each side (kImgRows + 1, see the image expansion)
constexpr uint32_t kSpecSlack = 128;  // bytes staged beyond the last read's first base
#include "bc_walk.h"
static_assert(kRcChunk == kRcChunkReads, "the upload summarises chunks of k_rc's size (bc_runs.h)");

// the image's CIGAR decode by decode_fast2 (bc_runs.h); -DBC_FAST_DECODE=0 builds the A/B variant
// that decodes every chunk with decode_runs
#ifndef BC_FAST_DECODE
#define BC_FAST_DECODE 1
#endif
constexpr bool kFastDecode = BC_FAST_DECODE != 0;
// s_waitcnt vmcnt(0) with expcnt / lgkmcnt left at their maxima (gfx9 encoding: vmcnt [3:0] and
// [15:14], expcnt [6:4], lgkmcnt [11:8]); as a builtin the compiler's waitcnt pass sees it
constexpr int kWaitVm0 = 0x0F70;
#ifndef BC_RC_EARLY_WAIT
#define BC_RC_EARLY_WAIT 1
#endif
constexpr bool kEarlyWait = BC_RC_EARLY_WAIT != 0;
// gather staging of chunks whose sequence is not one short segment (see `gather`); -DBC_RC_GATHER=0
// builds the variant that walks such chunks from HBM
#ifndef BC_RC_GATHER
#define BC_RC_GATHER 1
#endif
constexpr bool kGather = BC_RC_GATHER != 0;
// Gather staging (chunks whose sequence is not one short segment: the reads of a batch sorted on
// the device without moving its sequence, bc_sort.hip's fields-only sort): every simple read's
// bytes, from the 4-byte word holding its first base, into its own kRcSlot-byte slot of the
// stage by LDS-DMA.  The block's threads move the slots' words in stage order (instruction e of
// wave w: stage words (20 w + e) * 64 + lane, ~3 reads' consecutive words), so an instruction
// touches a handful of cache lines; one lane per read (each instruction 64 reads' lines) took
// 122 us at C3 in random order, the register copy before it 220.
constexpr int kRcSlot = 80;  // 20 words: a read of <= 77 bytes at any byte offset in its first word
static_assert(kRcSlot == 80, "stage word -> slot by multiply-shift: (g * 3277) >> 16 == g / 20 for g < 5120");
constexpr int kGStage = kRcSlot * kRcChunk;
constexpr int kRcWinPos = 512;             // positions of the LDS histogram (one window pass)
constexpr int kRcWin = kRcWinPos / 8;      // 8-position windows per pass

// Diagnostic phase totals (-DBC_PHASE_TRACE): per wave, cycles spent in each chunk phase,
// summed over its chunks (s_memtime), written once at the end.  Costs registers.
#ifdef BC_PHASE_TRACE
#define RC_STAMP(ph)                                                                 \
    do {                                                                             \
        const uint64_t now_ = __builtin_amdgcn_s_memtime();                          \
        if ((ph) > 0) tsum[(ph) - 1] += now_ - tlast;                                \
        tlast = now_;                                                                \
    } while (0)
#else
#define RC_STAMP(ph) \
    do {             \
    } while (0)
#endif
[[maybe_unused]] constexpr int kRcPhases = 7;

// k << (m mod 64): v_lshlrev_b64 reads only the low 6 bits of the shift (C's << may not)
__device__ __forceinline__ unsigned long long shl64_mod64(unsigned long long k, int m) {
    unsigned long long r;
    asm("v_lshlrev_b64 %0, %1, %2" : "=v"(r) : "v"(m), "s"(k));
    return r;
}

// X >> n as ONE v_lshrrev_b64 (the compiler splits a 64-bit shift into two 32-bit funnel ops)
template <int N>
__device__ __forceinline__ unsigned long long shr64(unsigned long long x) {
    unsigned long long r;
    asm("v_lshrrev_b64 %0, %1, %2" : "=v"(r) : "i"(N), "v"(x));
    return r;
}

// ---- bit-sliced counting (the event image's transposed sum) ----------------------------------
// A full adder over 32 bit positions at once: s = a ^ b ^ c, k = maj(a, b, c) (one v_bitop3 each)
__device__ __forceinline__ void fadd(uint32_t& s, uint32_t& k, uint32_t a, uint32_t b, uint32_t c) {
    s = __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
    k = __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);
}
// Harley-Seal carry-save tree over 16 words: adds their bits into the bit-sliced digits d[0..3]
// (weights 1, 2, 4, 8) and returns the carry word of weight 16 (15 full adders, 30 VALU).
__device__ __forceinline__ uint32_t csa16(uint32_t* d, const uint32_t* x) {
    uint32_t tA, tB, fA, fB, eA, eB, s16;
    fadd(d[0], tA, d[0], x[0], x[1]);
    fadd(d[0], tB, d[0], x[2], x[3]);
    fadd(d[1], fA, d[1], tA, tB);
    fadd(d[0], tA, d[0], x[4], x[5]);
    fadd(d[0], tB, d[0], x[6], x[7]);
    fadd(d[1], fB, d[1], tA, tB);
    fadd(d[2], eA, d[2], fA, fB);
    fadd(d[0], tA, d[0], x[8], x[9]);
    fadd(d[0], tB, d[0], x[10], x[11]);
    fadd(d[1], fA, d[1], tA, tB);
    fadd(d[0], tA, d[0], x[12], x[13]);
    fadd(d[0], tB, d[0], x[14], x[15]);
    fadd(d[1], fB, d[1], tA, tB);
    fadd(d[2], eB, d[2], fA, fB);
    fadd(d[3], s16, d[3], eA, eB);
    return s16;
}
// In-register transpose of 8 x (4 blocks of 8 x 8 bits): afterwards byte i of r[k] holds, in bit d,
// bit 8i + k of the input r[d] (three rounds of block swaps, two v_bfi_b32 and two shifts each).
// With bit-sliced digits r[d] this turns the 32 bit positions' counts into bytes.
__device__ __forceinline__ void bit_transpose8(uint32_t (&r)[8]) {
    auto swap = [&](int a, int b, int s, uint32_t m) {  // r[a] bits (k + s) <-> r[b] bits k, k in m
        const uint32_t ra = r[a], rb = r[b];
        // bitop3 0xCA = bit select (m ? x : y), kept as written (the compiler's own form of the
        // selects took ~2x the instructions)
        r[b] = __builtin_amdgcn_bitop3_b32(m, ra >> s, rb, 0xCA);
        r[a] = __builtin_amdgcn_bitop3_b32(m << s, rb << s, ra, 0xCA);
    };
#pragma unroll
    for (int d = 0; d < 4; ++d) swap(d, d + 4, 4, 0x0F0F0F0Fu);
#pragma unroll
    for (int d = 0; d < 8; d += 4) {
        swap(d, d + 2, 2, 0x33333333u);
        swap(d + 1, d + 3, 2, 0x33333333u);
    }
#pragma unroll
    for (int d = 0; d < 8; d += 2) swap(d, d + 1, 1, 0x55555555u);
}

// &base[i]; with a 32-bit index type as a 32-bit BYTE offset from the (uniform) base, so loads
// and atomics address as SGPR base + 32-bit VGPR offset (no 64-bit address arithmetic per lane)
template <typename IT, typename T>
__device__ __forceinline__ T* elem(T* base, IT i) {
    if constexpr (sizeof(IT) == 4) {
        using B = typename std::conditional<std::is_const<T>::value, const char, char>::type;
        return (T*)((B*)base + (uint32_t)i * (uint32_t)sizeof(T));
    } else {
        return base + i;
    }
}

// A 32-bit word at a wave-uniform address, by a scalar load (constant address space): no vector
// memory instruction, no readfirstlane, and counted in lgkmcnt, so waiting for it does not wait for
// the stage copy queued before it (vmcnt is in order).  Read-only data only (scalar cache).
__device__ __forceinline__ uint32_t sload(const uint32_t* p) {
    return *(const __attribute__((address_space(4))) uint32_t*)p;
}

struct RcArgs {
    const int32_t* pos;
    const uint32_t* cig_beg;
    const uint32_t* cig_n;
    const uint32_t* seq_nib;
    const uint32_t* cigar;
    const uint8_t* seq;
    const uint8_t* qual;
    int64_t n;
    int64_t L;
    uint32_t mbq;
    int64_t seq_words;
    int64_t qual_bytes;
    int64_t n_chunks;
    int32_t chunk_reads;  // reads per chunk (<= the block's threads; the last chunk may hold fewer)
    const uint4* runs;  // bc_reads.read_runs (run records, bc_runs.h) or NULL: decode the CIGARs
    const uint4* sums;  // the upload's chunk summaries (2 x uint4 per chunk, after the records) or NULL
    int32_t* counts;  // [ncols][L], accumulated into
    unsigned long long* err;
    int ablate;  // diagnostic only (BC_ABLATE): 4 no walk, 128 no folds, 256 trivial item events,
                 // 512 no staging, 2048 no flush, 8192 no event image, 16384 no image expansion,
                 // 65536 no boundary rows in the image expansion, 32768 no CIGAR load / decode,
                 // 131072 decode a fixed CIGAR (no CIGAR words waited for), 262144 no CIGAR prefetch
    unsigned long long* trace;  // diagnostic only (BC_PHASE_TRACE builds): [block][wave][kRcPhases]
};

// Block-wide reduction of NV <= 8 values (max or min per slot): wave reduce, then LDS across
// waves.  Lane k of each wave stores slot k (one masked store, not one per slot); every thread
// then reads the waves' rows as 16-byte words.  Must be called by the whole block.
// wave_partials (each wave's results into its row of red) + a barrier + block_combine (every thread
// folds the rows).
template <int NV>
__device__ __forceinline__ void wave_partials(const uint32_t (&v)[NV], const bool (&is_max)[NV], uint32_t (*red)[8]) {
    static_assert(NV <= 8, "one 8-word row per wave");
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint32_t mine = 0;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        const uint32_t r = is_max[k] ? wave_reduce<true>(v[k]) : wave_reduce<false>(v[k]);
        mine = lane == k ? r : mine;
    }
    if (lane < NV) red[wave][lane] = mine;
}
template <int NV, int NWAVES>
__device__ __forceinline__ void block_combine(uint32_t (&v)[NV], const bool (&is_max)[NV], uint32_t (*red)[8]) {
    uint32_t w[NWAVES][8];
#pragma unroll
    for (int q = 0; q < NWAVES; ++q) {
        const uint4 a = *(const uint4*)&red[q][0], b = *(const uint4*)&red[q][4];
        w[q][0] = a.x, w[q][1] = a.y, w[q][2] = a.z, w[q][3] = a.w;
        w[q][4] = b.x, w[q][5] = b.y, w[q][6] = b.z, w[q][7] = b.w;
    }
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        uint32_t r = w[0][k];
#pragma unroll
        for (int q = 1; q < NWAVES; ++q) r = is_max[k] ? (w[q][k] > r ? w[q][k] : r) : (w[q][k] < r ? w[q][k] : r);
        v[k] = r;
    }
}
template <int NV, int NWAVES>
__device__ __forceinline__ void block_reduce(uint32_t (&v)[NV], const bool (&is_max)[NV], uint32_t (*red)[8]) {
    wave_partials<NV>(v, is_max, red);
    __syncthreads();
    block_combine<NV, NWAVES>(v, is_max, red);
}

// Fold a wave's window counters into the LDS histogram: 8-slot sums per lane group (DPP), then
// each lane adds its own window position (s = lane & 7) for every column.
template <int NC>
__device__ __forceinline__ void rc_fold(Swar& W, uint32_t (*hist)[kRcWinPos], int g, int s8, int ablate = 0) {
    if (ablate & 128) return;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const uint32_t b0 = sum8(W.a4[c] & 0x0F0F0F0Fu), b1 = sum8((W.a4[c] >> 4) & 0x0F0F0F0Fu);
        const uint32_t v = (((s8 & 1) ? b1 : b0) >> (8 * (s8 >> 1))) & 0xFFu;
        if (v) atomicAdd(&hist[c >> 1][8 * g + s8], v << (16 * (c & 1)));
        W.a4[c] = 0;
    }
}

// A complex read (more than kPre CIGAR ops, more than 4 runs, or a huge span) walked by the
// whole wave, 64 consecutive reference offsets per step, straight into the global counts.
template <bool QUAL, int NC>
__device__ void rc_complex(const RcArgs& A, int64_t r, int64_t& bad) {
    const int lane = threadIdx.x & 63;
    const int64_t p0 = A.pos[r];
    const uint32_t* cg = A.cigar + A.cig_beg[r];
    const uint32_t cn = A.cig_n[r], sn = A.seq_nib[r];
    uint64_t span = 0;
    for (uint32_t k = 0; k < cn; ++k)
        if (mlike(cg[k] & 15u) || dlike(cg[k] & 15u)) span += cg[k] >> 4;
    for (uint64_t e0 = 0; e0 < span; e0 += 64) {
        const uint64_t j = e0 + lane;
        uint32_t e = kNone;
        uint64_t rc = 0, qc = 0;
        for (uint32_t k = 0; k < cn && rc < e0 + 64; ++k) {
            const uint32_t op = cg[k] & 15u, len = cg[k] >> 4;
            if (mlike(op) || dlike(op)) {
                if (j >= rc && j < rc + len) e = mlike(op) ? (uint32_t)(sn + qc + (j - rc)) : kDel;
                rc += len;
            }
            if (qcons(op)) qc += len;
        }
        if (e == kNone) continue;
        unsigned col = 4;
        bool ok = true;
        if (e != kDel) {
            col = nib_col6((A.seq[e >> 1] >> ((e & 1u) * 4)) & 15u);
            ok = col != 6u;
            if (QUAL) ok = ok && (uint32_t)A.qual[e] >= A.mbq;
        }
        if (!ok) continue;
        const int64_t p = p0 + (int64_t)j;
        if (p >= A.L) {
            if (r < bad) bad = r;
        } else if ((int)col < NC) {
            atomicAdd(&A.counts[(int64_t)col * A.L + p], 1);
        }
    }
}

// IT: the type of read indices and positions (int32_t when the batch and the reference are small
// enough, see launch_rc: uniform arithmetic then stays on the scalar unit)
template <bool QUAL, int NC, int NT, typename IT>
__global__ __launch_bounds__(NT, 3) void k_rc(RcArgs A) {
    using Geo = RcGeo<NT>;
    constexpr int kRcThreads = Geo::kThreads, kRcReads = Geo::kReads, kStage = Geo::kStage, kRcWaves = Geo::kWaves;
    // records (48 B per read) of the run-table walk, or, on the image path, the chunk's event
    // image: BC_SEQ_EVENT words [read][window row], kImgRows (odd) words per read, so that both
    // the expansion (lanes = reads, one row) and the accumulation (lanes = rows, one read) hit
    // 64 different LDS banks
    constexpr int kRecU4 = kRcReads * 3, kImgU4 = kImgRows * kRcReads / 4;
    // the image's 32-read groups are R words apart beyond their 736 (R = the chunk's rows, <= 23),
    // so the sum's lanes (row t mod R of group t / R) read 32 consecutive banks
    constexpr int kImgPadU4 = (7 * kImgRows + 3) / 4;
    constexpr int kRecAll = kRecU4 + kRcReads / 4;  // records + the read positions (run-table chunks)
    __shared__ uint4 rec[kRecAll > kImgU4 + kImgPadU4 ? kRecAll : kImgU4 + kImgPadU4];
    uint32_t* img = (uint32_t*)rec;
    // the chunk's read positions (window tables of the run-table walk), past its records: the
    // image path, which overwrites both, uses neither (1 KiB of LDS kept for the gather stage:
    // a 512-byte larger block no longer fits three times into a CU, k_rc 46 -> 71 us at C3)
    int32_t* const rpos = (int32_t*)(rec + kRecU4);
    // (the gather stage's slots reach kGStage bytes; both layouts keep kPadW words of pad after)
    __shared__ __attribute__((aligned(16))) uint8_t stage_raw[(kStage > kGStage ? kStage : kGStage) + 8 * kPadW];  // + pads
    __shared__ uint32_t hist[3][kRcWinPos];                              // {A|C, G|T, DS|N}
    __shared__ __attribute__((aligned(16))) uint32_t red[kRcWaves][8];
    __shared__ uint32_t wlo[kRcWin], whi[kRcWin], wpre[kRcWin + 1];
    __shared__ uint32_t cxl[kRcReads];
    __shared__ uint32_t ncx[2];  // complex reads of the chunk (by chunk parity: no barrier to reset)

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, s8 = lane & 7;
    uint8_t* stage = stage_raw + 4 * kPadW;
    auto U = [](uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); };
    int64_t bad = INT64_MAX;
    const IT n_reads = (IT)A.n, L = (IT)A.L, n_chunks = (IT)A.n_chunks, CR = (IT)A.chunk_reads;

    // run records (bc_reads.read_runs) in place of the first decode: the variants with spare
    // registers (the others spill with the extra path)
    constexpr bool kRunsOn = !QUAL && NC == 5;
    // the next chunk's per-read fields are loaded while the current one is walked
    uint32_t fpos = 0x7FFFFFFFu, fsn = 0, fcb = 0, fcn = 0, fsn_first = 0, fsn_last = 0;
    auto fetch_into = [&](IT ch, uint32_t& xpos, uint32_t& xsn, uint32_t& xcb, uint32_t& xcn, uint32_t& xfirst,
                          uint32_t& xlast) {
        if (ch >= n_chunks) return;
        const IT b0 = ch * CR;
        const int n = (int)(n_reads - b0 < CR ? n_reads - b0 : CR);
        if (tid < n) {
            xpos = (uint32_t)*elem(A.pos, b0 + tid);
            if (!kRunsOn || !A.runs) {  // (uniform) with run records the CIGAR is read only on demand
                xcb = *elem(A.cig_beg, b0 + tid);
                xcn = *elem(A.cig_n, b0 + tid);
            }
            xsn = *elem(A.seq_nib, b0 + tid);
        }
        xfirst = sload(elem(A.seq_nib, b0));  // speculative staging bounds (reads usually lie in file order)
        xlast = sload(elem(A.seq_nib, b0 + n - 1));
    };
    auto fetch_fields = [&](IT ch) { fetch_into(ch, fpos, fsn, fcb, fcn, fsn_first, fsn_last); };
    fetch_fields((IT)blockIdx.x);
    // the next chunk's first CIGAR words, loaded during this chunk's sum (pf_ok: loaded); not
    // with qualities and six columns, which sit at the VGPR cap without it
    constexpr bool kPfOn = !(QUAL && NC == 6);
    const uint4* const runs = kRunsOn ? A.runs : nullptr;
    // the upload's chunk summaries: the chunk bounds without the block reduction (and its barrier)
    const uint4* const sums = kRunsOn && A.runs ? A.sums : nullptr;
    if (tid < 2) ncx[tid] = 0;
    __syncthreads();
    int par = 0;                // chunk parity (ncx slot)
    constexpr int kPf = 6;
    uint32_t pw[kPf] = {0u, 0u, 0u, 0u, 0u, 0u};
    bool pf_ok = false;

    // An image chunk's counts (fin, in the image path's otherwise unused hist region) are flushed
    // by wave 3 during the NEXT image chunk's sum, in which it has no rows: waves 0-2 then never
    // issue atomics, and their next CIGAR loads do not wait behind them (vmcnt is in order).
    uint32_t* const fin = &hist[0][0];  // [class][8 kImgRows positions]
    static_assert(6 * 8 * kImgRows <= 3 * kRcWinPos, "fin fits the hist region");
    int pend_g0 = 0, pend_nw = 0;  // (uniform) the pending chunk's first window and window count
    auto flush_pending = [&](int t0, int stride) {
        for (int t = t0; t < ((BC_ABL(A) & 2048) ? 0 : 8 * pend_nw); t += stride) {
            const IT p = 8 * (IT)pend_g0 + t;
            if (p >= L) break;
            // the position's column counts read together (one LDS round trip), then the atomics
            uint32_t v[NC];
#pragma unroll
            for (int c = 0; c < NC; ++c) v[c] = fin[c * 8 * kImgRows + t];
#pragma unroll
            for (int c = 0; c < NC; ++c)
                if (v[c]) atomicAdd(elem(A.counts, (IT)c * L + p), (int32_t)v[c]);
        }
    };
#ifdef BC_PHASE_TRACE
    uint64_t tsum[kRcPhases] = {0, 0, 0, 0, 0, 0, 0}, tlast = 0;
#endif
    for (IT chunk = blockIdx.x; chunk < n_chunks; chunk += (IT)gridDim.x) {
        RC_STAMP(0);
        const IT c0 = chunk * CR;
        const int nr = (int)(n_reads - c0 < CR ? n_reads - c0 : CR);
        // ---- 1. setup: one read per thread
        const bool valid = tid < nr;
        uint32_t mpos = 0x7FFFFFFFu, msn = 0, mcb = 0, mcn = 0;
        if (valid) {
            mpos = fpos;
            mcb = fcb;
            mcn = fcn;
            msn = fsn;
        }
        // speculative staging: the chunk's sequence usually lies in [first read's seq_nib, last
        // read's seq_nib + one read): staged now, in parallel with the CIGAR loads, and checked
        // against the exact bounds after the decode
        uint32_t spec_lo = (U(fsn_first) >> 1) & ~15u;
        uint32_t spec_hi = (U(fsn_last) >> 1) + kSpecSlack;
        const uint32_t buf_end = (uint32_t)(A.seq_words * 4 < 0xFFFFFFFFll ? A.seq_words * 4 : 0xFFFFFFFFll);
        spec_hi = spec_hi < buf_end ? spec_hi : buf_end;
        const bool spec = !QUAL && spec_hi > spec_lo && spec_hi - spec_lo <= (uint32_t)kStage && !(BC_ABL(A) & 512);
        // Gather staging (see kRcSlot): each read's slot words by LDS-DMA in stage order.  A wave's
        // 20 instructions cover exactly its own 64 reads' slots, so lane l of instruction e moves
        // word k of read r = (64 e + l) / 20 of the wave, whose first word and word count come
        // from read r's lane (a shuffle: no table, no barrier).  nwords(): this lane's read's words.
        auto gather_dma = [&](uint32_t src_word, uint32_t nwords) {
#pragma unroll 1
            for (int e = 0; e < kRcSlot / 4; ++e) {
                const uint32_t g = (uint32_t)(e * 64 + lane);
                const int r = (int)((g * 3277u) >> 16);  // g / 20 (g < 1280)
                const uint32_t k = g - (uint32_t)(kRcSlot / 4) * (uint32_t)r;
                const uint32_t src = (uint32_t)__shfl((int)src_word, r), nw = (uint32_t)__shfl((int)nwords, r);
                if (k < nw)
                    __builtin_amdgcn_global_load_lds((gbl_void_t*)(A.seq + src + 4u * k),
                                                     (lds_void_t*)(stage + 256 * (wave * (kRcSlot / 4) + e)), 4, 0, 0);
            }
        };
        // a chunk whose reads' sequences are not one short segment (a batch sorted on the device
        // without moving its sequence) is gathered speculatively, now, in parallel with the decode
        // and the bounds: every read's whole slot (the words the buffer holds), checked after
        const bool spec_g = kGather && !QUAL && !spec && !(BC_ABL(A) & 512);  // (uniform)
        // The loads prefetched during the previous chunk (fields, run records or CIGAR words) are
        // waited for HERE, before the stage DMA is queued behind them: vmcnt is in order and the
        // compiler cannot count the DMA passes, so a wait at their first use below would be a
        // vmcnt(0) that also waits for this chunk's whole stage copy (the decode then sat behind
        // the copy's round trip).  They were issued a whole phase ago: this wait is ~free.
        if (kEarlyWait) __builtin_amdgcn_s_waitcnt(kWaitVm0);
        if (spec) stage_dma<kRcThreads>(stage, A.seq + spec_lo, spec_hi - spec_lo, tid);
        if (spec_g) {
            const uint32_t w0 = (msn >> 1) & ~3u;
            const uint32_t left = buf_end > w0 ? (buf_end - w0) >> 2 : 0u;  // words of the buffer from w0
            gather_dma(w0, valid ? (left < (uint32_t)(kRcSlot / 4) ? left : (uint32_t)(kRcSlot / 4)) : 0u);
        }
        RunTable T;
        T.nrun = 0;
        T.gap = T.complex = false;
        T.span = T.qlen = 0;
#pragma unroll
        for (int i = 0; i < kMaxRuns; ++i) T.st[i] = T.en[i] = 0, T.qd[i] = 0;
        // the CIGAR fields of a chunk read from run records: loaded only when a decode needs them
        auto cig_fields = [&]() {
            if (runs && valid) {
                mcb = *elem(A.cig_beg, c0 + tid);
                mcn = *elem(A.cig_n, c0 + tid);
            }
        };
        // the first two runs only (all the event image needs); a chunk with more re-decodes below
        auto decode = [&](auto nslot) {
            const int cmax = (int)U(wave_reduce<true>(valid ? (mcn < (uint32_t)kPre ? mcn : (uint32_t)kPre) : 0u));
            if (valid) {
                uint32_t w[kPre];
                const bool use_pf = kPfOn && pf_ok && !runs && cmax <= kPf;  // (uniform)
                if (BC_ABL(A) & 131072) {  // diagnostic: decode a fixed 150M CIGAR (no loads waited for)
#pragma unroll
                    for (int i = 0; i < kPre; ++i) w[i] = i == 0 ? (150u << 4) : 0u;
                } else if (use_pf) {
#pragma unroll
                    for (int i = 0; i < kPre; ++i) w[i] = i < kPf ? pw[i] : 0u;
                } else {
#pragma unroll
                    for (int i = 0; i < kPre; ++i) w[i] = (i < cmax && (uint32_t)i < mcn) ? A.cigar[mcb + i] : 0u;
                    // waited for on this path only: the prefetched words need no wait (kEarlyWait)
                    if (kEarlyWait) __builtin_amdgcn_s_waitcnt(kWaitVm0);
                }
                if constexpr (decltype(nslot)::value == 2 && kFastDecode) {
                    // the lane's scratch: the image region, dead until this chunk's barrier below
                    const bool ok = decode_fast2(w, mcn, cmax, img + 8 * tid, T);
                    if (__ballot(!ok)) T = decode_runs<2>(w, mcn, cmax);  // (uniform) a read with > 2 runs
                } else {
                    T = decode_runs<decltype(nslot)::value>(w, mcn, cmax);
                }
            }
        };
        if (runs) {  // (uniform) the upload's run records: no CIGAR load, no decode
            if (valid) {
                uint4 q;
                if (kPfOn && pf_ok) {
                    q = make_uint4(pw[0], pw[1], pw[2], pw[3]);
                } else {
                    q = *elem(runs, c0 + tid);
                    if (kEarlyWait) __builtin_amdgcn_s_waitcnt(kWaitVm0);  // (this path only, as above)
                }
                T = unpack_runs(q.x, q.y, q.z, q.w);
            }
        } else if (BC_ABL(A) & 32768) {  // diagnostic: no CIGAR load / decode (every read one 120-base run)
            if (valid) {
                T.nrun = 1;
                T.st[0] = 0;
                T.en[0] = 120;
                T.qd[0] = 0;
                T.span = 120;
                T.qlen = 120;
            }
        } else {
            decode(std::integral_constant<int, 2>{});
        }
        const bool cx = valid && T.complex;
        const bool simple = valid && !cx;
        if (tid == 0) ncx[par ^ 1] = 0;  // the next chunk's slot (last read before the previous end barrier)
        // chunk bounds: P0 / P1 over all reads (complex ones: their true span), sequence segment
        // and maxima over the simple reads
        uint32_t cspan = T.span;
        if (cx && !sums) {
            cig_fields();
            uint64_t sp = 0;
            for (uint32_t k = 0; k < mcn; ++k) {
                const uint32_t wk = A.cigar[mcb + k];
                if (mlike(wk & 15u) || dlike(wk & 15u)) sp += wk >> 4;
            }
            cspan = sp > 0x3FFFFFFFu ? 0x3FFFFFFFu : (uint32_t)sp;
        }
        // v[7]: the longest simple read's sequence bytes (gather staging's slot test; not in the
        // upload's summaries, whose chunks never take gather staging)
        uint32_t v[8];
        const uint32_t rbytes = ((msn & 1u) + T.qlen + 1u) >> 1;  // the read's sequence bytes
        const bool over_slot = ((msn >> 1) & 3u) + rbytes > (uint32_t)kRcSlot;  // (gather staging: a complex read)
        const bool is_max[8] = {false, true, false, true, true, true, true, true};
        if (sums) {  // (uniform) reduced by the upload (bc_capi.hip chunk_summary: the same values)
            const uint32_t* sw = (const uint32_t*)elem(sums, 2 * chunk);
#pragma unroll
            for (int k = 0; k < 7; ++k) v[k] = sload(sw + k);
            v[7] = 0u;
            RC_STAMP(1);
            RC_STAMP(2);
        } else {
            v[0] = valid ? mpos : 0xFFFFFFFFu;
            v[1] = valid ? mpos + cspan : 0u;
            v[2] = (simple && T.qlen) ? (msn >> 1) : 0xFFFFFFFFu;
            v[3] = (simple && T.qlen) ? ((msn + T.qlen + 1) >> 1) : 0u;
            v[4] = simple ? T.span : 0u;
            // reads the event image cannot take (first run not at the read start, last run not
            // at its end) count as 3 runs: such a chunk takes the run tables
            v[5] = simple ? run_shape(T) : 0u;
            v[6] = (simple && T.gap) ? 1u : 0u;
            v[7] = simple ? rbytes : 0u;
            RC_STAMP(1);
            block_reduce<8, kRcWaves>(v, is_max, red);  // contains a __syncthreads
            RC_STAMP(2);
        }
        const IT P0 = (IT)v[0], P1 = (IT)v[1];
        uint32_t seg_lo = v[2];
        const uint32_t seg_hi = v[3];
        const int maxspan = (int)v[4], maxrun = (int)v[5];
        const bool gap = v[6] != 0;
        if (maxrun > 2) {  // (uniform) full run tables
            cig_fields();
            decode(std::integral_constant<int, kMaxRuns>{});
        }
        seg_lo = seg_hi > seg_lo ? (seg_lo & ~15u) : 0u;
        const bool spec_ok = spec && (seg_hi <= seg_lo || (seg_lo >= spec_lo && seg_hi <= spec_hi));
        if (spec_ok) seg_lo = spec_lo;  // the stage holds [spec_lo, spec_hi)
        const bool staged = spec_ok || seg_hi - seg_lo <= (uint32_t)kStage;
        // Gather staging: the chunk's sequence is not one short segment (the reads of a batch
        // sorted on the device without relaying its sequence, bc_sort.hip): every simple read's
        // bytes are copied to its own kRcSlot-byte slot of the stage instead, and a read longer
        // than its slot is walked as a complex read (rc_complex, from HBM).
        // Only when every simple read fits its slot (a chunk of long reads would walk
        // most of them as complex reads, one per wave with global atomics, where the run-table walk
        // from HBM is the better fallback).
        // event-image path: a staged chunk of reads with <= 2 runs whose windows fit the image.
        // Each read's events are extracted ONCE per window (lane = read, its windows in a row)
        // instead of once per (window, run) item from the run table.
        const IT WBc = P0 & ~(IT)7;
        const int NWc = (int)(P1 > WBc ? (P1 - WBc + 7) / 8 : 0);
        const bool img_shape = maxrun <= 2 && NWc <= kImgRows && !(BC_ABL(A) & 8192);  // (uniform)
        const bool gather = kGather && !QUAL && !staged && !sums && v[7] <= (uint32_t)kRcSlot &&
                            !(BC_ABL(A) & 512);  // (uniform)
        const bool big = gather && simple && over_slot;
        const bool cxa = cx || big, simplea = simple && !big;
        const bool inlds = staged || gather;  // (uniform) the walks read the stage
        // the read's first base as a nibble index of the stage (or of the batch's buffer)
        const uint32_t rel = gather ? (uint32_t)(2 * kRcSlot * tid) + (msn & 7u) : msn - (staged ? 2u * seg_lo : 0u);
        if (cxa) cxl[atomicAdd(&ncx[par], 1u)] = (uint32_t)tid;
        const bool img_path = inlds && img_shape;
        const int gpad = NWc;  // (uniform) the image's group padding (see rec)
        uint32_t* const mycol = img + tid * kImgRows + (tid >> 5) * gpad;  // this read's image column
        if ((spec && !spec_ok) || (spec_g && !gather)) {  // (uniform) the speculative copy is overwritten
            stage_wait();
            __syncthreads();
        }
        // ---- stage the chunk's sequence exactly (16 B per thread per pass) unless done above
        if (!QUAL && staged && !spec_ok && !(BC_ABL(A) & 512)) stage_dma<kRcThreads>(stage, A.seq + seg_lo, seg_hi - seg_lo, tid);
        if (QUAL && staged && !spec_ok && !(BC_ABL(A) & 512)) {
            for (uint32_t off = tid * 16u; off < seg_hi - seg_lo; off += kRcThreads * 16u) {
                uint4 q4 = *(const uint4*)(A.seq + seg_lo + off);  // padded buffer: in bounds
                if (QUAL) {
                    const int64_t q0 = 2 * ((int64_t)seg_lo + off);
                    uint32_t qw[8];
                    if (((uintptr_t)A.qual & 15u) == 0 && q0 + 32 <= A.qual_bytes) {
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
                    q4.x &= qual_nibmask(qw[0], qw[1], A.mbq);
                    q4.y &= qual_nibmask(qw[2], qw[3], A.mbq);
                    q4.z &= qual_nibmask(qw[4], qw[5], A.mbq);
                    q4.w &= qual_nibmask(qw[6], qw[7], A.mbq);
                }
                *(uint4*)(stage + off) = q4;
            }
        }
        if (gather && !spec_g)  // (uniform) not gathered at the chunk start: the exact words now
            gather_dma((msn >> 1) & ~3u, (simple && !over_slot) ? (((msn >> 1) & 3u) + rbytes + 3u) >> 2 : 0u);
        // ---- records (pos kept for complex / padding entries so pos[] stays sorted)
        {
            uint32_t rr[kMaxRuns], nb[kMaxRuns];
#pragma unroll
            for (int k = 0; k < kMaxRuns; ++k) {
                rr[k] = simplea ? pack_rr(T.st[k], T.en[k]) : 0u;
                nb[k] = rel + (uint32_t)T.qd[k];
            }
            if (!img_path) {
                rec[tid * 3] = make_uint4(mpos, simplea ? T.span * 4u : 0u, rr[0], nb[0]);
                rec[tid * 3 + 1] = make_uint4(rr[1], nb[1], rr[2], nb[2]);
                rec[tid * 3 + 2] = make_uint4(rr[3], nb[3], 0u, 0u);
            }
            if (!img_path) rpos[tid] = (int32_t)mpos;  // (the window tables of the run-table walk)
        }
        if (!QUAL) stage_wait();  // this thread's LDS-DMA landed (hipcc does not track it)
        __syncthreads();  // stage, records and the complex-read list complete
        RC_STAMP(3);
        if (kPfOn) fetch_fields(chunk + (IT)gridDim.x);  // back before the CIGAR prefetch below
        if (img_path) {
            // ---- event image: thread tid writes column tid, rows = the chunk's windows
            // [G0, G0 + NWc): the 8 event classes its read has in each (zero outside the read)
            const int p7 = (int)(mpos & 7u);
            const int G0 = (int)(U((uint32_t)P0) >> 3);
            const int i0 = (int)(mpos >> 3) - G0;  // the read's first window row
            // run k: stage nibble of stream position 0 (= window row i0, nibble 0)
            const int s0 = (int)rel + T.qd[0] - p7, s1 = (int)rel + T.qd[1] - p7;
            const int wb0 = s0 >> 3, wb1 = s1 >> 3;
            const uint32_t sh0 = (uint32_t)(s0 & 7) * 4u, sh1 = (uint32_t)(s1 & 7) * 4u;
            // Stream bits (4 per nibble) from the image's first row: the read is [Z, SP), its
            // first run [Z, B0), the deletions [B0, A1), the second run [A1, SP) (one-run reads:
            // A1 = B0 = SP).  Row r's window is stream bits [32r, 32r + 32).
            const int ob = 32 * i0 + 4 * p7;  // stream bit of the read's reference offset 0
            const int Z = ob, SP = ob + 4 * (int)T.span;
            const int B0 = ob + 4 * (int)T.en[0];
            const int A1 = T.nrun == 2 ? ob + 4 * (int)T.st[1] : SP;
            const int B0e = T.nrun == 2 ? B0 : SP;
            // run k's stage word of row r is f_k + r (+1 for the funnel's upper word): within
            // [-kPadW + 1, kStage / 4 + kPadW - 1] for every simple read (f_k >= -1 - 22, the
            // read's sequence lies in the stage), so the stage's pads absorb it unclamped
            const uint32_t* w0 = (const uint32_t*)stage + (wb0 - i0);
            const uint32_t* w1 = (const uint32_t*)stage + (wb1 - i0);
            // Row r's 8 event classes, all rows unrolled without branches so the LDS reads of
            // later rows issue ahead.  ge(X): the row's stream bits at or above X, i.e. bits
            // >= d = clamp(X - 32r, 0, 32).  The clamp is one med3 of X against [32r, 32r + 32]
            // (constants the compiler keeps in registers), and 0xFFFFFFFF << (m mod 64) as 64
            // bits holds the mask in its low word (even r: m mod 64 = d) or its high word (odd r:
            // 32 + d, or 0 when d = 32).
            auto expand = [&](auto two_c, auto edge_c) {
                constexpr bool TWO = decltype(two_c)::value, EDGE = decltype(edge_c)::value;
                const int yz = Z, yb = B0e, ya = A1, ys = SP;
                uint32_t p0 = w0[0], p1 = TWO ? w1[0] : 0u;
#pragma unroll
                for (int row = 0; row < kImgRows; ++row) {
                    if (row >= kImgRows - 4 && row >= NWc) continue;  // (uniform) past the chunk
                    auto ge = [&](int Y) {
                        const int lo = 32 * row;
                        const int m = Y < lo ? lo : (Y > lo + 32 ? lo + 32 : Y);
                        const unsigned long long v = shl64_mod64(0xFFFFFFFFull, m);
                        return (row & 1) ? (uint32_t)(v >> 32) : (uint32_t)v;
                    };
                    const uint32_t gz = ge(yz), gb = ge(yb);
                    const uint32_t n0 = w0[row + 1];
                    uint32_t x = __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_alignbit(n0, p0, sh0), gz, gb, 0x40);
                    p0 = n0;
                    if (TWO) {
                        const uint32_t ga = ge(ya), gs = ge(ys);
                        const uint32_t n1 = w1[row + 1];
                        const uint32_t x1 = __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_alignbit(n1, p1, sh1), ga, gs, 0x40);
                        // (independent terms: a select chain measured slower, 57 vs 54 us)
                        // s0 & s1 & ~s2 (0x40); then s0 | s1 | s2 (0xFE) in one op
                        x = __builtin_amdgcn_bitop3_b32(x, x1, __builtin_amdgcn_bitop3_b32(kClsDel, gb, ga, 0x40), 0xFE);
                        p1 = n1;
                    }
                    if (EDGE) {
                        const IT rb = 8 * (IT)(G0 + row);  // (uniform) the row's first position
                        if (rb + 8 > L) {  // events at positions >= L: the reference's out_of_range
                            IT kL = L - rb;
                            kL = kL < 0 ? 0 : (kL > 8 ? 8 : kL);
                            const uint32_t bmask = ~(lo32_bit(4 * (int)kL) - 1u);
                            if ((x & bmask) && c0 + tid < bad) bad = c0 + tid;
                            x &= ~bmask;
                        }
                    }
                    mycol[row] = x;
                }
            };
            // Interior rows, then boundary rows.  A row that no boundary (Z, B0, A1, SP) falls
            // strictly inside lies entirely in one segment (run 0, the deletions, run 1) or
            // outside the read, so its word is one stream word, kClsDel or 0: the loop takes it
            // from per-lane row bitmasks (one v_bfe_i32 per row and segment) instead of four
            // clamped masks.  The <= 4 rows a boundary cuts are then overwritten with the exact
            // formula above, at their (per-lane) row.
            auto rowmask = [](int a, int b) -> uint32_t {  // rows lying entirely in stream bits [a, b)
                const int lo = (a + 31) >> 5, hi = b >> 5;
                return hi > lo ? lo32_bit(hi) - lo32_bit(lo) : 0u;
            };
            auto interior = [&]() {
                const uint32_t o0 = rowmask(Z, B0e), o1 = rowmask(A1, SP);
                uint32_t p0 = w0[0], p1 = w1[0];
#pragma unroll
                for (int row = 0; row < kImgRows; ++row) {
                    if (row >= kImgRows - 4 && row >= NWc) continue;  // (uniform) past the chunk
                    const uint32_t n0 = w0[row + 1], n1 = w1[row + 1];
                    const uint32_t m0 = (uint32_t)__builtin_amdgcn_sbfe((int)o0, row, 1);
                    const uint32_t m1 = (uint32_t)__builtin_amdgcn_sbfe((int)o1, row, 1);
                    const uint32_t x1 = __builtin_amdgcn_alignbit(n1, p1, sh1) & m1;
                    // (s0 & m0) | x1: a row lies in at most one segment
                    mycol[row] = __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_alignbit(n0, p0, sh0), m0, x1, 0xEA);
                    p0 = n0;
                    p1 = n1;
                }
                // rows lying entirely in a deletion (>= 8 deleted positions; none in most waves)
                for (uint32_t od = rowmask(B0e, A1); od; od &= od - 1u) mycol[__builtin_ctz(od)] = kClsDel;
                // The <= 4 rows the boundaries cut, rewritten with the exact formula, without
                // branches: all 8 stage-word pairs are read before any is used (one LDS round
                // trip, not two per boundary), and a boundary that cuts no row (b % 32 == 0) or
                // lies past the image rewrites a row the formula gets right anyway (row 22 at
                // most: its words are inside the stage pads).
                if (!(BC_ABL(A) & 65536)) {  // (diagnostic 65536: no boundary rows)
                    const int bs[4] = {Z, B0e, A1, SP};
                    int rbs[4];
                    uint2 q0[4], q1[4];
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const int rb = bs[k] >> 5;
                        rbs[k] = rb < kImgRows - 1 ? rb : kImgRows - 1;
                        q0[k] = make_uint2(w0[rbs[k]], w0[rbs[k] + 1]);
                        q1[k] = make_uint2(w1[rbs[k]], w1[rbs[k] + 1]);
                    }
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const int lo = 32 * rbs[k];
                        auto ge = [&](int Y) {
                            const int d = Y - lo;
                            return (uint32_t)shl64_mod64(0xFFFFFFFFull, d < 0 ? 0 : (d > 32 ? 32 : d));
                        };
                        const uint32_t gz = ge(Z), gb = ge(B0e), ga = ge(A1), gs = ge(SP);
                        const uint32_t x0 = __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_alignbit(q0[k].y, q0[k].x, sh0), gz, gb, 0x40);
                        const uint32_t x1 = __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_alignbit(q1[k].y, q1[k].x, sh1), ga, gs, 0x40);
                        mycol[rbs[k]] =
                            __builtin_amdgcn_bitop3_b32(x0, x1, __builtin_amdgcn_bitop3_b32(kClsDel, gb, ga, 0x40), 0xFE);
                    }
                }
            };
            if (!simplea || (BC_ABL(A) & 16384)) {
#pragma unroll
                for (int row = 0; row < kImgRows; ++row) mycol[row] = 0u;
            } else if (8 * (IT)(G0 + kImgRows) > L) {  // (uniform) rows may reach past L
                expand(std::true_type{}, std::true_type{});
            } else {
                interior();
            }
        }
        pf_ok = false;
        if (!kPfOn) {
            fetch_fields(chunk + (IT)gridDim.x);  // in flight during the walk
        } else if (chunk + (IT)gridDim.x < n_chunks) {
            const IT nb0 = (chunk + (IT)gridDim.x) * CR;
            const int nn = (int)(n_reads - nb0 < CR ? n_reads - nb0 : CR);
            const bool nv = tid < nn;
            if (runs) {  // (uniform) the next chunk's run records instead of its CIGAR words
                if (nv) {
                    const uint4 q = *elem(runs, nb0 + tid);
                    pw[0] = q.x, pw[1] = q.y, pw[2] = q.z, pw[3] = q.w;
                }
            } else {
                const int ncm = (BC_ABL(A) & 262144) ? 0 :  // diagnostic: no CIGAR prefetch
                                    (int)U(wave_reduce<true>(nv ? (fcn < (uint32_t)kPre ? fcn : (uint32_t)kPre) : 0u));
#pragma unroll
                for (int i = 0; i < kPf; ++i) pw[i] = (nv && i < ncm && (uint32_t)i < fcn) ? A.cigar[fcb + i] : 0u;
            }
            pf_ok = true;
        }
        const SeqSrc src{inlds ? (const uint32_t*)stage : (const uint32_t*)A.seq,
                         inlds ? (int64_t)((gather ? kGStage : kStage) / 4) : A.seq_words, A.qual, A.qual_bytes, A.mbq};
        const IT WB = P0 & ~(IT)7;
        const int G0w = (int)(WB >> 3);  // the image's first window (image path)
        const IT NW = P1 > WB ? (P1 - WB + 7) / 8 : 0;
        if (img_path) {
            __syncthreads();  // the image complete (columns are written by their read's thread)
            RC_STAMP(4);
            // ---- image path, transposed: thread t < 8 R (R = NWc rows) takes row g = t mod R and
            // read group q = t / R, and adds the 32 reads [32q, 32q + 32) of row g into SWAR nibble
            // counters, byte counters per class every <= 15 reads.  8 R <= 184 threads: the 4th
            // wave skips the sum (rows as lanes mod 32 left a third of the lanes idle).  The 8
            // groups' byte counters meet in LDS (the dead stage); thread (class c, row g) adds
            // them in 16-bit lanes and writes the row's 8 positions.
            const int R = NWc;
            const uint32_t inv = (65536u + (uint32_t)R - 1u) / (uint32_t)R;  // t / R = (t * inv) >> 16 (t < 256)
            constexpr int kPartStride = 24;                                  // >= kImgRows
            uint32_t* part = (uint32_t*)stage;                              // [q][2 NC][kPartStride]
            // Read pairs: the words of reads r and r + 1 of the row are one ds_read2 into a register
            // pair, and their three shifted copies (x >> 1, 2, 3) are three 64-bit shifts (the bits
            // shifted across the halves land on nibble bits the class masks drop): 1.5 shifts per
            // word instead of 3.
            constexpr int kGroups = 8;
            if (tid < 8 * R && !(BC_ABL(A) & 4)) {
                const int q = (int)(((uint32_t)tid * inv) >> 16), gr = tid - q * R;
                uint32_t blo[6], bhi[6];
                const uint32_t* col = img + 32 * q * kImgRows + q * gpad + gr;
                // Bit-sliced: a row word's 32 bits are (position j, plane p) = bit 4j + p of the
                // class nibble.  A carry-save tree counts every bit position over the 32 reads at
                // once (digits xd: plane counts A+N, C+N, G+DS, T+DS); the N (0011) and DS (1100)
                // planes, b0 & b1 and b2 & b3 of a nibble, are counted the same way with two reads
                // packed per word (yd).  A bit transpose turns the digits into byte counters.
                uint32_t xd[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u}, yd[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
                uint32_t y[16], x16 = 0u;
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    uint32_t w[16];
#pragma unroll
                    for (int k = 0; k < 16; ++k) w[k] = col[(16 * h + k) * kImgRows];
#pragma unroll
                    for (int k = 0; k < 16; k += 2) {
                        const unsigned long long X1 = shr64<1>(((unsigned long long)w[k + 1] << 32) | w[k]);
                        // bits 4j / 4j + 2: N / DS of read k; 4j + 1 / 4j + 3: those of read k + 1
                        const uint32_t ya = __builtin_amdgcn_bitop3_b32(w[k], (uint32_t)X1, 0x55555555u, 0x80);
                        const uint32_t yb = __builtin_amdgcn_bitop3_b32(w[k + 1], (uint32_t)(X1 >> 32), 0x55555555u, 0x80);
                        y[8 * h + k / 2] = (yb << 1) | ya;
                    }
                    const uint32_t c16 = csa16(xd, w);
                    if (h == 0) {
                        x16 = c16;
                    } else {
                        xd[4] = x16 ^ c16;
                        xd[5] = x16 & c16;
                    }
                }
                yd[4] = csa16(yd, y);
                bit_transpose8(xd);  // xd[4h + p]: plane p, byte i = position 2i + h (<= 32)
                bit_transpose8(yd);  // yd[4h + 0/1]: N of even / odd reads, 4h + 2/3: DS (<= 16)
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const uint32_t nn = yd[4 * h] + yd[4 * h + 1], ds = yd[4 * h + 2] + yd[4 * h + 3];
                    uint32_t* o = h ? bhi : blo;
                    o[0] = xd[4 * h] - nn;  // bytes: no borrow (plane count >= its N / DS count)
                    o[1] = xd[4 * h + 1] - nn;
                    o[2] = xd[4 * h + 2] - ds;
                    o[3] = xd[4 * h + 3] - ds;
                    o[4] = ds;
                    o[5] = nn;
                }
#pragma unroll
                for (int c = 0; c < NC; ++c) {
                    part[(q * 2 * NC + 2 * c) * kPartStride + gr] = blo[c];
                    part[(q * 2 * NC + 2 * c + 1) * kPartStride + gr] = bhi[c];
                }
            } else if (wave == kRcWaves - 1) {
                static_assert(8 * kImgRows <= 64 * (kRcWaves - 1), "the last wave has no image rows");
                flush_pending(lane, 64);  // the previous image chunk's counts (8 R <= 184 < 192)
            }
            static_assert(kGroups * 2 * 6 * kPartStride * 4 <= kStage, "the groups' partial rows fit the stage");
            __syncthreads();  // the groups' partial rows; the pending counts read
            RC_STAMP(5);
            // the rows' final counts in LDS, [class][position]
            if (tid < NC * R) {
                const int c = (int)(((uint32_t)tid * inv) >> 16), gr = tid - c * R;
                // byte k of the lo (hi) word = position 2k (2k + 1).  A group's byte is <= 32, so
                // four groups add as bytes (<= 128); the two halves of the block then meet in
                // 16-bit lanes (<= 256)
                static_assert(kGroups == 8, "two halves of four 32-read groups");
                uint32_t e = 0, o = 0, e2 = 0, o2 = 0;
                if (!(BC_ABL(A) & 4)) {
                    uint32_t vl[2] = {0u, 0u}, vh[2] = {0u, 0u};
#pragma unroll
                    for (int g8 = 0; g8 < kGroups; ++g8) {
                        vl[g8 >> 2] += part[(g8 * 2 * NC + 2 * c) * kPartStride + gr];
                        vh[g8 >> 2] += part[(g8 * 2 * NC + 2 * c + 1) * kPartStride + gr];
                    }
#pragma unroll
                    for (int hf = 0; hf < 2; ++hf) {
                        e += vl[hf] & 0x00FF00FFu;         // positions 0, 4 (16-bit halves)
                        e2 += (vl[hf] >> 8) & 0x00FF00FFu;  // positions 2, 6
                        o += vh[hf] & 0x00FF00FFu;         // positions 1, 5
                        o2 += (vh[hf] >> 8) & 0x00FF00FFu;  // positions 3, 7
                    }
                }
                uint32_t* f = fin + c * 8 * kImgRows + 8 * gr;
                f[0] = e & 0xFFFFu, f[1] = o & 0xFFFFu, f[2] = e2 & 0xFFFFu, f[3] = o2 & 0xFFFFu;
                f[4] = e >> 16, f[5] = o >> 16, f[6] = e2 >> 16, f[7] = o2 >> 16;
            }
            pend_g0 = G0w;  // flushed by wave 3 in the next image chunk, or below
            pend_nw = NWc;
        }
        if (!img_path && pend_nw) {  // (uniform) the run tables reuse hist: flush the pending counts
            flush_pending(tid, kRcThreads);
            pend_nw = 0;
            __syncthreads();
        }
        // ---- 2./3. window passes of up to kRcWin windows (run-table walk)
        for (int64_t wp = 0; wp < (img_path ? 0 : NW); wp += kRcWin) {
            const int nwin = (int)(NW - wp < kRcWin ? NW - wp : kRcWin);
            const int64_t PB = WB + 8 * wp;
            for (int t = tid; t < 3 * kRcWinPos; t += kRcThreads) (&hist[0][0])[t] = 0u;
            // reads overlapping window g are those with pos in [gb - maxspan + 1, gb + 8); pos is
            // sorted, so both ends are monotone in g: read t is the boundary for the windows
            // between its window and the next read's (no search, every entry written once)
            if (tid < nr) {
                auto win_of = [&](int64_t p) {  // window index of position p, clipped to [0, nwin]
                    const int64_t w = p >= PB ? (p - PB) >> 3 : -1;
                    return (int)(w < 0 ? 0 : (w > nwin ? nwin : w));
                };
                const int64_t p_t = rpos[tid];
                const int64_t p_n = tid + 1 < nr ? (int64_t)rpos[tid + 1] : INT64_MAX / 2;
                // hi: b_g = #{pos < gb + 8} = t + 1 for g in [win(p_t), win(p_next))
                const int b0 = tid == 0 ? 0 : win_of(p_t), b1 = tid + 1 < nr ? win_of(p_n) : nwin;
                if (tid == 0)
                    for (int g2 = 0; g2 < win_of(p_t); ++g2) whi[g2] = 0;
                for (int g2 = (tid == 0 ? win_of(p_t) : b0); g2 < b1; ++g2) whi[g2] = (uint32_t)tid + 1;
                // lo: a_g = #{pos + maxspan - 1 < gb} = t + 1 for g in [win(u_t) + 1, win(u_next) + 1)
                const int64_t u_t = p_t + maxspan - 1, u_n = p_n + maxspan - 1;
                const int a0 = win_of(u_t) + (u_t >= PB ? 1 : 0);
                const int a1 = tid + 1 < nr ? win_of(u_n) + (u_n >= PB ? 1 : 0) : nwin;
                if (tid == 0)
                    for (int g2 = 0; g2 < (a0 < nwin ? a0 : nwin); ++g2) wlo[g2] = 0;
                for (int g2 = a0; g2 < (a1 < nwin ? a1 : nwin); ++g2) wlo[g2] = (uint32_t)tid + 1;
            } else if (nr == 0 && tid < nwin) {
                wlo[tid] = whi[tid] = 0;
            }
            __syncthreads();  // window read ranges complete
            if (wave == 0) {
                uint32_t cnt = 0;
                if (lane < nwin) {
                    const uint32_t a = wlo[lane], b = whi[lane];
                    cnt = b > a ? (b - a + 63) / 64 : 0u;
                }
                // exclusive prefix of the item counts over the windows (DPP scan)
                uint32_t inc = cnt;
                inc += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)inc, 0x111, 0xF, 0xF, false);
                inc += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)inc, 0x112, 0xF, 0xF, false);
                inc += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)inc, 0x114, 0xF, 0xF, false);
                inc += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)inc, 0x118, 0xF, 0xF, false);
                inc += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)inc, 0x142, 0xA, 0xF, false);
                inc += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)inc, 0x143, 0xC, 0xF, false);
                if (lane < nwin) wpre[lane] = inc - cnt;
                if (lane == nwin - 1) wpre[nwin] = inc;
            }
            __syncthreads();  // hist zeroed, window table ready
            // this wave's items [k0, k1): contiguous, so it changes window only a few times
            const uint32_t I = U(wpre[nwin]);
            const uint32_t k0 = (uint32_t)(((uint64_t)I * wave) / kRcWaves);
            const uint32_t k1 = (uint32_t)(((uint64_t)I * (wave + 1)) / kRcWaves);
            Swar W;
#pragma unroll
            for (int c = 0; c < 6; ++c) W.a4[c] = 0;
            int g = 0, it4 = 0;
            while (g + 1 < nwin && U(wpre[g + 1]) <= k0) ++g;
            uint32_t gnext = U(wpre[g + 1]), gpre = U(wpre[g]), glo = U(wlo[g]), ghi = U(whi[g]);
            const uint32_t k1w = (BC_ABL(A) & 4) ? k0 : k1;
            for (uint32_t k = k0; k < k1w; ++k) {
                if (k >= gnext) {  // next window (wave-uniform)
                    if (it4) rc_fold<NC>(W, hist, g, s8, BC_ABL(A));
                    it4 = 0;
                    while (k >= U(wpre[g + 1])) ++g;
                    gnext = U(wpre[g + 1]);
                    gpre = U(wpre[g]);
                    glo = U(wlo[g]);
                    ghi = U(whi[g]);
                }
                const int gb = (int)(PB + 8 * g);
                // two items of the same window per step when there are (two independent LDS
                // chains in flight); the step's reads r and r + 64
                const bool two = k + 1 < k1w && k + 1 < gnext;  // (uniform)
                const uint32_t r = glo + 64u * (k - gpre) + (uint32_t)lane;
                auto events = [&](uint32_t rr) {
                    const int rs = rr < ghi ? (int)rr : 0;
                    uint32_t x;
                    if (BC_ABL(A) & 256) {
                        x = rec[rs * 3].x * 0x01010101u;
                    } else if (maxrun <= 1) {
                        x = gap ? (inlds ? window_events<1, true, true, QUAL>(src, rec, rs, gb)
                                         : window_events<1, true, false, QUAL>(src, rec, rs, gb))
                                : (inlds ? window_events<1, false, true, QUAL>(src, rec, rs, gb)
                                         : window_events<1, false, false, QUAL>(src, rec, rs, gb));
                    } else if (maxrun == 2) {
                        x = inlds ? window_events<2, true, true, QUAL>(src, rec, rs, gb)
                                  : window_events<2, true, false, QUAL>(src, rec, rs, gb);
                    } else {
                        x = inlds ? window_events<4, true, true, QUAL>(src, rec, rs, gb)
                                  : window_events<4, true, false, QUAL>(src, rec, rs, gb);
                    }
                    return rr < ghi ? x : 0u;
                };
                uint32_t x0 = events(r), x1 = two ? events(r + 64u) : 0u;
                if ((int64_t)gb + 8 > A.L) {  // window reaches past the reference end
                    int64_t kL = A.L - gb;
                    kL = kL < 0 ? 0 : (kL > 8 ? 8 : kL);
                    const uint32_t bmask = ~(lo32_bit(4 * (int)kL) - 1u);
                    if ((x0 & bmask) && c0 + (int64_t)r < bad) bad = c0 + (int64_t)r;
                    if ((x1 & bmask) && c0 + (int64_t)r + 64 < bad) bad = c0 + (int64_t)r + 64;
                    x0 &= ~bmask;
                    x1 &= ~bmask;
                }
                swar_add<NC>(W, x0);
                if (two) {
                    swar_add<NC>(W, x1);
                    ++k;
                    ++it4;
                }
                if (++it4 >= 13) {  // every nibble counter <= 14
                    rc_fold<NC>(W, hist, g, s8, BC_ABL(A));
                    it4 = 0;
                }
            }
            if (it4) rc_fold<NC>(W, hist, g, s8, BC_ABL(A));
            __syncthreads();
            // ---- 4. flush the pass's positions (< L) into the counts
            for (int t = tid; t < ((BC_ABL(A) & 2048) ? 0 : 8 * nwin); t += kRcThreads) {
                const int64_t p = PB + t;
                if (p >= A.L) break;
#pragma unroll
                for (int pl = 0; pl < 3; ++pl) {
                    const uint32_t hv = hist[pl][t];
                    const uint32_t lo = hv & 0xFFFFu, hi = hv >> 16;
                    if (lo && 2 * pl < NC) atomicAdd(&A.counts[(int64_t)(2 * pl) * A.L + p], (int32_t)lo);
                    if (hi && 2 * pl + 1 < NC) atomicAdd(&A.counts[(int64_t)(2 * pl + 1) * A.L + p], (int32_t)hi);
                }
            }
            __syncthreads();  // hist reused by the next pass / chunk
        }
        // ---- complex reads: one wave per read, global atomics
        const uint32_t nc = U(ncx[par]);
        for (uint32_t q = wave; q < nc; q += kRcWaves) rc_complex<QUAL, NC>(A, c0 + cxl[q], bad);
        __syncthreads();  // records / stage / cxl reused by the next chunk
        RC_STAMP(6);
        par ^= 1;
    }
#ifdef BC_PHASE_TRACE
    if (A.trace && lane == 0)
        for (int k = 0; k < kRcPhases; ++k)
            A.trace[((size_t)blockIdx.x * kRcWaves + wave) * kRcPhases + k] = tsum[k];
#endif
    flush_pending(tid, kRcThreads);  // the last image chunk's counts (written before its end barrier)
    // first offending read of this block (std::out_of_range in the reference)
    for (int o = 32; o > 0; o >>= 1) {
        const int64_t b2 = __shfl_down(bad, o);
        bad = b2 < bad ? b2 : bad;
    }
    if (lane == 0 && bad != INT64_MAX) atomicMin(A.err, (unsigned long long)bad);
}

}  // namespace

bool use_rc(const bc_reads& r, int64_t L, int shape) {
    if (!r.sorted || r.n_reads <= 0 || r.seq_layout != BC_SEQ_EVENT) return false;
    if (shape == BC_SHAPE_RC) return true;
    if (shape == BC_SHAPE_TILE || shape == BC_SHAPE_TILE_NO_SOLO) return r.max_span > kTileMaxSpan;
    if (r.max_span > kTileMaxSpan) return true;  // the tiled kernel's look-back gets too long
    const int64_t reach = r.max_end > L ? r.max_end : L;
    const double per_tile = reach > 0 ? (double)r.n_reads * (double)(r.max_span + 63) / (double)reach : 0.0;
    return per_tile >= kRcMinReadsPerTile;
}

hipError_t launch_rc(hipStream_t s, const bc_reads& r, int64_t L, uint32_t mbq, int ncols, int32_t* counts,
                     unsigned long long* d_err) {
    if (r.n_reads <= 0) return hipSuccess;
    RcArgs A;
    A.pos = r.pos;
    A.cig_beg = r.cig_beg;
    A.cig_n = r.cig_n;
    A.seq_nib = r.seq_nib;
    A.cigar = r.cigar;
    A.seq = r.seq;
    A.qual = r.qual;
    A.n = r.n_reads;
    A.L = L;
    A.mbq = mbq;
    A.seq_words = (int64_t)(seq_event_bytes(r.seq_bytes) / 4);
    A.qual_bytes = r.qual ? r.qual_bytes : 0;
    A.runs = r.read_runs && !((uintptr_t)r.read_runs & 15u) && index_valid(r) ? (const uint4*)r.read_runs : nullptr;
    A.counts = counts;
    A.err = d_err;
    A.ablate = 0;
#ifdef BC_DIAG
    if (const char* ab = std::getenv("BC_ABLATE")) A.ablate = std::atoi(ab);
#endif
    constexpr int nt = kRcChunk;
    A.n_chunks = (r.n_reads + nt - 1) / nt;
    A.chunk_reads = nt;
    A.sums = A.runs && r.run_chunks == A.n_chunks ? A.runs + r.n_reads : nullptr;
    // resident blocks: LDS bounds a CU to 3 (event image + stage + histogram)
    const int64_t cap = 256 * 3;
    const int64_t blocks = A.n_chunks < cap ? A.n_chunks : cap;
    const dim3 grid((unsigned)blocks), block(nt);
    A.trace = nullptr;
#ifdef BC_PHASE_TRACE
    // diagnostic only: BC_TRACE=<file> dumps the per-wave phase totals of the 20th launch
    static unsigned long long* tbuf = nullptr;
    static int tcalls = 0;
    const char* tpath = std::getenv("BC_TRACE");
    const size_t tn = (size_t)blocks * (nt / 64) * kRcPhases;
    if (tpath && !tbuf) (void)hipMallocManaged((void**)&tbuf, tn * 8);
    if (tpath) A.trace = tbuf;
#endif
    // 32-bit indices when every byte offset (16 B per read, 4 B per count) fits 32 bits
    const bool i32 = A.n < ((int64_t)1 << 27) && L < ((int64_t)1 << 27);
#define BC_RC(Q, KK)                                                                   \
    do {                                                                               \
        if (i32) hipLaunchKernelGGL((k_rc<Q, KK, nt, int32_t>), grid, block, 0, s, A); \
        else hipLaunchKernelGGL((k_rc<Q, KK, nt, int64_t>), grid, block, 0, s, A);     \
    } while (0)
    if (mbq > 0) {
        if (ncols == 6) BC_RC(true, 6);
        else BC_RC(true, 5);
    } else {
        if (ncols == 6) BC_RC(false, 6);
        else BC_RC(false, 5);
    }
#undef BC_RC
#ifdef BC_PHASE_TRACE
    if (A.trace && ++tcalls == 20) {
        (void)hipStreamSynchronize(s);
        if (FILE* f = std::fopen(tpath, "wb")) {
            std::fwrite(A.trace, 8, tn, f);
            std::fclose(f);
        }
    }
#endif
    return hipGetLastError();
}

}  // namespace bc
