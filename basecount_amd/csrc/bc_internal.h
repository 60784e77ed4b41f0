// bc_internal.h — shared between the kernel file and the C-ABI file.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <string>
#include <utility>
#include <vector>

#include "basecount_hip.h"

struct bc_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    unsigned long long* d_err = nullptr;  // first out-of-range read index (atomicMin), ~0 = none
    unsigned long long* h_err = nullptr;  // pinned mirror
    bool timing = false;                  // bc_timing_enable: hipEvents around every launch
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev[BC_KERNEL_IDS];
    hipEvent_t mark[BC_EVENT_SLOTS] = {};   // bc_event_record slots (created on first use)
    hipEvent_t sig = nullptr;               // bc_ctx_wait: "everything enqueued so far"
    int32_t* rc_scratch = nullptr;         // bc_pileup's k_rc accumulation buffer, kept zeroed
    size_t rc_scratch_bytes = 0;
    void* out_scratch = nullptr;           // bc_pileup_partials without outputs: their stand-ins
    size_t out_scratch_bytes = 0;
    void* sum_scratch = nullptr;           // the read-parallel summary's leaf arrays, kept zeroed
    size_t sum_scratch_bytes = 0;
    // kernel-shape overrides (bc_ctx_set_shape); 0 = chosen from the batch
    int shape = BC_SHAPE_AUTO;
    int tile_waves = 0;
    int reads_per_block = 0;
};

// Diagnostic work-skipping switches (BC_ABLATE) exist only in -DBC_DIAG builds
// (scripts/ablate.sh); the shipped library compiles them out.
#ifdef BC_DIAG
#define BC_ABL(A) ((A).ablate)
#else
#define BC_ABL(A) 0
#endif

struct bc_graph {
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
};

namespace bc {

// Kernel-1 geometry.  One 256-thread workgroup (4 waves) per chunk of consecutive reads.
constexpr int kCountThreads = 256;
// LDS window: counts of one chunk's reads, packed two 16-bit columns per 32-bit word
// (planes {A|C, G|T, DS|N}); a chunk holds < 65536 reads so a 16-bit half never overflows.
constexpr int kWinMax = 4096;  // positions per window -> 3 * 4096 * 4 B = 48 KiB
constexpr int kNpBuf = 8192;   // numpy's default ufunc buffer size (reduction chunk)

// launchers (bc_kernels.hip); all async on `s`, return hipError_t
hipError_t launch_count(hipStream_t s, const bc_reads& r, int64_t ref_len, uint32_t mbq, int ncols,
                        int32_t* hist, int reads_per_block, unsigned long long* d_err);
size_t seq_event_bytes(int64_t seq_bytes);
hipError_t launch_seq_event(hipStream_t s, const uint8_t* src, int64_t nbytes, uint8_t* dst);
hipError_t launch_span(hipStream_t s, const bc_reads& r, int* d_max_span);
// scratch_counts_out != nullptr: hist is the context's zeroed accumulation scratch; its counts go
// to scratch_counts_out and it is zeroed again (k_stats)
hipError_t launch_stats(hipStream_t s, const int32_t* hist, int64_t L, int k, double nf, double nf2,
                        int32_t* cov, double* pc, double* ent, double* sec, int32_t* scratch_counts_out = nullptr);
// Summary partials (the per-8192-buffer sums bc_summary starts from): when the sparse sweep
// runs with `parts`, it writes those of the whole buffers [0, full_chunks) itself (fused = true).
struct SumParts {
    int32_t* hdr;  // the work buffer's header: [0] = buffers whose partials are the quarters'
    double* ent;  // per buffer
    long long* cov;
    long long* nz;
    double* sub_ent;  // per quarter buffer (2048 positions), written by the sparse sweep
    long long* sub_cov;
    long long* sub_nz;
    bool fused;
    int64_t full_chunks;  // buffers whose partials are in the quarter arrays (fused)
    // summary only (in): the sweep writes no per-position output except the coverage and entropy
    // of the positions past the whole buffers, into cov_tail / ent_tail (index P - full_chunks *
    // 8192; at most 8192 positions) for the fold's last partial buffer.  Honoured only when the
    // sweep fuses the partials (out: fused); otherwise the caller must give full outputs.
    bool no_store = false;
    bool whole_buffers = false;  // (out) the partials of [0, full_chunks) are per buffer, not per quarter
    int32_t* cov_tail = nullptr;
    double* ent_tail = nullptr;
};
// shape: BC_SHAPE_*; tile_waves: 0 = from the depth, else 1/2/4/8 waves per tile
hipError_t launch_pileup_tiles(hipStream_t s, const bc_reads& r, int64_t L, int64_t max_end, uint32_t mbq, int k,
                               bool stats, bool accumulate, double nf, double nf2, int32_t* counts, int32_t* cov,
                               double* pc, double* ent, double* sec, unsigned long long* d_err, int shape = 0,
                               int tile_waves = 0, SumParts* parts = nullptr);
// Summary only (main.py:469-499) for a sparse sorted batch: the read-parallel summary (counted
// positions per 128-position leaf, exact walks of the leaves two reads share; k_sum_buffers adds
// each 8192-position buffer's 64 leaves in numpy's tree order) into WHOLE-buffer partials
// (parts.ent / cov / nz, parts.whole_buffers set: the fold is told so through a header value of
// 0) and the tail arrays; `scratch` (>= sum_sparse_bytes(L) bytes, laid out by its capacity)
// zeroed when allocated, left zeroed (on a launch error the caller drops it).  Needs L >= kNpBuf.
size_t sum_sparse_bytes(int64_t L);
hipError_t launch_sum_sparse(hipStream_t s, const bc_reads& r, int64_t L, uint32_t mbq, int k, double nf,
                             unsigned long long* d_err, SumParts& parts, void* scratch, size_t scratch_bytes);
hipError_t launch_rc(hipStream_t s, const bc_reads& r, int64_t L, uint32_t mbq, int ncols, int32_t* counts,
                     unsigned long long* d_err);
// bc_pileup / bc_count choose the read-chunked k_rc over the tiled k_pileup when a tile would
// walk at least this many reads (deep batches; bc_ctx_set_shape overrides)
constexpr double kRcMinReadsPerTile = 2048.0;
bool use_rc(const bc_reads& r, int64_t L, int shape);
constexpr int kTileMaxSpan = 4096;  // beyond this span the tiled kernel's look-back gets too long
// the tiled kernels: waves per 64-position tile from the depth (1 = the sparse sweep k_pileup_solo)
int pileup_waves(const bc_reads& r, int64_t L, int64_t max_end, int tile_waves);
inline bool pileup_is_solo(const bc_reads& r, int64_t L, int shape, int tile_waves) {
    return shape != BC_SHAPE_TILE_NO_SOLO && pileup_waves(r, L, r.max_end, tile_waves) == 1;
}

// ---- the coordinate-sorted copy of an unsorted batch (bc_sort.hip) ----
// fields: sort only the per-read fields (+ run records) and leave the sequence where it is (k_rc
// stages a chunk's scattered reads by LDS-DMA gathers); else copy the sequence (and qualities)
// into start order as well
size_t sort_bytes(const bc_reads& r, bool fields);
// enqueues the sort into mem (sort_bytes(r, fields) bytes; stream-ordered, no host round trip)
// and fills `out` (sorted; no index, or with fields the run records); needs sort_fits(r)
hipError_t launch_sort(hipStream_t s, const bc_reads& r, bc_reads& out, void* mem, bool fields);
bool sort_fits(const bc_reads& r);
// device word of caller errors (read after a sync): bit 0 the reads' sequences overlap (the copy
// did not fit), bit 1 a start outside [0, max_end]
const uint32_t* sort_flags_word(const bc_reads& r, const void* mem);

// ---- the device index of a sorted batch (bc_index.hip) ----
// bc_reads.index_tag: the batch identity an index was built for (never 0)
inline uint64_t index_tag(const bc_reads& r) {
    uint64_t h = 0x243F6A8885A308D3ull;
    auto mix = [&h](uint64_t v) { h ^= v + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2); };
    mix((uint64_t)r.n_reads);
    mix((uint64_t)(uint32_t)r.sorted);
    mix((uint64_t)(uint32_t)r.max_span);
    mix((uint64_t)r.max_end);
    mix((uint64_t)(uintptr_t)r.pos);
    mix((uint64_t)(uintptr_t)r.cig_beg);
    return h | 1u;
}
inline bool index_valid(const bc_reads& r) { return r.index_tag != 0 && r.index_tag == index_tag(r); }
struct IndexPlan {
    size_t runs_bytes = 0, sums_bytes = 0, tiles_bytes = 0, total = 0;
    int64_t n_chunks = 0, n_tiles = 0;
};
// what = BC_INDEX_RUNS | BC_INDEX_TILES (AUTO resolved by the caller)
IndexPlan index_plan(const bc_reads& r, int what);
// builds the planned parts into mem (plan.total bytes) and sets r's index fields and tag
hipError_t launch_index(hipStream_t s, bc_reads& r, const IndexPlan& plan, void* mem);
size_t summary_work_bytes(int64_t L);
hipError_t launch_summary(hipStream_t s, const int32_t* cov, const double* ent, int64_t L, void* work,
                          double* out, int64_t first_chunk = 0);
// (quarters: the buffers before first_chunk come as quarter partials, else as whole-buffer ones)
hipError_t launch_summary_partials(hipStream_t s, const int32_t* cov, const double* ent, int64_t L, void* work,
                                   int64_t first_chunk, bool quarters = true);
// (the work buffers' headers say which leading buffers come as quarters)
hipError_t launch_summary_fold(hipStream_t s, int n, const int64_t* L, void* const* work, double* const* out);
// the partial arrays inside a summary work buffer
SumParts summary_parts(void* work, int64_t L);
hipError_t launch_amplicons(hipStream_t s, const int32_t* cov, const double* ent, const double* sec,
                            int64_t L, const int64_t* lo, const int64_t* hi, int n_tiles, double* out);
// The fused --summarise-with-bed tail (bc_pileup_summary_amplicons): kernel 2 that also writes
// numpy's 128-position leaf partials into the summary work buffer, then ONE launch for the
// summary (out: mean coverage, mean entropy, non-zero positions, coverage sum) and every
// amplicon window (amp: 6 doubles per window)
hipError_t launch_stats_leaves(hipStream_t s, int32_t* hist, int64_t L, int k, double nf, double nf2, int32_t* cov,
                               double* ent, double* sec, int32_t* counts_out, void* work);
hipError_t launch_tail(hipStream_t s, const int32_t* cov, const double* ent, const double* sec, int64_t L, void* work,
                       double* out, const int64_t* lo, const int64_t* hi, int n_tiles, double* amp);

}  // namespace bc
