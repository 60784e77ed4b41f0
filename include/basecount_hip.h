/*
 * basecount_hip.h — C-ABI of the MI355X (gfx950) pileup counter.
 *
 * This is the drop-in boundary for the reference's only native operator:
 *
 *     count.bcount(refLen, minBaseQuality, reads, qualities, starts, ctuples)
 *         -> list[list[int]]   (refLen x 6: A, C, G, T, DS, N)
 *
 *   defined at /root/reference/basecount/count.cpp:7-99, exported at count.cpp:102-105,
 *   built as the top-level module `count` by /root/reference/setup.py:5 and called from
 *   /root/reference/basecount/main.py:146-153 and :179-186,
 *
 * plus the per-position statistics the reference computes in Python right after it
 * (get_stats / get_entropy, /root/reference/basecount/main.py:10-79) and the summary /
 * amplicon reductions of main.py:469-595.
 *
 * Conventions
 *   - Every function returns BC_OK (0) or a negative BC_E_* status; bc_last_error() gives the
 *     message of the calling thread's last failure.
 *   - Pointers named d_* are device (HBM) pointers, h_* are host pointers.  Device buffers passed
 *     in are caller-owned; buffers created by bc_reads_upload()/bc_malloc() are library-owned and
 *     released with bc_reads_free()/bc_free().
 *   - Compute calls are stream-ordered and asynchronous on the context's stream; bc_sync() blocks.
 *     No compute call allocates or synchronises, so a sequence of them can be captured into a
 *     hipGraph (bc_graph_* below).
 *   - Nothing here falls back to the CPU: without a gfx950 device, bc_ctx_create() fails.
 */
#ifndef BASECOUNT_HIP_H
#define BASECOUNT_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BC_OK 0
#define BC_E_ARG (-1)   /* invalid argument (mirrors pybind11's TypeError on bad bcount args)   */
#define BC_E_HIP (-2)   /* HIP runtime error                                                     */
#define BC_E_RANGE (-3) /* a counted event fell outside [0, refLen) (count.cpp:60-65,85 .at())   */
#define BC_E_NODEV (-4) /* no usable gfx950 device                                               */
#define BC_E_COMM (-5)  /* RCCL error in a multi-GPU call                                        */

#define BC_ABI_VERSION 8

/* Layouts of bc_reads.seq.
 *   BC_SEQ_BAM   BAM packing: "=ACMGRSVTWYHKDBN" codes, two per byte, high nibble first
 *                (what the host decoder produces; bc_reads_upload/bc_bcount_host inputs).
 *   BC_SEQ_EVENT the device layout of the tiled kernel: one nibble per base in LINEAR order
 *                (base i at bits 4*(i%8) of little-endian 32-bit word i/8), pre-classified to
 *                event classes  A 0001, C 0010, G 0100, T 1000, N 0011, not counted 0000
 *                (count.cpp:58-65 through pysam's decode: '=' and IUPAC codes count nowhere).
 *                The buffer must hold bc_seq_event_bytes(seq_bytes) bytes (zero padding).
 * bc_reads_upload produces BC_SEQ_EVENT; bc_seq_to_event converts a device buffer in place. */
#define BC_SEQ_BAM 0
#define BC_SEQ_EVENT 1

/* A batch of pre-decoded, accepted reads of ONE reference, struct-of-arrays.
 * For read i (all fields as the reference's bcount sees them, count.cpp:22-38):
 *   starts[i]  = pos[i]                              (0-based reference_start)
 *   ctuples[i] = cigar[cig_beg[i] .. cig_beg[i]+cig_n[i])   BAM words: len << 4 | op
 *   reads[i][j]     = SEQ nibble at index seq_nib[i] + j    (layout: seq_layout, BC_SEQ_*)
 *   qualities[i][j] = qual[seq_nib[i] + j]                  (qual is indexed by nibble index)
 * i.e. seq_nib already includes the query_alignment_start (soft-clip) offset.
 * The same struct describes host arrays (bc_reads_upload input, bc_bcount_host) and device
 * arrays (bc_count input).                                                                     */
typedef struct bc_reads {
    int64_t n_reads;
    const int32_t* pos;
    const uint32_t* cig_beg;
    const uint32_t* cig_n;
    const uint32_t* seq_nib;
    const uint32_t* cigar;
    int64_t n_cigar_words;
    const uint8_t* seq;
    int64_t seq_bytes;
    const uint8_t* qual;      /* may be NULL; then minBaseQuality must be 0                    */
    int64_t qual_bytes;       /* >= 2*seq_bytes when qual != NULL                              */
    int32_t sorted;           /* 1 if pos[] is non-decreasing (enables the tiled kernel)       */
    int32_t max_span;         /* upper bound of every read's reference span (M/D/N/=/X bases)  */
    int64_t max_end;          /* upper bound of pos[i] + span[i] over the batch                */
    int32_t seq_layout;       /* BC_SEQ_BAM or BC_SEQ_EVENT                                    */
    int32_t run_chunks;       /* chunk summaries after the run records (see read_runs), or 0   */
    /* Optional device index of a sorted batch (NULL / 0: the tiled kernel searches pos[]).  For
     * the 64-position tile t < n_tiles, tile_reads[2t] and tile_reads[2t+1] are the reads
     * [lo, hi) that can overlap it: lo = first i with pos[i] > 64t - max_span, hi = first i with
     * pos[i] >= 64t + 64 (so valid for this max_span only).  Built on the device by
     * bc_reads_upload / bc_reads_index (k_index_tiles) for dense batches (fewer tiles than
     * reads/16, fewer than 2^31 reads); host inputs ignore it.                                  */
    const int32_t* tile_reads;
    int64_t n_tiles;
    /* Optional device run records of a sorted batch (NULL: the kernels decode the CIGARs): 4
     * words per read, the first two aligned runs of its CIGAR as the read-chunked kernel needs
     * them (layout in basecount_amd/csrc/bc_runs.h).  Built on the device by bc_reads_upload /
     * bc_reads_index (k_index_runs: the same decode the kernels run) for sorted batches that
     * take the read-chunked kernel; host inputs ignore it.
     * When run_chunks > 0, read_runs[4 n_reads ..] then holds run_chunks summaries of 8 words,
     * one per 256 consecutive reads (the read-chunked kernel's chunk): min start, max end,
     * first / last-plus-one byte of their aligned sequence, max span, a run-shape code and a
     * deletion flag over the reads with simple CIGARs (bc_runs.h: chunk_summary).              */
    const uint32_t* read_runs;
    /* Identity of the batch the index above was built for (bc_reads_upload / bc_reads_index):
     * a hash of n_reads, sorted, max_span, max_end and the pos / cig_beg pointers.  The kernels
     * use tile_reads / read_runs only while it matches, so a copied struct that was sliced (pos
     * offset, n_reads shrunk) or given another max_span falls back to searching / decoding
     * instead of reading another batch's index.  0 = no index.
     * The tag detects slicing, not new CONTENT in the same buffers: a caller that refills the
     * arrays of a struct in place (same pointers, same counts and bounds) must set index_tag = 0
     * or rebuild the index (bc_reads_index) before the next launch.                          */
    uint64_t index_tag;
} bc_reads;

typedef struct bc_ctx bc_ctx;

const char* bc_last_error(void);
int bc_abi_version(void);
/* Build description, e.g. "gfx950 diag=0 phase_trace=0": diag=1 marks a diagnostic build whose
 * kernels can skip work on request (BC_ABLATE); bench.py refuses to report numbers from one.    */
const char* bc_build_info(void);
int bc_device_count(int* n);

/* Create a context on `device`.  `stream` is a hipStream_t (NULL: the library creates and owns
 * a non-blocking stream).  The context holds only small scratch state (the range-error word).   */
int bc_ctx_create(int device, void* stream, bc_ctx** out);
int bc_ctx_destroy(bc_ctx* ctx);
int bc_ctx_stream(bc_ctx* ctx, void** stream);
/* Give back the context's grow-only device scratch (bc_pileup's k_rc accumulation buffer,
 * bc_pileup_partials' stand-in outputs and the read-parallel summary's leaf arrays) after
 * finishing the work enqueued on its stream; the next call that needs one allocates it again
 * (outside any graph capture).  The context stays usable.                                      */
int bc_ctx_release_scratch(bc_ctx* ctx);

/* Kernel-shape selection for bc_count / bc_pileup on this context (parity tests and tuning; no
 * shape skips work, every one computes the same counts).  The default, BC_SHAPE_AUTO, picks
 * from the batch's depth:
 *   BC_SHAPE_TILE         tiled k_pileup, or its sparse sweep k_pileup_solo (read-chunked k_rc
 *                         only for spans > 4096)
 *   BC_SHAPE_RC           read-chunked k_rc (+ k_stats) for every sorted batch
 *   BC_SHAPE_TILE_NO_SOLO tiled k_pileup, never the sparse sweep
 * tile_waves: 0 = from the depth, else 1, 2, 4 or 8 waves per 64-position tile (BC_E_ARG
 * otherwise).  reads_per_block: 0 = automatic, else 1..32768 reads per k_count workgroup
 * (unsorted batches).                                                                          */
#define BC_SHAPE_AUTO 0
#define BC_SHAPE_TILE 1
#define BC_SHAPE_RC 2
#define BC_SHAPE_TILE_NO_SOLO 3
int bc_ctx_set_shape(bc_ctx* ctx, int shape, int tile_waves, int reads_per_block);
int bc_sync(bc_ctx* ctx);

/* Library-owned device memory helpers (for hosts without another allocator). */
int bc_malloc(bc_ctx* ctx, size_t bytes, void** d_ptr);
int bc_free(bc_ctx* ctx, void* d_ptr);
int bc_memcpy_h2d(bc_ctx* ctx, void* d_dst, const void* h_src, size_t bytes);  /* async */
int bc_memcpy_d2h(bc_ctx* ctx, void* h_dst, const void* d_src, size_t bytes);  /* async */
int bc_memset(bc_ctx* ctx, void* d_dst, int value, size_t bytes);              /* async */

/* Bytes a BC_SEQ_EVENT buffer needs for seq_bytes bytes of packed sequence. */
size_t bc_seq_event_bytes(int64_t seq_bytes);
/* Convert BAM-packed sequence (device) to BC_SEQ_EVENT: d_event (bc_seq_event_bytes bytes) may
 * alias d_bam.  Async on the context's stream.                                                */
int bc_seq_to_event(bc_ctx* ctx, const uint8_t* d_bam, int64_t seq_bytes, uint8_t* d_event);

/* Copy a host batch to HBM (library-owned, BC_SEQ_EVENT on the device).  A BC_SEQ_EVENT host
 * batch (the layout the host decoder already emits, bcio_records.seq_event) is copied as is; a
 * BC_SEQ_BAM one is converted on the device after the copy (k_seq_event).  `sorted`,
 * `max_span` and `max_end` of the device batch are derived from the data (the host's values
 * are ignored).  For batches assembled directly in
 * device memory the caller must set both truthfully: the tiled kernel trusts them.           */
int bc_reads_upload(bc_ctx* ctx, const bc_reads* h_reads, bc_reads* d_reads);
int bc_reads_free(bc_ctx* ctx, bc_reads* d_reads);

/* The device index of a sorted batch assembled in device memory by the caller (e.g. one
 * reference's slice of a file-wide upload), built ON THE DEVICE into caller-owned memory:
 *   BC_INDEX_RUNS   run records + k_rc chunk summaries (read_runs, run_chunks)
 *   BC_INDEX_TILES  the tile index (tile_reads, n_tiles; dense batches only)
 *   BC_INDEX_AUTO   what this context's kernels would use for a reference of length ref_len
 *                   (records for the read-chunked shape, tiles for the tiled one, nothing for
 *                   the sparse sweep)
 * bc_reads_index_bytes gives the bytes d_mem must hold (0: nothing to build); bc_reads_index
 * launches the build on the context's stream (async, no allocation: capturable) and sets the
 * index fields and index_tag of *d_reads.  d_reads->sorted / max_span / max_end must be
 * truthful.  bc_reads_upload builds BC_INDEX_AUTO for ref_len = max_end into its own slab.    */
/* A coordinate-sorted copy of an unsorted device batch, built on the device (bc_sort.hip):
 * the reads bucketed by start (per-block LDS histograms, one block per bucket ordering it), their
 * per-read arrays written in start order and each read's aligned sequence (and qualities) copied
 * so that consecutive reads have consecutive sequence again.  The copy shares d_reads' CIGAR
 * buffer; everything else lives in d_mem (bc_reads_sort_bytes bytes, 256-byte aligned), which
 * must outlive its use.  *d_sorted is then a sorted batch (sorted = 1, same max_span / max_end,
 * no index: build one with bc_reads_index) that every kernel takes, with the same counts as the
 * input (count.cpp's sums do not depend on the read order).  Needs seq_layout == BC_SEQ_EVENT
 * and seq_bytes + 5 n_reads + 16 <= 0x55555550 (BC_E_ARG otherwise: split the batch).
 * Stream-ordered and capturable (round 6): the call only enqueues four kernels; every layout
 * decision is taken on the device, so there is no host round trip and no fallback path.
 * Caller errors that only the device can see -- a read starting outside [0, max_end], reads whose
 * aligned sequences overlap so that the copy would not fit -- leave a flag in d_mem (the sorted
 * copy stays safe to count: such reads start at 0 / carry no CIGAR): bc_reads_sort_check waits
 * for the stream and returns BC_E_ARG with the reason if a flag is set, BC_OK otherwise.      */
int bc_reads_sort_bytes(bc_ctx* ctx, const bc_reads* d_reads, size_t* bytes);
int bc_reads_sort(bc_ctx* ctx, const bc_reads* d_reads, bc_reads* d_sorted, void* d_mem, size_t bytes);
int bc_reads_sort_check(bc_ctx* ctx, const bc_reads* d_reads, const void* d_mem);

#define BC_INDEX_RUNS 1
#define BC_INDEX_TILES 2
#define BC_INDEX_AUTO 4
int bc_reads_index_bytes(bc_ctx* ctx, const bc_reads* d_reads, int64_t ref_len, int what, size_t* bytes);
int bc_reads_index(bc_ctx* ctx, bc_reads* d_reads, int64_t ref_len, int what, void* d_mem, size_t bytes);

/* Kernel 1 — CIGAR-expand + scatter-add (count.cpp:22-97).
 * Accumulates into d_hist, an int32 histogram of `ncols` planes of `ref_len` positions
 * (plane-major: d_hist[c * ref_len + p]).  ncols = 6 gives the reference's full layout
 * (A,C,G,T,DS,N); ncols = 5 drops N (main.py:19-31 never uses it unless show_n_bases).
 * M/=/X bases with qual >= min_base_quality count A/C/G/T/N; other letters count nowhere;
 * I advances the read; D/N-skip count DS with no quality test; S/H/P/B are no-ops.
 * A counted event at position >= ref_len is recorded (first offending read index kept);
 * read it with bc_range_error().  Async; does not zero d_hist.                               */
int bc_count(bc_ctx* ctx, const bc_reads* d_reads, int64_t ref_len, uint32_t min_base_quality,
             int ncols, int32_t* d_hist);

/* Fused kernel 1 + kernel 2 — the hot path in ONE launch.  For a coordinate-sorted batch
 * (d_reads->sorted == 1, max_span / max_end truthful) the reference is cut into
 * 64-position tiles; each tile finds its reads by a search over pos[], walks them with lanes
 * owning 8-position windows and SWAR register counters (no atomics, no histogram memset;
 * needs seq_layout == BC_SEQ_EVENT), and writes
 *   d_counts [k][L] int32 (the reference's baseCounts columns, N only when k == 6),
 *   d_cov, d_pc (may be NULL), d_ent, d_sec  exactly as bc_stats defines them.
 * Deep batches (many reads per tile) and spans > 4096 instead run the read-chunked kernel 1
 * (each read decoded once, per-block LDS event image / histograms, atomic flush into a
 * context-owned scratch kept zeroed) followed by kernel 2, which moves the counts to d_counts
 * and re-zeroes the scratch: two stream-ordered launches, same results.  The scratch grows on
 * first use for a larger k * ref_len (a synchronizing allocation: make that first call outside
 * a graph capture).
 * Out-of-range counted events are recorded for bc_range_error() as with bc_count.
 * Overwrites its outputs; async; capturable.                                                   */
int bc_pileup(bc_ctx* ctx, const bc_reads* d_reads, int64_t ref_len, uint32_t min_base_quality, int k,
              double nf, double nf2, int32_t* d_counts, int32_t* d_cov, double* d_pc, double* d_ent,
              double* d_sec);

/* hipGraph capture of a sequence of compute calls on the context's stream (the context must own
 * its stream or have been given a non-default one).  bc_graph_end instantiates the graph;
 * bc_graph_launch replays it on the context's stream.                                         */
typedef struct bc_graph bc_graph;
int bc_graph_begin(bc_ctx* ctx);
int bc_graph_end(bc_ctx* ctx, bc_graph** out);
int bc_graph_launch(bc_ctx* ctx, bc_graph* g);
int bc_graph_destroy(bc_graph* g);

/* Stream order between two contexts of one device: ctx's later work waits for everything enqueued
 * on other's stream so far (an event, no host wait).  Independent references can then run on
 * several contexts' streams at once, e.g. inside a capture begun on `main`: fork with
 * bc_ctx_wait(side, main), enqueue on each, join with bc_ctx_wait(main, side).                */
int bc_ctx_wait(bc_ctx* ctx, bc_ctx* other);

/* Per-kernel timing (SURVEY §5 tracing): when enabled, every launch made through the context is
 * bracketed by hipEvents on its stream.  bc_timing_report() synchronises and returns, per kernel
 * id (BC_K_*), the number of timed launches and their mean duration in microseconds, then clears
 * the record.  Do not enable while capturing a graph.                                          */
#define BC_K_COUNT 0      /* event-parallel kernel 1 (unsorted / long-span batches) */
#define BC_K_STATS 1      /* kernel 2                                              */
#define BC_K_RC 2         /* read-chunked kernel 1 (deep sorted batches)           */
#define BC_K_PILEUP 3     /* fused tiled kernel 1 + 2                              */
#define BC_K_SUMMARY 4
#define BC_K_AMPLICONS 5
#define BC_K_INDEX 6      /* the device index build (bc_reads_index / bc_reads_upload)  */
#define BC_K_SOLO 7       /* the sparse sweep k_pileup_solo (fused kernel 1 + 2)     */
#define BC_K_SORT 8       /* the device sort of an unsorted batch (bc_reads_sort)     */
#define BC_KERNEL_IDS 9
int bc_timing_enable(bc_ctx* ctx, int on);
int bc_timing_report(bc_ctx* ctx, int64_t* launches /* [BC_KERNEL_IDS] */, double* mean_us /* [..] */);

/* Region timing: bc_event_record(ctx, slot) records hipEvent `slot` (0 .. BC_EVENT_SLOTS-1) on the
 * context's stream; bc_event_elapsed_ms synchronises on the later one and returns the time
 * between two recorded slots.  Measures a whole sequence of launches (e.g. K steps) on-device. */
#define BC_EVENT_SLOTS 4
int bc_event_record(bc_ctx* ctx, int slot);
int bc_event_elapsed_ms(bc_ctx* ctx, int slot0, int slot1, float* ms);

/* Blocking: returns the smallest read index that produced an out-of-range counted event since
 * the last call (or -1) and clears the record.                                                 */
int bc_range_error(bc_ctx* ctx, int64_t* first_bad_read);

/* Kernel 2 — per-position statistics (main.py:14-79), fp64, same operation order as CPython:
 *   cov = sum(c);  pc_j = 100 * (c_j / cov);  H = nf * sum_j -(p_j*log2(p_j)) [p_j != 0];
 *   H2 = nf2 * (same over the counts with the first argmax removed, over cov - max).
 * k = 5 (A,C,G,T,DS) or 6 (+N, show_n_bases); planes 0..k-1 of d_hist are used.
 * Outputs (device, caller-owned; any of d_pc / d_ent / d_sec may be NULL to skip):
 *   d_cov [L] int32, d_pc [k][L] f64, d_ent [L] f64, d_sec [L] f64.
 * Where cov == 0 the reference emits ints (-1 / 1 / 1): here pc = -1.0, H = H2 = 1.0.
 * Where cov2 == 0 the reference emits int 1 for H2: here 1.0.                                 */
int bc_stats(bc_ctx* ctx, const int32_t* d_hist, int64_t ref_len, int k, double nf, double nf2,
             int32_t* d_cov, double* d_pc, double* d_ent, double* d_sec);

/* Summary reductions of one reference (main.py:469-495), bit-identical to numpy:
 *   out[0] = np.mean(coverages)     out[1] = np.mean(entropies)
 *   out[2] = number of positions with coverage != 0 (as double, exact)
 *   out[3] = sum of coverages (exact, as double when < 2^53)
 * numpy's float64 add.reduce is emulated exactly: 8192-element buffer chunks added left to right,
 * each chunk summed by numpy's pairwise_sum (8-way unrolled leaves of <= 128).  d_out: 4 doubles,
 * device memory.  d_work must hold bc_summary_work_bytes(ref_len) bytes.                     */
size_t bc_summary_work_bytes(int64_t ref_len);
int bc_summary(bc_ctx* ctx, const int32_t* d_cov, const double* d_ent, int64_t ref_len,
               void* d_work, double* d_out);

/* Fused pileup + summary (main.py:469-499's numbers for one reference, as bc_pileup followed by
 * bc_summary, bit-identical): for sparse batches the pileup sweep computes numpy's per-buffer
 * partial sums while the statistics are still in registers, so the per-position coverage and
 * entropies are not read back; other batches run bc_pileup + bc_summary.  Arguments as bc_pileup
 * (all per-position outputs written) plus d_work (bc_summary_work_bytes(ref_len)) and d_out (4
 * doubles, as bc_summary).  ref_len must be > 0.                                              */
int bc_pileup_summary(bc_ctx* ctx, const bc_reads* d_reads, int64_t ref_len, uint32_t min_base_quality, int k,
                      double nf, double nf2, int32_t* d_counts, int32_t* d_cov, double* d_pc, double* d_ent,
                      double* d_sec, void* d_work, double* d_out);
/* The same in two parts, for several references: bc_pileup_partials leaves numpy's per-buffer
 * partial sums of one reference in d_work; bc_summary_fold then folds n references' partials
 * (one workgroup each, side by side: the fold is one dependent add per 8192 positions, the only
 * sequential step of the summary) and writes each reference's 4 doubles to d_outs[i].
 * ref_lens / d_works / d_outs are host arrays of n entries (device pointers).
 * Summary only: with d_counts, d_cov, d_pc, d_ent and d_sec ALL NULL, bc_pileup_partials (and
 * bc_pileup_summary) write no per-position output (the CLI's --summarise prints six numbers per
 * reference): a sparse batch's sweep writes only the summary partials (and the coverage /
 * entropy of the last partial 8192-position buffer, into context scratch); other batches write
 * their outputs into context scratch.  Same numbers, bit for bit.  The scratch grows on first use
 * (a synchronizing allocation: make that call outside a graph capture).                        */
int bc_pileup_partials(bc_ctx* ctx, const bc_reads* d_reads, int64_t ref_len, uint32_t min_base_quality, int k,
                       double nf, double nf2, int32_t* d_counts, int32_t* d_cov, double* d_pc, double* d_ent,
                       double* d_sec, void* d_work);
int bc_summary_fold(bc_ctx* ctx, int n, const int64_t* ref_lens, void* const* d_works, double* const* d_outs);

/* Amplicon vectors (main.py:501-551): for each tile t with inclusive window
 * [lo[t], hi[t]] (already clipped to [0, ref_len-1]; lo > hi = empty), np.mean and np.median of
 * coverage, entropy and secondary entropy over the window.  d_out: [n_tiles][6] f64 device
 * (mean_cov, median_cov, mean_ent, median_ent, mean_sec, median_sec); empty tiles give -1.0. */
int bc_amplicons(bc_ctx* ctx, const int32_t* d_cov, const double* d_ent, const double* d_sec,
                 int64_t ref_len, const int64_t* d_lo, const int64_t* d_hi, int32_t n_tiles,
                 double* d_out);

/* --summarise-with-bed for one reference (main.py:469-551): bc_pileup_summary and bc_amplicons
 * in one call, same numbers bit for bit.  For a deep batch (the read-chunked k_rc) the tail after
 * kernel 1 is two launches: kernel 2 that also leaves numpy's 128-position leaf partials in
 * d_work, and ONE launch for the summary fold and every window's means and medians (instead of
 * kernel 2, the summary's chunk sums, its fold and the amplicon kernel); other batches run
 * bc_pileup_summary + bc_amplicons.  Arguments as those two (d_counts, d_cov, d_ent and d_sec all
 * non-NULL: the windows read them; no percentages), n_tiles >= 0.                             */
int bc_pileup_summary_amplicons(bc_ctx* ctx, const bc_reads* d_reads, int64_t ref_len, uint32_t min_base_quality,
                                int k, double nf, double nf2, int32_t* d_counts, int32_t* d_cov, double* d_ent,
                                double* d_sec, void* d_work, double* d_out, const int64_t* d_lo,
                                const int64_t* d_hi, int32_t n_tiles, double* d_amp);

/* ---- Multi-GPU: one process per GPU, RCCL over xGMI ---------------------------
 * Counting needs no exchange: references are independent, so each rank owns whole references
 * and runs the single-GPU path on them.  What crosses GPUs is small: the per-reference results
 * the reference prints (main.py:469-595) gathered to rank 0, the reference order rank 0 chose
 * (main.py:92 iterates a set, whose order is per process), and every reference's first
 * out-of-range read (so all ranks raise the reference's first error).  The reference itself has
 * no collective: this replaces nothing in it, it is what lets its per-reference loop
 * (main.py:130-205) run on N GPUs.
 * Rendezvous: rank 0 calls bc_comm_unique_id and hands the BC_COMM_ID_BYTES bytes to the other
 * ranks out of band (basecount_amd/dist.py: a TCP socket next to MASTER_ADDR:MASTER_PORT); then
 * every rank calls bc_comm_init with its own context (one GPU per rank).  Every call below but
 * bc_gather_layout is collective: all ranks make it, in the same order.  Collectives run on the
 * context's stream; the bc_*_bytes / _i64 / barrier calls are blocking, bc_gather_dev is
 * stream-ordered and asynchronous.                                                            */
#define BC_COMM_ID_BYTES 128
typedef struct bc_comm bc_comm;
int bc_comm_unique_id(uint8_t* id /* [BC_COMM_ID_BYTES] */);
int bc_comm_init(bc_ctx* ctx, const uint8_t* id, int rank, int world, bc_comm** out);
int bc_comm_destroy(bc_comm* comm);
int bc_comm_rank(const bc_comm* comm, int* rank, int* world);
int bc_comm_barrier(bc_comm* comm);
/* h_recv[r * n + i] = rank r's h_send[i] (n is the same on every rank). */
int bc_allgather_i64(bc_comm* comm, const int64_t* h_send, int64_t n, int64_t* h_recv);
/* root's n bytes to every rank (n the same on every rank). */
int bc_broadcast_bytes(bc_comm* comm, void* h_buf, int64_t n, int root);
/* Ragged gather layout (host arithmetic, no GPU): offsets[r] = sum of sizes[0..r),
 * offsets[world] = total.  BC_E_ARG on a negative size or an overflowing total.             */
int bc_gather_layout(const int64_t* sizes, int world, int64_t* offsets /* [world + 1] */);
/* Ragged gather to `root`: rank r sends n_r bytes; sizes[0..world) holds every n_r on every rank
 * (exchange them first with bc_allgather_i64).  On root the payloads land concatenated in rank
 * order at bc_gather_layout's offsets; other ranks' receive pointers are ignored.
 *   bc_gather_bytes: host buffers, blocking (h_recv: offsets[world] bytes on root).
 *   bc_gather_dev:   device buffers, stream-ordered on the context's stream, capturable.       */
int bc_gather_bytes(bc_comm* comm, const void* h_send, int64_t n, void* h_recv, const int64_t* sizes, int root);
int bc_gather_dev(bc_comm* comm, const void* d_send, int64_t n, void* d_recv, const int64_t* sizes, int root);
/* One reference's reads split over the ranks (a single contig on N GPUs): every
 * rank's int32 histogram [n] summed into root's d_recv (may alias d_send; ignored off the root).
 * Device buffers, stream-ordered on the context's stream, capturable (RCCL reduce over xGMI). */
int bc_reduce_i32_dev(bc_comm* comm, const int32_t* d_send, int32_t* d_recv, int64_t n, int root);

/* Drop-in for count.bcount with host buffers: uploads, counts all 6 columns, downloads.
 * h_out: refLen x 6 uint32, ROW-major like the reference's vector<vector<unsigned>>
 * (h_out[p*6 + c]).  On BC_E_RANGE, *bad_read / *bad_pos give the first offending read (in
 * read order) and the refPos the reference's .at() would have rejected (count.cpp:60-65,85). */
int bc_bcount_host(int device, int64_t ref_len, uint32_t min_base_quality, const bc_reads* h_reads,
                   uint32_t* h_out, int64_t* bad_read, int64_t* bad_pos);

#ifdef __cplusplus
}
#endif
#endif
