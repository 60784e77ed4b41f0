/*
 * bcio.h — host-side BAM I/O and byte-exact text formatting for basecount_amd.
 *
 * This is the step BEFORE and AFTER the GPU hot path:
 *
 *   - BGZF inflate (multi-threaded, zlib) + BAM record decode into a struct-of-arrays that is
 *     uploaded to HBM unchanged.  It replaces the pysam iteration the reference performs at
 *     /root/reference/basecount/main.py:119-127 and the per-read field extraction at
 *     main.py:165-173 (query_alignment_sequence / _qualities, reference_start, cigartuples).
 *   - A BGZF/BAM writer used by the synthetic-input generator (configs C1..C5).
 *   - A formatter that reproduces `str(round(x, dp))` (main.py:457-466) byte for byte.
 *
 * Plain C ABI: no torch, no Python types.  All arrays are owned by the library handle and stay
 * valid until bcio_close().  Every function returns 0 on success or a negative BCIO_E_* code;
 * bcio_last_error() returns a message for the calling thread.
 */
#ifndef BCIO_H
#define BCIO_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BCIO_OK 0
#define BCIO_E_IO (-1)      /* file cannot be opened / read / written              */
#define BCIO_E_FORMAT (-2)  /* not BGZF / not BAM / truncated record                */
#define BCIO_E_ZLIB (-3)    /* inflate/deflate failure                             */
#define BCIO_E_ARG (-4)     /* bad argument                                        */

/* Per-record status bits (bcio_records.rec_err).  They mirror what the reference would raise
 * when the record is handed to count.bcount (SURVEY.md §8 notes):                            */
#define BCIO_REC_NO_CIGAR 1u   /* n_cigar == 0  -> cigartuples is None  -> TypeError            */
#define BCIO_REC_NO_SEQ 2u     /* l_seq == 0    -> query_alignment_sequence None -> TypeError    */
#define BCIO_REC_NO_QUAL 4u    /* QUAL[0]==0xFF -> query_alignment_qualities None -> TypeError   */
#define BCIO_REC_BAD_CLIP 8u   /* pysam getQueryStart/End raise ValueError('Invalid clipping')  */
#define BCIO_REC_NEG_POS 16u   /* mapped record with pos < 0 -> pybind11 uint conversion error  */

typedef struct bcio_file bcio_file;

/* All records of a BAM file, in file order ("raw" view, nothing filtered). */
typedef struct bcio_records {
    int64_t n;              /* number of records                                             */
    const int32_t* tid;     /* [n] reference id, -1 = none                                   */
    const int32_t* pos;     /* [n] 0-based leftmost reference position                       */
    const uint16_t* flag;   /* [n]                                                           */
    const uint8_t* mapq;    /* [n]                                                           */
    const int32_t* l_seq;   /* [n] query length (full SEQ, soft clips included)               */
    const int32_t* qstart;  /* [n] pysam query_alignment_start                                */
    const int32_t* qend;    /* [n] pysam query_alignment_end                                  */
    const uint32_t* rec_err;/* [n] BCIO_REC_* bits                                            */
    const uint64_t* cig_off;/* [n+1] CSR into cigar                                           */
    const uint32_t* cigar;  /* BAM-native words: len<<4 | op                                  */
    const uint64_t* seq_off;/* [n+1] byte CSR into seq (each record's packed SEQ, 2 bases/B)  */
    const uint8_t* seq;     /* packed 4-bit SEQ, high nibble first (BAM order)                */
    const uint8_t* qual;    /* QUAL laid out by NIBBLE index: base i of record r is at
                               qual[2*seq_off[r] + i]  (so one offset addresses both)         */
    uint64_t seq_bytes;     /* = seq_off[n]                                                   */
    const int64_t* ref_span;/* [n] reference span: sum of M/D/N/=/X lengths                     */
    const uint8_t* seq_event;/* the same SEQ bytes in the kernels' BC_SEQ_EVENT layout
                                (basecount_hip.h): byte m of a record = its bases 2m (low
                                nibble) and 2m+1 (high), pre-classified; built during the
                                decode so the upload needs no device conversion pass          */
    uint64_t seq_event_bytes;/* seq_bytes rounded up to 16, plus 16 zero bytes (padding)       */
} bcio_records;

/* Open and fully decode a BAM file with `nthreads` inflate/decode threads (<=0: hardware). */
int bcio_open(const char* path, int nthreads, bcio_file** out);
void bcio_close(bcio_file* f);
const char* bcio_last_error(void);

int32_t bcio_n_refs(const bcio_file* f);
const char* bcio_ref_name(const bcio_file* f, int32_t i);
int64_t bcio_ref_len(const bcio_file* f, int32_t i);
int bcio_get_records(const bcio_file* f, bcio_records* out);

/* Per-reference selection of the reads the reference's read loop accepts
 * (main.py:165: `not read.is_unmapped and read.mapping_quality >= min_mapping_quality`).
 * `ref_sel[tid]` != 0 marks references that were requested.  Produces, per requested reference,
 * the read-index arrays of the GPU batch format (see basecount_hip.h, bc_reads):
 *     pos[i], cig_beg[i], cig_n[i], seq_nib[i] (= 2*seq_off[rec] + qstart[rec]), qlen[i],
 *     ordinal[i] (global accepted-read ordinal, used only for error ordering), rec[i].
 * Arrays for reference t are at offset ref_beg[t] .. ref_beg[t+1] of the flat outputs.
 * keyerror_ordinal = ordinal of the first accepted read whose reference is not requested
 * (reference raises KeyError there, main.py:166), or -1.                                      */
typedef struct bcio_selection {
    int64_t n_accepted;           /* accepted reads over ALL refs (requested or not)           */
    int64_t keyerror_ordinal;     /* -1 if none                                                */
    int64_t keyerror_rec;         /* record index of that read, -1 if none                      */
    const int64_t* ref_beg;       /* [n_refs+1]                                                 */
    const int32_t* pos;
    const uint32_t* cig_beg;
    const uint32_t* cig_n;
    const uint32_t* seq_nib;
    const uint32_t* qlen;
    const int64_t* ordinal;
    const int64_t* rec;
    const int64_t* span;          /* ref_span[rec[i]]                                           */
} bcio_selection;

int bcio_select(bcio_file* f, int64_t min_mapq, const uint8_t* ref_sel, bcio_selection* out);

/* ---- streaming decode: bounded memory (the reference's --chunk-size, main.py:142-162) ----------
 * bcio_stream_open reads the header; bcio_stream_next decodes the next at most max_records records
 * (file order) into a new bcio_file handle — bcio_get_records / bcio_select work on it as on a
 * whole file, its record indices and ordinals counting from the batch's first record — which the
 * caller releases with bcio_close.  *out = NULL at the end of the file.  Live memory is one
 * batch plus the inflated bytes it was cut from: the file is mapped read-only, each fill
 * inflates just the blocks the batch is estimated to need in one parallel pass, and the pages
 * of consumed compressed blocks are given back (MADV_DONTNEED).  bcio_stream_records: records
 * handed out so far (the next batch's first record index in the file).                       */
typedef struct bcio_stream bcio_stream;
int bcio_stream_open(const char* path, int nthreads, bcio_stream** out);
int bcio_stream_next(bcio_stream* s, int64_t max_records, bcio_file** out);
int64_t bcio_stream_records(const bcio_stream* s);
int32_t bcio_stream_n_refs(const bcio_stream* s);
const char* bcio_stream_ref_name(const bcio_stream* s, int32_t i);
int64_t bcio_stream_ref_len(const bcio_stream* s, int32_t i);
void bcio_stream_close(bcio_stream* s);

/* ---- one file decoded by several ranks (each only its own references' records) ----------------
 * Positions are BAM virtual offsets: (BGZF block file offset << 16) | offset in its inflated bytes.
 * bcio_find_ref_start: the position of the first record whose refID is >= tid or -1 (unmapped),
 * 0 if there is none (the file ends first).  The file is not inflated: a bisection over the BGZF
 * blocks (each probe finds a block header and then a record start by validating a chain of
 * records) narrows the search to a few blocks, which are then hopped record by record.  The
 * answer is exact when the file is grouped by reference (coordinate-sorted) and the probes
 * synchronised correctly; neither is assumed: a caller verifies them with the range streams.
 * bcio_stream_open_range: a stream over the records of [voff_begin, voff_end) (voff_end 0: to the
 * end of the file; voff_end <= voff_begin otherwise: no records) with the header's references.
 * voff_begin must be a record start.  If the record chain does not end exactly at voff_end,
 * bcio_stream_next fails with BCIO_E_FORMAT ("truncated BAM record"): the split was wrong. */
int bcio_find_ref_start(const char* path, int32_t tid, uint64_t* voff);
/* The same for the first record at or past (tid, pos) in coordinate order (refID tid and
 * position >= pos, or a later refID, or -1): a split point inside one reference's reads. */
int bcio_find_record(const char* path, int32_t tid, int32_t pos, uint64_t* voff);
int bcio_stream_open_range(const char* path, int nthreads, uint64_t voff_begin, uint64_t voff_end,
                           bcio_stream** out);

/* BAM-packed SEQ bytes -> BC_SEQ_EVENT (basecount_hip.h), on the host with `nthreads` threads
 * (<= 0: hardware).  out_bytes >= nbytes rounded up to 16 plus 16; the tail is zero-filled.
 * The decoder already provides this layout for a file's records (bcio_records.seq_event).   */
int bcio_seq_to_event(const uint8_t* bam, int64_t nbytes, uint8_t* out, int64_t out_bytes, int nthreads);

/* ---- writer: BAM records -> BGZF file (used by the synthetic generator) ----------------- */
typedef struct bcio_write_spec {
    int32_t n_refs;
    const char* const* ref_names;
    const int64_t* ref_lens;
    int64_t n;                     /* records */
    const int32_t* tid;
    const int32_t* pos;
    const uint16_t* flag;
    const uint8_t* mapq;
    const uint64_t* cig_off;       /* [n+1] */
    const uint32_t* cigar;
    const int32_t* l_seq;          /* [n] */
    const uint64_t* seq_off;       /* [n+1] byte CSR of packed SEQ */
    const uint8_t* seq;
    const uint64_t* qual_off;      /* [n+1] byte CSR of QUAL (l_seq bytes each; 0xFF.. = absent) */
    const uint8_t* qual;
    int level;                     /* deflate level 0..9 */
    int nthreads;
} bcio_write_spec;

int bcio_write_bam(const char* path, const bcio_write_spec* spec);

/* ---- formatter ------------------------------------------------------------------------------
 * Reproduces `str(round(x, dp))` for Python ints and floats (main.py:461), 0 <= dp <= 323.
 * Wide rows (main.py:69-78) and long rows (main.py:57-68) of one reference.
 *   counts : int32 [k][L] planes (k = 5 or 6, column order A,C,G,T,DS[,N])
 *   pc     : f64   [k][L] planes (ignored where coverage == 0: printed as int -1)
 *   ent    : f64   [L]    (int 1 where coverage == 0)
 *   sec    : f64   [L]    (int 1 where coverage == 0 or only one nonzero count)
 * The text is appended to an internal buffer; fetch it with bcio_fmt_take().              */
typedef struct bcio_fmt bcio_fmt;
int bcio_fmt_new(bcio_fmt** out);
void bcio_fmt_free(bcio_fmt* b);
int bcio_fmt_rows(bcio_fmt* b, const char* ref, int64_t L, int k, const int32_t* counts,
                  const double* pc, const double* ent, const double* sec, int dp, int long_format,
                  int nthreads);
/* returns pointer+size of the accumulated text and resets the buffer on the next append */
int bcio_fmt_take(bcio_fmt* b, const char** data, int64_t* size);
/* scalar helpers (used by tests to compare against CPython on random values) */
int bcio_fmt_pyround_float(double x, int dp, char* out, int cap);
int bcio_fmt_pyround_int(int64_t v, int dp, char* out, int cap);

#ifdef __cplusplus
}
#endif
#endif
