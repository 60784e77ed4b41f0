// bc_capi.hip — extern "C" boundary (include/basecount_hip.h).  Host-side glue only: argument
// checks, stream/memory management, launch geometry; every count/stat is computed by the
// kernels in bc_kernels.hip.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "bc_internal.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& m) {
    g_err = m;
    return code;
}

int hip_fail(hipError_t e, const char* where) {
    return fail(BC_E_HIP, std::string(where) + ": " + hipGetErrorString(e));
}

#define HIP_TRY(expr)                                   \
    do {                                                \
        hipError_t _e = (expr);                         \
        if (_e != hipSuccess) return hip_fail(_e, #expr); \
    } while (0)

// hipEvents around one launch when the context's timing is on
struct Timed {
    bc_ctx* c;
    int id;
    hipEvent_t a = nullptr, b = nullptr;
    Timed(bc_ctx* ctx, int kid) : c(ctx), id(kid) {
        if (c->timing && hipEventCreate(&a) == hipSuccess && hipEventCreate(&b) == hipSuccess)
            (void)hipEventRecord(a, c->stream);
    }
    ~Timed() {
        if (a && b) {
            (void)hipEventRecord(b, c->stream);
            c->ev[id].emplace_back(a, b);
        }
    }
};

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

// Reads per kernel-1 workgroup: enough workgroups to fill 256 CUs several times over, and few
// enough reads per chunk that a sorted chunk's positions fit one LDS window.
int choose_rpb(int64_t n, int64_t L, int max_span, int sorted, int forced) {
    if (forced > 0) return std::min(forced, 32768);
    int64_t target = std::min<int64_t>(8192, std::max<int64_t>(32, n / 2048));
    if (!sorted || max_span <= 0 || max_span >= bc::kWinMax || L <= 0) return (int)target;
    const double density = (double)n / (double)L;
    const double fit = (bc::kWinMax - max_span) * density * 0.75;
    if (fit >= 32.0) return (int)std::min<double>((double)target, fit);
    return (int)target;  // sparse: chunks take the global-atomic path
}

bool host_sorted(const int32_t* pos, int64_t n) {
    for (int64_t i = 1; i < n; ++i)
        if (pos[i] < pos[i - 1]) return false;
    return true;
}

// max reference span and max read end (pos + span) of a host batch
std::pair<int, int64_t> host_spans(const bc_reads& r) {
    uint64_t best = 0;
    int64_t end = 0;
    for (int64_t i = 0; i < r.n_reads; ++i) {
        const uint32_t* cg = r.cigar + r.cig_beg[i];
        uint64_t span = 0;
        for (uint32_t k = 0; k < r.cig_n[i]; ++k) {
            uint32_t op = cg[k] & 15u;
            if (op == 0 || op == 2 || op == 3 || op == 7 || op == 8) span += cg[k] >> 4;
        }
        best = std::max(best, span);
        end = std::max<int64_t>(end, (int64_t)r.pos[i] + (int64_t)span);
    }
    return {(int)std::min<uint64_t>(best, 0x7fffffff), end};
}

// BC_INDEX_AUTO resolved for this context: the run records when the read-chunked kernel would
// take the batch, else the tile index when the tiled one would (the sparse sweep uses neither)
int index_what(const bc_ctx* c, const bc_reads& r, int64_t L, int what = BC_INDEX_AUTO) {
    if (!(what & BC_INDEX_AUTO)) return what & (BC_INDEX_RUNS | BC_INDEX_TILES);
    if (!r.sorted || r.n_reads <= 0 || r.seq_layout != BC_SEQ_EVENT) return 0;
    if (bc::use_rc(r, L, c->shape)) return BC_INDEX_RUNS;
    return bc::pileup_is_solo(r, L, c->shape, c->tile_waves) ? 0 : BC_INDEX_TILES;
}

int check_host_reads(const bc_reads* r) {
    if (!r) return fail(BC_E_ARG, "reads is NULL");
    if (r->n_reads < 0) return fail(BC_E_ARG, "n_reads < 0");
    if (r->n_reads == 0) return BC_OK;
    if (!r->pos || !r->cig_beg || !r->cig_n || !r->seq_nib) return fail(BC_E_ARG, "missing per-read array");
    for (int64_t i = 0; i < r->n_reads; ++i) {
        if ((uint64_t)r->cig_beg[i] + r->cig_n[i] > (uint64_t)r->n_cigar_words)
            return fail(BC_E_ARG, "read " + std::to_string(i) + ": CIGAR outside the cigar buffer");
        if (r->pos[i] < 0) return fail(BC_E_ARG, "read " + std::to_string(i) + ": negative start");
        // query consumption must stay inside the packed sequence (and quality) buffers
        uint64_t q = 0;
        const uint32_t* cg = r->cigar + r->cig_beg[i];
        for (uint32_t k = 0; k < r->cig_n[i]; ++k) {
            uint32_t op = cg[k] & 15u;
            if (op == 0 || op == 1 || op == 7 || op == 8) q += cg[k] >> 4;
        }
        if (q && (uint64_t)r->seq_nib[i] + q > 2ull * (uint64_t)r->seq_bytes)
            return fail(BC_E_ARG, "read " + std::to_string(i) + ": CIGAR consumes past the sequence");
        if (q && r->qual && (uint64_t)r->seq_nib[i] + q > (uint64_t)r->qual_bytes)
            return fail(BC_E_ARG, "read " + std::to_string(i) + ": CIGAR consumes past the qualities");
    }
    return BC_OK;
}

// refPos the reference's .at() rejects first for read i (host walk in count.cpp:40-96 order)
int64_t host_bad_pos(const bc_reads& r, int64_t i, int64_t ref_len, uint32_t mbq) {
    static const int col_of[16] = {-1, 0, 1, -1, 2, -1, -1, -1, 3, -1, -1, -1, -1, -1, -1, 5};
    int64_t rp = r.pos[i];
    uint64_t qp = r.seq_nib[i];
    const uint32_t* cg = r.cigar + r.cig_beg[i];
    for (uint32_t k = 0; k < r.cig_n[i]; ++k) {
        uint32_t op = cg[k] & 15u, len = cg[k] >> 4;
        if (op == 0 || op == 7 || op == 8) {
            for (uint32_t j = 0; j < len; ++j, ++rp, ++qp) {
                if (r.qual && r.qual[qp] < mbq) continue;
                if (!r.qual && mbq > 0) continue;
                unsigned b = r.seq[qp >> 1];
                unsigned nib = (qp & 1) ? (b & 15u) : (b >> 4);
                if (col_of[nib] >= 0 && rp >= ref_len) return rp;
            }
        } else if (op == 1) {
            qp += len;
        } else if (op == 2 || op == 3) {
            for (uint32_t j = 0; j < len; ++j, ++rp)
                if (rp >= ref_len) return rp;
        }
    }
    return -1;
}

}  // namespace

namespace bc {
int set_error(int code, const std::string& m) { return fail(code, m); }
}  // namespace bc

extern "C" {

const char* bc_last_error(void) { return g_err.c_str(); }
int bc_abi_version(void) { return BC_ABI_VERSION; }

const char* bc_build_info(void) {
    return "gfx950"
#ifdef BC_DIAG
           " diag=1"
#else
           " diag=0"
#endif
#ifdef BC_PHASE_TRACE
           " phase_trace=1"
#else
           " phase_trace=0"
#endif
        ;
}

int bc_device_count(int* n) {
    if (!n) return fail(BC_E_ARG, "n is NULL");
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    *n = (e == hipSuccess) ? c : 0;
    return BC_OK;
}

int bc_ctx_create(int device, void* stream, bc_ctx** out) {
    if (!out) return fail(BC_E_ARG, "out is NULL");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail(BC_E_NODEV, "no HIP device visible");
    if (device < 0 || device >= n) return fail(BC_E_ARG, "device index out of range");
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(BC_E_NODEV, std::string("built for gfx950, device is ") + prop.gcnArchName);
    DeviceGuard g(device);
    auto* c = new bc_ctx();
    c->device = device;
    if (stream) {
        c->stream = (hipStream_t)stream;
    } else {
        hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
        if (e != hipSuccess) {
            delete c;
            return hip_fail(e, "hipStreamCreate");
        }
        c->own_stream = true;
    }
    hipError_t e = hipMalloc(&c->d_err, sizeof(unsigned long long));
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->sig, hipEventDisableTiming);
    if (e == hipSuccess) e = hipHostMalloc(&c->h_err, sizeof(unsigned long long), hipHostMallocDefault);
    if (e == hipSuccess) e = hipMemsetAsync(c->d_err, 0xFF, sizeof(unsigned long long), c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) {
        bc_ctx_destroy(c);
        return hip_fail(e, "context scratch");
    }
    *out = c;
    return BC_OK;
}

int bc_ctx_destroy(bc_ctx* c) {
    if (!c) return BC_OK;
    DeviceGuard g(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->d_err) (void)hipFree(c->d_err);
    if (c->rc_scratch) (void)hipFree(c->rc_scratch);
    if (c->out_scratch) (void)hipFree(c->out_scratch);
    if (c->sum_scratch) (void)hipFree(c->sum_scratch);
    if (c->h_err) (void)hipHostFree(c->h_err);
    for (auto& v : c->ev)
        for (auto& pr : v) {
            (void)hipEventDestroy(pr.first);
            (void)hipEventDestroy(pr.second);
        }
    for (auto& e : c->mark)
        if (e) (void)hipEventDestroy(e);
    if (c->sig) (void)hipEventDestroy(c->sig);
    if (c->own_stream && c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return BC_OK;
}

int bc_ctx_release_scratch(bc_ctx* c) {
    if (!c) return fail(BC_E_ARG, "ctx is NULL");
    DeviceGuard g(c->device);
    if (c->rc_scratch || c->out_scratch || c->sum_scratch) HIP_TRY(hipStreamSynchronize(c->stream));
    // one buffer at a time: its pointer and size are cleared whether or not its free succeeded,
    // so no later call frees it twice; the first error is returned after all three
    hipError_t first = hipSuccess;
    const char* where = nullptr;
    auto drop = [&](void*& p, size_t& bytes, const char* what) {
        if (p) {
            const hipError_t e = hipFree(p);
            if (e != hipSuccess && first == hipSuccess) first = e, where = what;
        }
        p = nullptr;
        bytes = 0;
    };
    void* rc = c->rc_scratch;
    drop(rc, c->rc_scratch_bytes, "hipFree(rc_scratch)");
    c->rc_scratch = nullptr;
    drop(c->out_scratch, c->out_scratch_bytes, "hipFree(out_scratch)");
    drop(c->sum_scratch, c->sum_scratch_bytes, "hipFree(sum_scratch)");
    if (first != hipSuccess) return hip_fail(first, where);
    return BC_OK;
}

int bc_ctx_stream(bc_ctx* c, void** s) {
    if (!c || !s) return fail(BC_E_ARG, "NULL argument");
    *s = (void*)c->stream;
    return BC_OK;
}

int bc_ctx_set_shape(bc_ctx* c, int shape, int tile_waves, int rpb) {
    if (!c) return fail(BC_E_ARG, "ctx is NULL");
    if (shape < BC_SHAPE_AUTO || shape > BC_SHAPE_TILE_NO_SOLO) return fail(BC_E_ARG, "unknown BC_SHAPE_* value");
    if (tile_waves != 0 && tile_waves != 1 && tile_waves != 2 && tile_waves != 4 && tile_waves != 8)
        return fail(BC_E_ARG, "tile_waves must be 0, 1, 2, 4 or 8");
    if (rpb < 0 || rpb > 32768) return fail(BC_E_ARG, "reads_per_block must be 0..32768");
    c->shape = shape;
    c->tile_waves = tile_waves;
    c->reads_per_block = rpb;
    return BC_OK;
}

int bc_sync(bc_ctx* c) {
    if (!c) return fail(BC_E_ARG, "ctx is NULL");
    DeviceGuard g(c->device);
    HIP_TRY(hipStreamSynchronize(c->stream));
    return BC_OK;
}

int bc_malloc(bc_ctx* c, size_t bytes, void** p) {
    if (!c || !p) return fail(BC_E_ARG, "NULL argument");
    DeviceGuard g(c->device);
    *p = nullptr;
    if (bytes == 0) bytes = 16;
    HIP_TRY(hipMalloc(p, bytes));
    return BC_OK;
}

int bc_free(bc_ctx* c, void* p) {
    if (!c) return fail(BC_E_ARG, "ctx is NULL");
    if (!p) return BC_OK;
    DeviceGuard g(c->device);
    HIP_TRY(hipStreamSynchronize(c->stream));
    HIP_TRY(hipFree(p));
    return BC_OK;
}

int bc_memcpy_h2d(bc_ctx* c, void* d, const void* h, size_t bytes) {
    if (!c) return fail(BC_E_ARG, "ctx is NULL");
    if (!bytes) return BC_OK;
    DeviceGuard g(c->device);
    HIP_TRY(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, c->stream));
    return BC_OK;
}

int bc_memcpy_d2h(bc_ctx* c, void* h, const void* d, size_t bytes) {
    if (!c) return fail(BC_E_ARG, "ctx is NULL");
    if (!bytes) return BC_OK;
    DeviceGuard g(c->device);
    HIP_TRY(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, c->stream));
    return BC_OK;
}

int bc_memset(bc_ctx* c, void* d, int v, size_t bytes) {
    if (!c) return fail(BC_E_ARG, "ctx is NULL");
    if (!bytes) return BC_OK;
    DeviceGuard g(c->device);
    HIP_TRY(hipMemsetAsync(d, v, bytes, c->stream));
    return BC_OK;
}

int bc_reads_upload(bc_ctx* c, const bc_reads* h, bc_reads* d) {
    if (!c || !d) return fail(BC_E_ARG, "NULL argument");
    int rc = check_host_reads(h);
    if (rc) return rc;
    DeviceGuard g(c->device);
    std::memset(d, 0, sizeof *d);
    d->n_reads = h->n_reads;
    d->n_cigar_words = h->n_cigar_words;
    d->seq_bytes = h->seq_bytes;
    d->qual_bytes = h->qual ? h->qual_bytes : 0;
    // the tiled kernel relies on both properties: always derive them from the data itself
    d->sorted = h->n_reads ? (host_sorted(h->pos, h->n_reads) ? 1 : 0) : 1;
    const auto sp = h->n_reads ? host_spans(*h) : std::pair<int, int64_t>(0, 0);
    d->max_span = sp.first;
    d->max_end = sp.second;
    if (h->seq_layout != BC_SEQ_BAM && h->seq_layout != BC_SEQ_EVENT)
        return fail(BC_E_ARG, "bc_reads_upload: unknown seq_layout");
    // BC_SEQ_EVENT from the host (the decoder's bcio_records.seq_event): a plain copy, no device
    // conversion pass; BC_SEQ_BAM is converted in place by k_seq_event after the copy
    const bool host_event = h->seq_layout == BC_SEQ_EVENT;
    const size_t n = (size_t)h->n_reads;
    // the batch's device index (bc_index.hip), built on the device after the copies: run
    // records + chunk summaries when the read-chunked kernel would take the batch, else the tile
    // index when the tiled one would (nothing for the sparse sweep)
    d->seq_layout = BC_SEQ_EVENT;  // (the device copy's layout, whatever the host's)
    const int what = index_what(c, *d, d->max_end);
    const bc::IndexPlan plan = bc::index_plan(*d, what);
    constexpr int kArr = 8;
    void* p[kArr] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
    // the sequence buffer is sized for BC_SEQ_EVENT (converted in place after the copy)
    const size_t sz[kArr] = {n * 4, n * 4, n * 4, n * 4, (size_t)h->n_cigar_words * 4,
                             bc::seq_event_bytes(h->seq_bytes), h->qual ? (size_t)h->qual_bytes : 0, plan.total};
    const size_t cp[kArr] = {sz[0], sz[1], sz[2], sz[3], sz[4], (size_t)h->seq_bytes, sz[6], 0};
    const void* src[kArr] = {h->pos, h->cig_beg, h->cig_n, h->seq_nib, h->cigar, h->seq, h->qual, nullptr};
    // ONE slab for the whole batch (arrays 4 KiB-aligned inside it, the slab a multiple of 2 MiB):
    // the kernels' first touches of a batch then miss the GPU TLB on a few large fragments
    // instead of on every small buffer's pages.  The first array present is the slab base
    // (bc_reads_free).
    size_t off[kArr], total = 0;
    for (int i = 0; i < kArr; ++i) {
        off[i] = total;
        total += (sz[i] + 4095) / 4096 * 4096;
    }
    total = (total + (2u << 20) - 1) / (2u << 20) * (2u << 20);
    void* slab = nullptr;
    HIP_TRY(hipMalloc(&slab, total));
    for (int i = 0; i < kArr; ++i) {
        if (!sz[i]) continue;
        p[i] = (uint8_t*)slab + off[i];
        hipError_t e = cp[i] ? hipMemcpyAsync(p[i], src[i], cp[i], hipMemcpyHostToDevice, c->stream) : hipSuccess;
        if (e == hipSuccess && i == 5) {
            if (host_event)  // zero padding past the copied bytes
                e = hipMemsetAsync((uint8_t*)p[5] + cp[5], 0, sz[5] - cp[5], c->stream);
            else
                e = bc::launch_seq_event(c->stream, (const uint8_t*)p[5], h->seq_bytes, (uint8_t*)p[5]);
        }
        if (e != hipSuccess) {
            (void)hipStreamSynchronize(c->stream);
            (void)hipFree(slab);
            return hip_fail(e, "bc_reads_upload");
        }
    }
    d->pos = (const int32_t*)p[0];
    d->cig_beg = (const uint32_t*)p[1];
    d->cig_n = (const uint32_t*)p[2];
    d->seq_nib = (const uint32_t*)p[3];
    d->cigar = (const uint32_t*)p[4];
    d->seq = (const uint8_t*)p[5];
    d->qual = (const uint8_t*)p[6];
    d->seq_layout = BC_SEQ_EVENT;
    if (plan.total) {
        Timed tm(c, BC_K_INDEX);
        hipError_t e = bc::launch_index(c->stream, *d, plan, p[7]);
        if (e != hipSuccess) {
            (void)hipStreamSynchronize(c->stream);
            (void)hipFree(slab);
            std::memset(d, 0, sizeof *d);
            return hip_fail(e, "bc_reads_upload: index");
        }
    }
    HIP_TRY(hipStreamSynchronize(c->stream));
    return BC_OK;
}

int bc_reads_index_bytes(bc_ctx* c, const bc_reads* r, int64_t L, int what, size_t* bytes) {
    if (!c || !r || !bytes) return fail(BC_E_ARG, "NULL argument");
    if (what & ~(BC_INDEX_RUNS | BC_INDEX_TILES | BC_INDEX_AUTO)) return fail(BC_E_ARG, "unknown BC_INDEX_* bits");
    *bytes = bc::index_plan(*r, index_what(c, *r, L, what)).total;
    return BC_OK;
}

int bc_reads_index(bc_ctx* c, bc_reads* r, int64_t L, int what, void* d_mem, size_t bytes) {
    if (!c || !r) return fail(BC_E_ARG, "NULL argument");
    if (what & ~(BC_INDEX_RUNS | BC_INDEX_TILES | BC_INDEX_AUTO)) return fail(BC_E_ARG, "unknown BC_INDEX_* bits");
    r->read_runs = nullptr;
    r->run_chunks = 0;
    r->tile_reads = nullptr;
    r->n_tiles = 0;
    r->index_tag = 0;
    const bc::IndexPlan plan = bc::index_plan(*r, index_what(c, *r, L, what));
    if (!plan.total) return BC_OK;
    if (!d_mem || bytes < plan.total) return fail(BC_E_ARG, "bc_reads_index: d_mem smaller than bc_reads_index_bytes");
    if ((uintptr_t)d_mem & 15u) return fail(BC_E_ARG, "bc_reads_index: d_mem must be 16-byte aligned");
    if (!r->pos || !r->cig_beg || !r->cig_n || !r->seq_nib || (r->n_cigar_words > 0 && !r->cigar))
        return fail(BC_E_ARG, "bc_reads_index: missing per-read array");
    DeviceGuard g(c->device);
    Timed tm(c, BC_K_INDEX);
    HIP_TRY(bc::launch_index(c->stream, *r, plan, d_mem));
    return BC_OK;
}

// The sort leaves the sequence in place (sorts the fields + run records only) when the sorted
// batch will take the read-chunked k_rc, which gathers a chunk's scattered reads into LDS itself;
// batches with qualities (a quality threshold: k_rc's variants that stage through registers) and
// the tiled kernels' shallower batches get the sequence copied into start order.
static bool sort_fields_only(const bc_ctx* c, const bc_reads& r) {
    if (r.qual) return false;
    bc_reads v = r;
    v.sorted = 1;
    return bc::use_rc(v, r.max_end, c->shape);
}

int bc_reads_sort_bytes(bc_ctx* c, const bc_reads* r, size_t* bytes) {
    if (!c || !r || !bytes) return fail(BC_E_ARG, "NULL argument");
    *bytes = bc::sort_bytes(*r, sort_fields_only(c, *r));
    return BC_OK;
}

int bc_reads_sort(bc_ctx* c, const bc_reads* r, bc_reads* out, void* d_mem, size_t bytes) {
    if (!c || !r || !out) return fail(BC_E_ARG, "NULL argument");
    if (r->n_reads < 0 || r->max_end < 0) return fail(BC_E_ARG, "bc_reads_sort: negative n_reads / max_end");
    if (r->n_reads >= (int64_t)0xFFFFFFFF) return fail(BC_E_ARG, "bc_reads_sort: more than 2^32 - 1 reads");
    if (r->n_reads == 0) {
        *out = *r;
        out->sorted = 1;
        return BC_OK;
    }
    if (r->seq_layout != BC_SEQ_EVENT) return fail(BC_E_ARG, "bc_reads_sort needs seq_layout == BC_SEQ_EVENT");
    if (!r->pos || !r->cig_beg || !r->cig_n || !r->seq_nib || !r->seq) return fail(BC_E_ARG, "bc_reads_sort: missing array");
    const bool fields = sort_fields_only(c, *r);
    const size_t need = bc::sort_bytes(*r, fields);
    if (!d_mem || bytes < need) return fail(BC_E_ARG, "bc_reads_sort: d_mem smaller than bc_reads_sort_bytes");
    if ((uintptr_t)d_mem & 255u) return fail(BC_E_ARG, "bc_reads_sort: d_mem must be 256-byte aligned");
    if (!bc::sort_fits(*r))
        return fail(BC_E_ARG, "bc_reads_sort: batch too large to sort (seq_bytes + 5 n_reads + 16 > 0x55555550): "
                              "split it");
    DeviceGuard g(c->device);
    bc_reads tmp;
    {
        Timed tm(c, BC_K_SORT);
        HIP_TRY(bc::launch_sort(c->stream, *r, tmp, d_mem, fields));
    }
    *out = tmp;
    return BC_OK;
}

int bc_reads_sort_check(bc_ctx* c, const bc_reads* r, const void* d_mem) {
    if (!c || !r) return fail(BC_E_ARG, "NULL argument");
    if (r->n_reads <= 0) return BC_OK;
    if (!d_mem) return fail(BC_E_ARG, "bc_reads_sort_check: d_mem is NULL");
    DeviceGuard g(c->device);
    HIP_TRY(hipMemcpyAsync(c->h_err, bc::sort_flags_word(*r, d_mem), 4, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    const uint32_t flags = (uint32_t)(*c->h_err & 0xFFFFFFFFu);
    if (flags & 2u) return fail(BC_E_ARG, "bc_reads_sort: a read starts outside [0, max_end] (max_end not truthful)");
    if (flags & 1u) return fail(BC_E_ARG, "bc_reads_sort: the reads' sequences overlap (sorted copy would not fit)");
    return BC_OK;
}

int bc_reads_free(bc_ctx* c, bc_reads* d) {
    if (!c || !d) return fail(BC_E_ARG, "NULL argument");
    DeviceGuard g(c->device);
    (void)hipStreamSynchronize(c->stream);
    const void* p[9] = {d->pos, d->cig_beg, d->cig_n, d->seq_nib, d->cigar, d->seq, d->qual, d->read_runs, d->tile_reads};
    for (auto q : p)  // the first array present is the base of the batch's slab (bc_reads_upload)
        if (q) {
            (void)hipFree((void*)q);
            break;
        }
    std::memset(d, 0, sizeof *d);
    return BC_OK;
}

int bc_count(bc_ctx* c, const bc_reads* r, int64_t ref_len, uint32_t mbq, int ncols, int32_t* d_hist) {
    if (!c || !r) return fail(BC_E_ARG, "NULL argument");
    if (ncols != 5 && ncols != 6) return fail(BC_E_ARG, "ncols must be 5 or 6");
    if (ref_len < 0) return fail(BC_E_ARG, "ref_len < 0");
    if (r->n_reads == 0) return BC_OK;
    if (!d_hist && ref_len > 0) return fail(BC_E_ARG, "d_hist is NULL");
    if (mbq > 0 && !r->qual) return fail(BC_E_ARG, "min_base_quality > 0 needs qualities");
    DeviceGuard g(c->device);
    const bool event = r->seq_layout == BC_SEQ_EVENT && !((uintptr_t)r->seq & 15u);
    if (r->sorted && event && bc::use_rc(*r, ref_len, c->shape)) {
        Timed tm(c, BC_K_RC);
        HIP_TRY(bc::launch_rc(c->stream, *r, ref_len, mbq, ncols, d_hist, c->d_err));
        return BC_OK;
    }
    if (r->sorted && r->max_span <= bc::kTileMaxSpan && event) {
        // sorted batch: the tiled kernel in accumulate mode (plain read-add-write per owned tile)
        Timed tm(c, bc::pileup_is_solo(*r, ref_len, c->shape, c->tile_waves) ? BC_K_SOLO : BC_K_PILEUP);
        HIP_TRY(bc::launch_pileup_tiles(c->stream, *r, ref_len, r->max_end, mbq, ncols, false, true, 0.0, 0.0,
                                        d_hist, nullptr, nullptr, nullptr, nullptr, c->d_err, c->shape,
                                        c->tile_waves));
        return BC_OK;
    }
    const int rpb = choose_rpb(r->n_reads, ref_len, r->max_span, r->sorted, c->reads_per_block);
    Timed tm(c, BC_K_COUNT);
    HIP_TRY(bc::launch_count(c->stream, *r, ref_len, mbq, ncols, d_hist, rpb, c->d_err));
    return BC_OK;
}

int bc_pileup(bc_ctx* c, const bc_reads* r, int64_t L, uint32_t mbq, int k, double nf, double nf2, int32_t* d_counts,
              int32_t* d_cov, double* d_pc, double* d_ent, double* d_sec) {
    if (!c || !r) return fail(BC_E_ARG, "NULL argument");
    if (k != 5 && k != 6) return fail(BC_E_ARG, "k must be 5 or 6");
    if (L < 0) return fail(BC_E_ARG, "ref_len < 0");
    if (!r->sorted) return fail(BC_E_ARG, "bc_pileup needs a coordinate-sorted batch (sorted == 1)");
    if (mbq > 0 && r->n_reads > 0 && !r->qual) return fail(BC_E_ARG, "min_base_quality > 0 needs qualities");
    if (r->n_reads > 0 && r->seq_layout != BC_SEQ_EVENT)
        return fail(BC_E_ARG, "bc_pileup needs seq_layout == BC_SEQ_EVENT (see bc_seq_to_event)");
    if (r->n_reads > 0 && ((uintptr_t)r->seq & 15u))
        return fail(BC_E_ARG, "bc_pileup needs a 16-byte aligned sequence buffer");
    if (L > 0 && (!d_counts || !d_cov || !d_ent || !d_sec)) return fail(BC_E_ARG, "NULL output");
    DeviceGuard g(c->device);
    if (bc::use_rc(*r, L, c->shape)) {
        // deep batch: counts by the read-chunked kernel (atomics into the context's zeroed
        // scratch), then kernel 2, which also moves the counts to d_counts and re-zeroes the
        // scratch (no memset launch per call)
        const size_t need = (size_t)k * (size_t)L * 4;
        if (need > c->rc_scratch_bytes) {
            if (c->rc_scratch) {
                HIP_TRY(hipStreamSynchronize(c->stream));
                HIP_TRY(hipFree(c->rc_scratch));
                c->rc_scratch = nullptr;
                c->rc_scratch_bytes = 0;
            }
            HIP_TRY(hipMalloc((void**)&c->rc_scratch, need));
            c->rc_scratch_bytes = need;
            HIP_TRY(hipMemsetAsync(c->rc_scratch, 0, need, c->stream));
        }
        {
            Timed tm(c, BC_K_RC);
            HIP_TRY(bc::launch_rc(c->stream, *r, L, mbq, k, c->rc_scratch, c->d_err));
        }
        Timed tm(c, BC_K_STATS);
        HIP_TRY(bc::launch_stats(c->stream, c->rc_scratch, L, k, nf, nf2, d_cov, d_pc, d_ent, d_sec, d_counts));
        return BC_OK;
    }
    Timed tm(c, bc::pileup_is_solo(*r, L, c->shape, c->tile_waves) ? BC_K_SOLO : BC_K_PILEUP);
    HIP_TRY(bc::launch_pileup_tiles(c->stream, *r, L, r->max_end, mbq, k, true, false, nf, nf2, d_counts, d_cov,
                                    d_pc, d_ent, d_sec, c->d_err, c->shape, c->tile_waves));
    return BC_OK;
}

// grow-only context scratch (a synchronizing allocation when it grows: outside graph capture)
static int out_scratch(bc_ctx* c, size_t need) {
    if (need <= c->out_scratch_bytes) return BC_OK;
    if (c->out_scratch) {
        HIP_TRY(hipStreamSynchronize(c->stream));
        HIP_TRY(hipFree(c->out_scratch));
        c->out_scratch = nullptr;
        c->out_scratch_bytes = 0;
    }
    HIP_TRY(hipMalloc(&c->out_scratch, need));
    c->out_scratch_bytes = need;
    return BC_OK;
}

int bc_pileup_partials(bc_ctx* c, const bc_reads* r, int64_t L, uint32_t mbq, int k, double nf, double nf2,
                       int32_t* d_counts, int32_t* d_cov, double* d_pc, double* d_ent, double* d_sec, void* d_work) {
    if (!c || !r || !d_work) return fail(BC_E_ARG, "NULL argument");
    if (L <= 0) return fail(BC_E_ARG, "ref_len must be > 0 (np.mean of an empty list)");
    const bool sparse_path = !bc::use_rc(*r, L, c->shape) && r->n_reads > 0;
    if (!d_counts && !d_cov && !d_pc && !d_ent && !d_sec) {
        // Summary only (main.py:469-499 prints six numbers per reference): the sparse sweep writes
        // no per-position output but the last partial buffer's coverage / entropy (into context
        // scratch); the other paths write their outputs into context scratch.
        if (k != 5 && k != 6) return fail(BC_E_ARG, "k must be 5 or 6");
        DeviceGuard g(c->device);
        // (the sparse sweep k_pileup_solo is the kernel that fuses the partials)
        if (sparse_path && L >= bc::kNpBuf && bc::pileup_is_solo(*r, L, c->shape, c->tile_waves)) {
            if (!r->sorted) return fail(BC_E_ARG, "bc_pileup needs a coordinate-sorted batch (sorted == 1)");
            if (mbq > 0 && !r->qual) return fail(BC_E_ARG, "min_base_quality > 0 needs qualities");
            if (r->seq_layout != BC_SEQ_EVENT) return fail(BC_E_ARG, "bc_pileup needs seq_layout == BC_SEQ_EVENT");
            if ((uintptr_t)r->seq & 15u) return fail(BC_E_ARG, "bc_pileup needs a 16-byte aligned sequence buffer");
            if (int rc = out_scratch(c, (size_t)bc::kNpBuf * 12)) return rc;
            bc::SumParts parts = bc::summary_parts(d_work, L);
            parts.no_store = true;
            parts.ent_tail = (double*)c->out_scratch;
            parts.cov_tail = (int32_t*)((double*)c->out_scratch + bc::kNpBuf);
#ifdef BC_SUM_SWEEP  // A/B builds only: the per-tile sweep k_pileup_solo<STORE = false>
            {
                Timed tm(c, BC_K_SOLO);
                HIP_TRY(bc::launch_pileup_tiles(c->stream, *r, L, r->max_end, mbq, k, true, false, nf, nf2, nullptr,
                                                nullptr, nullptr, nullptr, nullptr, c->d_err, c->shape, c->tile_waves,
                                                &parts));
            }
#else
            {
                const size_t need = bc::sum_sparse_bytes(L);
                if (need > c->sum_scratch_bytes) {  // grow-only, zeroed once (the kernels leave it zeroed)
                    if (c->sum_scratch) {
                        HIP_TRY(hipStreamSynchronize(c->stream));
                        HIP_TRY(hipFree(c->sum_scratch));
                        c->sum_scratch = nullptr;
                        c->sum_scratch_bytes = 0;
                    }
                    HIP_TRY(hipMalloc(&c->sum_scratch, need));
                    c->sum_scratch_bytes = need;
                    HIP_TRY(hipMemsetAsync(c->sum_scratch, 0, need, c->stream));
                }
                Timed tm(c, BC_K_SOLO);
                const hipError_t e = bc::launch_sum_sparse(c->stream, *r, L, mbq, k, nf, c->d_err, parts,
                                                           c->sum_scratch, c->sum_scratch_bytes);
                if (e != hipSuccess) {
                    // the leaf arrays may be left partly counted (k_sum_buffers re-zeroes them at the
                    // end of the chain): give them back, so the next call allocates and zeroes afresh
                    (void)hipStreamSynchronize(c->stream);
                    (void)hipFree(c->sum_scratch);
                    c->sum_scratch = nullptr;
                    c->sum_scratch_bytes = 0;
                    return hip_fail(e, "bc::launch_sum_sparse");
                }
            }
#endif
            if (!parts.fused) return fail(BC_E_ARG, "internal: summary-only sweep without fused partials");
            // the fold's last partial buffer reads positions [full_chunks * 8192, L): the tail
            // arrays stand at that offset (only those elements are addressed)
            const int64_t off = parts.full_chunks * bc::kNpBuf;
            const int32_t* cov_base = (const int32_t*)((uintptr_t)parts.cov_tail - (uintptr_t)off * 4u);
            const double* ent_base = (const double*)((uintptr_t)parts.ent_tail - (uintptr_t)off * 8u);
            Timed tm(c, BC_K_SUMMARY);
            // (the read-parallel summary writes whole-buffer partials, the sweep quarter ones)
            HIP_TRY(bc::launch_summary_partials(c->stream, cov_base, ent_base, L, d_work, parts.full_chunks,
                                                !parts.whole_buffers));
            return BC_OK;
        }
        // counts [k][L] int32, cov [L] int32, ent / sec [L] double
        const size_t need = (size_t)L * (4u * (size_t)k + 4u + 16u);
        if (int rc = out_scratch(c, need)) return rc;
        double* ent = (double*)c->out_scratch;
        double* sec = ent + L;
        int32_t* cov = (int32_t*)(sec + L);
        int32_t* counts = cov + L;
        return bc_pileup_partials(c, r, L, mbq, k, nf, nf2, counts, cov, nullptr, ent, sec, d_work);
    }
    if (!sparse_path) {
        int rc = bc_pileup(c, r, L, mbq, k, nf, nf2, d_counts, d_cov, d_pc, d_ent, d_sec);
        if (rc) return rc;
        if (!d_cov || !d_ent) return fail(BC_E_ARG, "NULL coverage / entropy");
        DeviceGuard g(c->device);
        Timed tm(c, BC_K_SUMMARY);
        HIP_TRY(bc::launch_summary_partials(c->stream, d_cov, d_ent, L, d_work, 0));
        return BC_OK;
    }
    // the argument checks of bc_pileup
    if (k != 5 && k != 6) return fail(BC_E_ARG, "k must be 5 or 6");
    if (!r->sorted) return fail(BC_E_ARG, "bc_pileup needs a coordinate-sorted batch (sorted == 1)");
    if (mbq > 0 && !r->qual) return fail(BC_E_ARG, "min_base_quality > 0 needs qualities");
    if (r->seq_layout != BC_SEQ_EVENT) return fail(BC_E_ARG, "bc_pileup needs seq_layout == BC_SEQ_EVENT");
    if ((uintptr_t)r->seq & 15u) return fail(BC_E_ARG, "bc_pileup needs a 16-byte aligned sequence buffer");
    if (!d_counts || !d_cov || !d_ent || !d_sec) return fail(BC_E_ARG, "NULL output");
    DeviceGuard g(c->device);
    bc::SumParts parts = bc::summary_parts(d_work, L);
    {
        Timed tm(c, bc::pileup_is_solo(*r, L, c->shape, c->tile_waves) ? BC_K_SOLO : BC_K_PILEUP);
        HIP_TRY(bc::launch_pileup_tiles(c->stream, *r, L, r->max_end, mbq, k, true, false, nf, nf2, d_counts, d_cov,
                                        d_pc, d_ent, d_sec, c->d_err, c->shape, c->tile_waves, &parts));
    }
    const int64_t first = parts.fused ? parts.full_chunks : 0;
    Timed tm(c, BC_K_SUMMARY);  // the last, partial buffer (or all of them), and the header
    HIP_TRY(bc::launch_summary_partials(c->stream, d_cov, d_ent, L, d_work, first));
    return BC_OK;
}

int bc_summary_fold(bc_ctx* c, int n, const int64_t* ref_lens, void* const* d_works, double* const* d_outs) {
    if (!c || n < 0 || (n > 0 && (!ref_lens || !d_works || !d_outs))) return fail(BC_E_ARG, "NULL argument");
    for (int i = 0; i < n; ++i) {
        if (ref_lens[i] <= 0) return fail(BC_E_ARG, "ref_len must be > 0 (np.mean of an empty list)");
        if (!d_works[i] || !d_outs[i]) return fail(BC_E_ARG, "NULL work / output");
    }
    if (n == 0) return BC_OK;
    DeviceGuard g(c->device);
    Timed tm(c, BC_K_SUMMARY);
    HIP_TRY(bc::launch_summary_fold(c->stream, n, ref_lens, d_works, d_outs));
    return BC_OK;
}

int bc_pileup_summary(bc_ctx* c, const bc_reads* r, int64_t L, uint32_t mbq, int k, double nf, double nf2,
                      int32_t* d_counts, int32_t* d_cov, double* d_pc, double* d_ent, double* d_sec, void* d_work,
                      double* d_out) {
    if (!d_out) return fail(BC_E_ARG, "NULL argument");
    if (c && r && d_work && L > 0 && !d_pc && bc::use_rc(*r, L, c->shape) && (k == 5 || k == 6)) {
        // a deep batch: kernel 2 leaves numpy's leaf partials and ONE launch folds them (the fused
        // tail of bc_pileup_summary_amplicons, no windows); summary only: context stand-ins
        if (!d_counts && !d_cov && !d_ent && !d_sec) {
            const size_t need = (size_t)L * (4u * (size_t)k + 4u + 16u);
            DeviceGuard g(c->device);
            if (int rc = out_scratch(c, need)) return rc;
            d_ent = (double*)c->out_scratch;
            d_sec = d_ent + L;
            d_cov = (int32_t*)(d_sec + L);
            d_counts = d_cov + L;
        }
        if (d_counts && d_cov && d_ent && d_sec)
            return bc_pileup_summary_amplicons(c, r, L, mbq, k, nf, nf2, d_counts, d_cov, d_ent, d_sec, d_work, d_out,
                                               nullptr, nullptr, 0, nullptr);
    }
    int rc = bc_pileup_partials(c, r, L, mbq, k, nf, nf2, d_counts, d_cov, d_pc, d_ent, d_sec, d_work);
    if (rc) return rc;
    return bc_summary_fold(c, 1, &L, &d_work, &d_out);
}

int bc_graph_begin(bc_ctx* c) {
    if (!c) return fail(BC_E_ARG, "ctx is NULL");
    if (!c->stream) return fail(BC_E_ARG, "cannot capture the legacy default stream");
    DeviceGuard g(c->device);
    HIP_TRY(hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
    return BC_OK;
}

int bc_graph_end(bc_ctx* c, bc_graph** out) {
    if (!c || !out) return fail(BC_E_ARG, "NULL argument");
    DeviceGuard g(c->device);
    auto* gr = new bc_graph();
    hipError_t e = hipStreamEndCapture(c->stream, &gr->graph);
    if (e == hipSuccess) e = hipGraphInstantiate(&gr->exec, gr->graph, nullptr, nullptr, 0);
    if (e != hipSuccess) {
        bc_graph_destroy(gr);
        return hip_fail(e, "graph capture");
    }
    *out = gr;
    return BC_OK;
}

int bc_graph_launch(bc_ctx* c, bc_graph* gr) {
    if (!c || !gr) return fail(BC_E_ARG, "NULL argument");
    DeviceGuard g(c->device);
    HIP_TRY(hipGraphLaunch(gr->exec, c->stream));
    return BC_OK;
}

int bc_graph_destroy(bc_graph* gr) {
    if (!gr) return BC_OK;
    if (gr->exec) (void)hipGraphExecDestroy(gr->exec);
    if (gr->graph) (void)hipGraphDestroy(gr->graph);
    delete gr;
    return BC_OK;
}

int bc_timing_enable(bc_ctx* c, int on) {
    if (!c) return fail(BC_E_ARG, "ctx is NULL");
    c->timing = on != 0;
    return BC_OK;
}

int bc_timing_report(bc_ctx* c, int64_t* launches, double* mean_us) {
    if (!c || !launches || !mean_us) return fail(BC_E_ARG, "NULL argument");
    DeviceGuard g(c->device);
    HIP_TRY(hipStreamSynchronize(c->stream));
    for (int id = 0; id < BC_KERNEL_IDS; ++id) {
        double tot = 0.0;
        for (auto& pr : c->ev[id]) {
            float ms = 0.f;
            if (hipEventElapsedTime(&ms, pr.first, pr.second) == hipSuccess) tot += ms;
            (void)hipEventDestroy(pr.first);
            (void)hipEventDestroy(pr.second);
        }
        launches[id] = (int64_t)c->ev[id].size();
        mean_us[id] = c->ev[id].empty() ? 0.0 : tot * 1e3 / (double)c->ev[id].size();
        c->ev[id].clear();
    }
    return BC_OK;
}

int bc_ctx_wait(bc_ctx* c, bc_ctx* other) {
    if (!c || !other) return fail(BC_E_ARG, "NULL argument");
    if (c->device != other->device) return fail(BC_E_ARG, "bc_ctx_wait: contexts on different devices");
    if (c == other || c->stream == other->stream) return BC_OK;
    DeviceGuard g(c->device);
    HIP_TRY(hipEventRecord(other->sig, other->stream));
    HIP_TRY(hipStreamWaitEvent(c->stream, other->sig, 0));
    return BC_OK;
}

int bc_event_record(bc_ctx* c, int slot) {
    if (!c || slot < 0 || slot >= BC_EVENT_SLOTS) return fail(BC_E_ARG, "bad context or event slot");
    DeviceGuard g(c->device);
    if (!c->mark[slot]) HIP_TRY(hipEventCreate(&c->mark[slot]));
    HIP_TRY(hipEventRecord(c->mark[slot], c->stream));
    return BC_OK;
}

int bc_event_elapsed_ms(bc_ctx* c, int s0, int s1, float* ms) {
    if (!c || !ms || s0 < 0 || s1 < 0 || s0 >= BC_EVENT_SLOTS || s1 >= BC_EVENT_SLOTS)
        return fail(BC_E_ARG, "bad context, slot or output");
    if (!c->mark[s0] || !c->mark[s1]) return fail(BC_E_ARG, "event slot never recorded");
    DeviceGuard g(c->device);
    HIP_TRY(hipEventSynchronize(c->mark[s1]));
    HIP_TRY(hipEventElapsedTime(ms, c->mark[s0], c->mark[s1]));
    return BC_OK;
}

int bc_range_error(bc_ctx* c, int64_t* first_bad) {
    if (!c || !first_bad) return fail(BC_E_ARG, "NULL argument");
    DeviceGuard g(c->device);
    HIP_TRY(hipMemcpyAsync(c->h_err, c->d_err, sizeof(unsigned long long), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipMemsetAsync(c->d_err, 0xFF, sizeof(unsigned long long), c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    *first_bad = (*c->h_err == ~0ull) ? -1 : (int64_t)*c->h_err;
    return BC_OK;
}

int bc_stats(bc_ctx* c, const int32_t* d_hist, int64_t L, int k, double nf, double nf2, int32_t* d_cov,
             double* d_pc, double* d_ent, double* d_sec) {
    if (!c) return fail(BC_E_ARG, "ctx is NULL");
    if (k != 5 && k != 6) return fail(BC_E_ARG, "k must be 5 or 6");
    if (L < 0) return fail(BC_E_ARG, "ref_len < 0");
    if (L == 0) return BC_OK;
    if (!d_hist) return fail(BC_E_ARG, "d_hist is NULL");
    DeviceGuard g(c->device);
    Timed tm(c, BC_K_STATS);
    HIP_TRY(bc::launch_stats(c->stream, d_hist, L, k, nf, nf2, d_cov, d_pc, d_ent, d_sec));
    return BC_OK;
}

size_t bc_summary_work_bytes(int64_t L) { return bc::summary_work_bytes(L); }

size_t bc_seq_event_bytes(int64_t seq_bytes) { return bc::seq_event_bytes(seq_bytes); }

int bc_seq_to_event(bc_ctx* c, const uint8_t* d_bam, int64_t seq_bytes, uint8_t* d_event) {
    if (!c || !d_event || (seq_bytes > 0 && !d_bam)) return fail(BC_E_ARG, "NULL argument");
    if (seq_bytes < 0) return fail(BC_E_ARG, "seq_bytes < 0");
    DeviceGuard g(c->device);
    HIP_TRY(bc::launch_seq_event(c->stream, d_bam, seq_bytes, d_event));
    return BC_OK;
}

int bc_summary(bc_ctx* c, const int32_t* d_cov, const double* d_ent, int64_t L, void* d_work, double* d_out) {
    if (!c || !d_out || !d_work) return fail(BC_E_ARG, "NULL argument");
    if (L <= 0) return fail(BC_E_ARG, "ref_len must be > 0 (np.mean of an empty list)");
    if (!d_cov || !d_ent) return fail(BC_E_ARG, "NULL coverage / entropy");
    DeviceGuard g(c->device);
    Timed tm(c, BC_K_SUMMARY);
    HIP_TRY(bc::launch_summary(c->stream, d_cov, d_ent, L, d_work, d_out));
    return BC_OK;
}

int bc_amplicons(bc_ctx* c, const int32_t* d_cov, const double* d_ent, const double* d_sec, int64_t L,
                 const int64_t* d_lo, const int64_t* d_hi, int32_t n_tiles, double* d_out) {
    if (!c) return fail(BC_E_ARG, "ctx is NULL");
    if (n_tiles < 0) return fail(BC_E_ARG, "n_tiles < 0");
    if (n_tiles == 0) return BC_OK;
    if (!d_cov || !d_ent || !d_sec || !d_lo || !d_hi || !d_out) return fail(BC_E_ARG, "NULL argument");
    DeviceGuard g(c->device);
    Timed tm(c, BC_K_AMPLICONS);
    HIP_TRY(bc::launch_amplicons(c->stream, d_cov, d_ent, d_sec, L, d_lo, d_hi, n_tiles, d_out));
    return BC_OK;
}

int bc_pileup_summary_amplicons(bc_ctx* c, const bc_reads* r, int64_t L, uint32_t mbq, int k, double nf, double nf2,
                                int32_t* d_counts, int32_t* d_cov, double* d_ent, double* d_sec, void* d_work,
                                double* d_out, const int64_t* d_lo, const int64_t* d_hi, int32_t n_tiles,
                                double* d_amp) {
    if (!c || !r || !d_work || !d_out) return fail(BC_E_ARG, "NULL argument");
    if (L <= 0) return fail(BC_E_ARG, "ref_len must be > 0 (np.mean of an empty list)");
    if (n_tiles < 0) return fail(BC_E_ARG, "n_tiles < 0");
    if (n_tiles > 0 && (!d_lo || !d_hi || !d_amp)) return fail(BC_E_ARG, "NULL window argument");
    if (!d_counts || !d_cov || !d_ent || !d_sec) return fail(BC_E_ARG, "NULL output");
    if (!bc::use_rc(*r, L, c->shape)) {  // shallow batches: the fused sweeps, then the windows
        int rc = bc_pileup_summary(c, r, L, mbq, k, nf, nf2, d_counts, d_cov, nullptr, d_ent, d_sec, d_work, d_out);
        if (rc) return rc;
        return bc_amplicons(c, d_cov, d_ent, d_sec, L, d_lo, d_hi, n_tiles, d_amp);
    }
    // the argument checks of bc_pileup
    if (k != 5 && k != 6) return fail(BC_E_ARG, "k must be 5 or 6");
    if (!r->sorted) return fail(BC_E_ARG, "bc_pileup needs a coordinate-sorted batch (sorted == 1)");
    if (mbq > 0 && r->n_reads > 0 && !r->qual) return fail(BC_E_ARG, "min_base_quality > 0 needs qualities");
    if (r->n_reads > 0 && r->seq_layout != BC_SEQ_EVENT)
        return fail(BC_E_ARG, "bc_pileup needs seq_layout == BC_SEQ_EVENT (see bc_seq_to_event)");
    if (r->n_reads > 0 && ((uintptr_t)r->seq & 15u))
        return fail(BC_E_ARG, "bc_pileup needs a 16-byte aligned sequence buffer");
    DeviceGuard g(c->device);
    const size_t need = (size_t)k * (size_t)L * 4;
    if (need > c->rc_scratch_bytes) {  // as bc_pileup: grow-only, kept zeroed by kernel 2
        if (c->rc_scratch) {
            HIP_TRY(hipStreamSynchronize(c->stream));
            HIP_TRY(hipFree(c->rc_scratch));
            c->rc_scratch = nullptr;
            c->rc_scratch_bytes = 0;
        }
        HIP_TRY(hipMalloc((void**)&c->rc_scratch, need));
        c->rc_scratch_bytes = need;
        HIP_TRY(hipMemsetAsync(c->rc_scratch, 0, need, c->stream));
    }
    {
        Timed tm(c, BC_K_RC);
        HIP_TRY(bc::launch_rc(c->stream, *r, L, mbq, k, c->rc_scratch, c->d_err));
    }
    {
        Timed tm(c, BC_K_STATS);
        HIP_TRY(bc::launch_stats_leaves(c->stream, c->rc_scratch, L, k, nf, nf2, d_cov, d_ent, d_sec, d_counts, d_work));
    }
    Timed tm(c, BC_K_AMPLICONS);
    HIP_TRY(bc::launch_tail(c->stream, d_cov, d_ent, d_sec, L, d_work, d_out, d_lo, d_hi, n_tiles, d_amp));
    return BC_OK;
}

int bc_bcount_host(int device, int64_t ref_len, uint32_t mbq, const bc_reads* h, uint32_t* h_out, int64_t* bad_read,
                   int64_t* bad_pos) {
    if (bad_read) *bad_read = -1;
    if (bad_pos) *bad_pos = -1;
    if (ref_len < 0 || ref_len > 0xFFFFFFFFll) return fail(BC_E_ARG, "refLen out of uint32 range");
    if (ref_len > 0 && !h_out) return fail(BC_E_ARG, "h_out is NULL");
    int rc = check_host_reads(h);
    if (rc) return rc;
    if (mbq > 0 && h->n_reads > 0 && !h->qual) return fail(BC_E_ARG, "min_base_quality > 0 needs qualities");
    if (h->seq_layout != BC_SEQ_BAM) return fail(BC_E_ARG, "bc_bcount_host takes BC_SEQ_BAM sequences");
    bc_ctx* c = nullptr;
    rc = bc_ctx_create(device, nullptr, &c);
    if (rc) return rc;
    struct Cleanup {
        bc_ctx* c;
        bc_reads d{};
        int32_t* hist = nullptr;
        ~Cleanup() {
            if (hist) bc_free(c, hist);
            bc_reads_free(c, &d);
            bc_ctx_destroy(c);
        }
    } cl{c};
    rc = bc_reads_upload(c, h, &cl.d);
    if (rc) return rc;
    const size_t hb = (size_t)std::max<int64_t>(ref_len, 1) * 6 * sizeof(int32_t);
    rc = bc_malloc(c, hb, (void**)&cl.hist);
    if (rc) return rc;
    rc = bc_memset(c, cl.hist, 0, hb);
    if (rc) return rc;
    rc = bc_count(c, &cl.d, ref_len, mbq, 6, cl.hist);
    if (rc) return rc;
    int64_t bad = -1;
    rc = bc_range_error(c, &bad);
    if (rc) return rc;
    if (bad >= 0) {
        if (bad_read) *bad_read = bad;
        const int64_t bp = host_bad_pos(*h, bad, ref_len, mbq);
        if (bad_pos) *bad_pos = bp;
        return fail(BC_E_RANGE, "vector::_M_range_check: __n (which is " + std::to_string(bp) +
                                    ") >= this->size() (which is " + std::to_string(ref_len) + ")");
    }
    if (ref_len == 0) return BC_OK;
    std::vector<int32_t> planes((size_t)ref_len * 6);
    rc = bc_memcpy_d2h(c, planes.data(), cl.hist, (size_t)ref_len * 6 * sizeof(int32_t));
    if (rc) return rc;
    rc = bc_sync(c);
    if (rc) return rc;
    for (int64_t p = 0; p < ref_len; ++p)
        for (int col = 0; col < 6; ++col) h_out[p * 6 + col] = (uint32_t)planes[(size_t)col * ref_len + p];
    return BC_OK;
}

}  // extern "C"
