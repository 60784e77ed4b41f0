// bcio.cpp — host BAM decode / encode and byte-exact formatter (see include/bcio.h).
//
// Decode pipeline (replaces pysam at /root/reference/basecount/main.py:119-127):
//   1. read the whole file, walk BGZF block headers (sequential, header hops only);
//   2. inflate every block in parallel (raw deflate: the system libdeflate when it loads, ~2.5x
//      zlib's speed on BAM blocks, else zlib) into one contiguous buffer;
//   3. parse the BAM header, then one sequential hop over record lengths that records the starts
//      and the prefix sums of cigar / seq sizes (prefetching ahead of its load chain);
//   4. parallel fill of a struct-of-arrays that is uploaded to HBM as is.
// The input is mmap'd and no large buffer is zero-filled: every byte of the inflate buffer and of
// the output arrays is first touched by the (parallel) thread that writes it.
// The pysam fields the reference reads (main.py:165-173) are reproduced exactly:
//   is_unmapped = flag & 4; mapping_quality; reference_start = pos; cigartuples (None if
//   n_cigar == 0); query_alignment_sequence / _qualities = SEQ/QUAL[qstart:qend] where
//   qstart/qend follow pysam's getQueryStart/getQueryEnd (leading S after optional H;
//   trailing S walking back but never looking at op 0), None if l_seq == 0 or QUAL[0] == 0xFF.
#include "../../include/bcio.h"

#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <chrono>
#include <memory>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include <dlfcn.h>
#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

int hw_threads(int n) {
    if (n > 0) return n;
    unsigned h = std::thread::hardware_concurrency();
    return h ? (int)std::min(h, 16u) : 4;
}

template <class F>
void parallel_for(int64_t n, int nthreads, F&& fn) {
    // dynamic chunked loop; fn(begin, end)
    if (n <= 0) return;
    nthreads = (int)std::max<int64_t>(1, std::min<int64_t>(nthreads, n));
    if (nthreads == 1) {
        fn((int64_t)0, n);
        return;
    }
    const int64_t chunk = std::max<int64_t>(1, n / (nthreads * 8));
    std::atomic<int64_t> next{0};
    std::vector<std::thread> ts;
    for (int t = 0; t < nthreads; ++t)
        ts.emplace_back([&] {
            for (;;) {
                int64_t b = next.fetch_add(chunk);
                if (b >= n) break;
                fn(b, std::min(n, b + chunk));
            }
        });
    for (auto& t : ts) t.join();
}

inline uint16_t rd16(const uint8_t* p) { return (uint16_t)(p[0] | (p[1] << 8)); }
inline uint32_t rd32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
inline int32_t rd32s(const uint8_t* p) { return (int32_t)rd32(p); }
inline void wr16(std::string& s, uint16_t v) {
    s.push_back((char)(v & 0xff));
    s.push_back((char)(v >> 8));
}
inline void wr32(std::string& s, uint32_t v) {
    for (int i = 0; i < 4; ++i) s.push_back((char)((v >> (8 * i)) & 0xff));
}

// munmap in 16 MiB pieces: one munmap of a GB-sized range holds the process's mmap lock for tens
// of ms, stalling every page fault and allocation of the other threads (the formatter right after
// a batch is released, say); in pieces they interleave.
inline void unmap_gradually(void* p, size_t n) {
    constexpr size_t kPiece = 16u << 20;
    uint8_t* b = (uint8_t*)p;
    for (size_t off = 0; off < n; off += kPiece) {
        munmap(b + off, std::min(kPiece, n - off));
        if (off + kPiece < n) sched_yield();
    }
}

// Anonymous mapping for the inflate buffer: no zero fill pass, hugepages where the kernel allows.
class MapBuf {
public:
    explicit MapBuf(size_t n) : n_(n) {
        if (n_ == 0) return;
        void* m = mmap(nullptr, n_, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (m == MAP_FAILED) return;
        madvise(m, n_, MADV_HUGEPAGE);
        p_ = (uint8_t*)m;
    }
    ~MapBuf() { release(); }
    MapBuf(const MapBuf&) = delete;
    MapBuf& operator=(const MapBuf&) = delete;
    bool ok() const { return n_ == 0 || p_ != nullptr; }
    uint8_t* data() { return p_; }
    size_t size() const { return n_; }
    void release() {
        if (p_) unmap_gradually(p_, n_);
        p_ = nullptr;
    }

private:
    uint8_t* p_ = nullptr;
    size_t n_ = 0;
};

// Read-only mapping of the BAM file (read() into a buffer only if mmap is refused).
class FileMap {
public:
    enum Advice { kWillNeed, kSequential, kRandom };
    int open(const char* path, bool sequential = false) { return open_as(path, sequential ? kSequential : kWillNeed); }
    int open_as(const char* path, Advice advice) {
        int fd = ::open(path, O_RDONLY | O_CLOEXEC);
        if (fd < 0) return -1;
        struct stat st;
        if (fstat(fd, &st) != 0) {
            ::close(fd);
            return -1;
        }
        n_ = (size_t)st.st_size;
        if (n_) {
            void* m = mmap(nullptr, n_, PROT_READ, MAP_PRIVATE, fd, 0);
            if (m != MAP_FAILED) {
                madvise(m, n_, advice == kSequential ? MADV_SEQUENTIAL : advice == kRandom ? MADV_RANDOM : MADV_WILLNEED);
                map_ = (const uint8_t*)m;
            } else {
                buf_.resize(n_);
                size_t got = 0;
                while (got < n_) {
                    ssize_t r = ::read(fd, buf_.data() + got, n_ - got);
                    if (r <= 0) break;
                    got += (size_t)r;
                }
                if (got != n_) {
                    ::close(fd);
                    return -2;
                }
            }
        }
        ::close(fd);
        return 0;
    }
    ~FileMap() { release(); }
    void release() {
        if (map_) unmap_gradually((void*)map_, n_);
        map_ = nullptr;
        buf_.clear();
        buf_.shrink_to_fit();
    }
    const uint8_t* data() const { return map_ ? map_ : buf_.data(); }
    size_t size() const { return n_; }
    // give pages of [off, off + len) back (page-aligned off); the mapping stays valid
    void drop(size_t off, size_t len) {
        if (map_ && len) madvise((void*)(map_ + off), len, MADV_DONTNEED);
    }

private:
    const uint8_t* map_ = nullptr;
    std::vector<uint8_t> buf_;
    size_t n_ = 0;
};

}  // namespace

// Default-initialising allocator: resize() leaves trivially constructible elements unwritten, so
// the parallel fill is the first (and only) writer of the output arrays.
template <class T>
struct UninitAlloc : std::allocator<T> {
    template <class U>
    struct rebind {
        using other = UninitAlloc<U>;
    };
    UninitAlloc() = default;
    template <class U>
    UninitAlloc(const UninitAlloc<U>&) noexcept {}
    template <class U>
    void construct(U* p) noexcept {
        ::new ((void*)p) U;
    }
    template <class U, class... A>
    void construct(U* p, A&&... a) {
        ::new ((void*)p) U(std::forward<A>(a)...);
    }
    // large arrays (a batch's sequence, qualities, CIGARs) straight from mmap, given back in
    // pieces (unmap_gradually) when the batch is released
    static constexpr size_t kBig = 4u << 20;
    T* allocate(size_t n) {
        const size_t bytes = n * sizeof(T);
        if (bytes < kBig) return std::allocator<T>::allocate(n);
        void* m = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (m == MAP_FAILED) throw std::bad_alloc();
        return (T*)m;
    }
    void deallocate(T* p, size_t n) {
        const size_t bytes = n * sizeof(T);
        if (bytes < kBig) std::allocator<T>::deallocate(p, n);
        else unmap_gradually(p, bytes);
    }
};
template <class T>
using uvec = std::vector<T, UninitAlloc<T>>;

struct bcio_file {
    std::vector<std::string> names;
    std::vector<int64_t> lens;
    // raw SoA
    uvec<int32_t> tid, pos, l_seq, qstart, qend;
    uvec<int64_t> ref_span;
    uvec<uint16_t> flag;
    uvec<uint8_t> mapq;
    uvec<uint32_t> rec_err;
    uvec<uint64_t> cig_off, seq_off;
    uvec<uint32_t> cigar;
    uvec<uint8_t> seq, qual;
    uvec<uint8_t> seq_ev;  // the same bases in the kernels' BC_SEQ_EVENT layout (+ zero pad)
    // selection outputs: one block per bcio_select call, alive until bcio_close
    struct Sel {
        std::vector<int64_t> ref_beg;
        uvec<int64_t> ordinal, rec, span;
        uvec<int32_t> pos;
        uvec<uint32_t> cig_beg, cig_n, seq_nib, qlen;
    };
    std::vector<std::unique_ptr<Sel>> sels;
};

extern "C" const char* bcio_last_error(void) { return g_err.c_str(); }

namespace {

// pysam getQueryStart (libcalignedsegment.pyx): leading soft clips, hard clips allowed only at the
// very start or once the whole query has been clipped.
int32_t query_start(const uint32_t* cig, uint32_t n, int32_t l_qseq, bool* bad) {
    int32_t start = 0;
    for (uint32_t k = 0; k < n; ++k) {
        uint32_t op = cig[k] & 0xf;
        if (op == 5) {
            if (start != 0 && start != l_qseq) *bad = true;
        } else if (op == 4) {
            start += (int32_t)(cig[k] >> 4);
        } else {
            break;
        }
    }
    return start;
}

// pysam getQueryEnd: walk back from the last op, never looking at op 0.
int32_t query_end(const uint32_t* cig, uint32_t n, int32_t l_qseq, bool* bad) {
    int32_t end = l_qseq;
    if (end == 0) {
        for (uint32_t k = 0; k < n; ++k) {
            uint32_t op = cig[k] & 0xf, len = cig[k] >> 4;
            if (op == 0 || op == 1 || op == 7 || op == 8 || (op == 4 && end == 0)) end += (int32_t)len;
        }
    } else {
        for (uint32_t k = n; k-- > 1;) {
            uint32_t op = cig[k] & 0xf;
            if (op == 5) {
                if (end != l_qseq) *bad = true;
            } else if (op == 4) {
                end -= (int32_t)(cig[k] >> 4);
            } else {
                break;
            }
        }
    }
    return end;
}

// libdeflate (Debian libdeflate0, ABI .so.0, stable since v1.0): whole-buffer raw-deflate
// decode, bound at run time so a missing library only costs speed.
struct Deflate {
    using Alloc = void* (*)();
    using Free = void (*)(void*);
    using Decomp = int (*)(void*, const void*, size_t, void*, size_t, size_t*);
    Alloc alloc = nullptr;
    Free free = nullptr;
    Decomp decomp = nullptr;
    Deflate() {
        if (std::getenv("BCIO_ZLIB")) return;
        void* h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
        if (!h) return;
        alloc = (Alloc)dlsym(h, "libdeflate_alloc_decompressor");
        free = (Free)dlsym(h, "libdeflate_free_decompressor");
        decomp = (Decomp)dlsym(h, "libdeflate_deflate_decompress");
        if (!alloc || !free || !decomp) alloc = nullptr;
    }
    bool ok() const { return alloc != nullptr; }
};

const Deflate& libdeflate() {
    static const Deflate d;
    return d;
}

// BAM 4-bit code -> BC_SEQ_EVENT class (basecount_hip.h): A 1, C 2, G 4, T 8, N 3, others 0
// ('=' and IUPAC codes count nowhere, count.cpp:58-65 through pysam's decode).  A BAM byte holds
// base 2m in its high nibble; the event layout keeps base i at bits 4*(i%8) of little-endian
// word i/8, i.e. base 2m in the LOW nibble of byte m: swap and classify, one table lookup.
struct EventLut {
    uint8_t t[256];
    EventLut() {
        static const uint8_t cls[16] = {0, 1, 2, 0, 4, 0, 0, 0, 8, 0, 0, 0, 0, 0, 0, 3};
        for (int b = 0; b < 256; ++b) t[b] = (uint8_t)(cls[b >> 4] | (cls[b & 15] << 4));
    }
};
const EventLut kEventLut;

inline void seq_to_event(const uint8_t* src, uint64_t n, uint8_t* dst) {
    for (uint64_t j = 0; j < n; ++j) dst[j] = kEventLut.t[src[j]];
}

// bytes of a BC_SEQ_EVENT buffer for n packed bytes (= bc_seq_event_bytes of basecount_hip.h)
inline uint64_t seq_event_bytes(uint64_t n) { return (n + 15) / 16 * 16 + 16; }

struct Block {
    uint64_t coff, clen, uoff;
    uint32_t isize;
};

}  // namespace

struct PhaseTimer {  // BCIO_PROFILE=1: per-phase wall times of bcio_open on stderr
    bool on = std::getenv("BCIO_PROFILE") != nullptr;
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    void mark(const char* what) {
        if (!on) return;
        auto now = std::chrono::steady_clock::now();
        std::fprintf(stderr, "bcio %-10s %8.1f ms\n", what, std::chrono::duration<double, std::milli>(now - t).count());
        t = now;
    }
};

namespace {

// One BGZF block header at h[0, avail).  BCIO_OK: *b holds the deflate data's offset (from h),
// length and inflated size, *bsize the whole block's size; 1: the block is cut off at avail (the
// message says where); < 0: malformed.
int scan_block(const uint8_t* h, uint64_t avail, Block* b, uint64_t* bsize_out) {
    if (avail < 18) return (g_err = "truncated BGZF header", 1);
    if (h[0] != 31 || h[1] != 139 || h[2] != 8 || !(h[3] & 4))
        return fail(BCIO_E_FORMAT, "not a BGZF file (bad gzip magic / no FEXTRA)");
    uint16_t xlen = rd16(h + 10);
    // the extra field itself must lie inside the file before any subfield is read
    if ((uint64_t)12 + xlen > avail) return (g_err = "truncated BGZF extra field", 1);
    uint64_t bsize = 0;
    bool found = false;
    for (uint32_t x = 0; x + 4 <= xlen;) {
        const uint8_t* sf = h + 12 + x;
        uint16_t slen = rd16(sf + 2);
        if ((uint64_t)x + 4 + slen > xlen) return fail(BCIO_E_FORMAT, "BGZF subfield past the extra field");
        if (sf[0] == 66 && sf[1] == 67 && slen == 2) {
            bsize = (uint64_t)rd16(sf + 4) + 1;
            found = true;
        }
        x += 4 + slen;
    }
    if (!found) return fail(BCIO_E_FORMAT, "BGZF block without BC subfield");
    // header (12 + xlen) + deflate data + CRC32 + ISIZE (8): a smaller BSIZE would underflow
    // the compressed length handed to the inflater
    if (bsize < (uint64_t)12 + xlen + 8) return fail(BCIO_E_FORMAT, "BGZF block size smaller than its header");
    if (bsize > avail) return (g_err = "truncated BGZF block", 1);
    b->coff = 12 + xlen;
    b->clen = bsize - xlen - 20;
    b->isize = rd32(h + bsize - 4);
    b->uoff = 0;
    if (b->isize > 65536) return fail(BCIO_E_FORMAT, "BGZF block inflates past 64 KiB");
    *bsize_out = bsize;
    return BCIO_OK;
}

// Inflate every block (deflate data at comp + coff) to out + uoff, on nthreads threads.
bool inflate_blocks(const uint8_t* comp, const std::vector<Block>& blocks, uint8_t* out, int nthreads) {
    std::atomic<int> zerr{0};
    const Deflate& ld = libdeflate();
    parallel_for((int64_t)blocks.size(), nthreads, [&](int64_t b0, int64_t b1) {
        if (ld.ok()) {
            void* d = ld.alloc();
            if (!d) {
                zerr = 1;
                return;
            }
            for (int64_t i = b0; i < b1; ++i) {
                const Block& b = blocks[i];
                if (b.isize == 0) continue;
                size_t got = 0;
                if (ld.decomp(d, comp + b.coff, b.clen, out + b.uoff, b.isize, &got) != 0 || got != b.isize)
                    zerr = 1;
            }
            ld.free(d);
            return;
        }
        z_stream zs;
        std::memset(&zs, 0, sizeof zs);
        if (inflateInit2(&zs, -15) != Z_OK) {
            zerr = 1;
            return;
        }
        for (int64_t i = b0; i < b1; ++i) {
            const Block& b = blocks[i];
            if (b.isize == 0) continue;
            inflateReset(&zs);
            zs.next_in = const_cast<uint8_t*>(comp + b.coff);
            zs.avail_in = (uInt)b.clen;
            zs.next_out = out + b.uoff;
            zs.avail_out = b.isize;
            int r = inflate(&zs, Z_FINISH);
            if (r != Z_STREAM_END || zs.avail_out != 0) zerr = 1;
        }
        inflateEnd(&zs);
    });
    return zerr == 0;
}

// The BAM header (magic, text, reference list) at p[0, N): BCIO_OK and *q_end = first record
// offset; 1 = more bytes needed (the message says what is truncated); < 0 = malformed.
int parse_header(const uint8_t* p, uint64_t N, std::vector<std::string>& names, std::vector<int64_t>& lens,
                 uint64_t* q_end) {
    names.clear();
    lens.clear();
    if (N < 4) return (g_err = "missing BAM magic", 1);
    if (std::memcmp(p, "BAM\1", 4) != 0) return fail(BCIO_E_FORMAT, "missing BAM magic");
    if (N < 12) return (g_err = "missing BAM magic", 1);
    uint64_t q = 4;
    int32_t l_text = rd32s(p + q);
    q += 4;
    if (l_text < 0) return fail(BCIO_E_FORMAT, "bad header text length");
    if (q + (uint64_t)l_text + 4 > N) return (g_err = "bad header text length", 1);
    q += (uint64_t)l_text;
    int32_t n_ref = rd32s(p + q);
    q += 4;
    if (n_ref < 0) return fail(BCIO_E_FORMAT, "negative n_ref");
    for (int32_t i = 0; i < n_ref; ++i) {
        if (q + 4 > N) return (g_err = "truncated reference list", 1);
        int32_t ln = rd32s(p + q);
        q += 4;
        if (ln <= 0) return fail(BCIO_E_FORMAT, "truncated reference name");
        if (q + (uint64_t)ln + 4 > N) return (g_err = "truncated reference name", 1);
        names.emplace_back((const char*)(p + q), strnlen((const char*)(p + q), (size_t)ln));
        q += (uint64_t)ln;
        lens.push_back((int64_t)rd32s(p + q));
        q += 4;
    }
    *q_end = q;
    return BCIO_OK;
}

}  // namespace

// The hop over record lengths: starts of the complete records and the prefix sums of their cigar
// / seq sizes, continued from where it stopped (q) at each call.  With partial_ok a truncated
// record at the end waits for more bytes; without, it is a format error.
struct Hop {
    uvec<uint64_t> starts;
    uvec<uint64_t> cig_off{0}, seq_off{0};
    uint64_t q = 0, cig_tot = 0, seq_tot = 0, pf = 0;
};

int hop_records(Hop& h, const uint8_t* p, uint64_t N, int64_t max_records, bool partial_ok) {
    constexpr uint64_t kPf = 4096;  // prefetch distance: the hop's dependent loads become a stream
    uint64_t q = h.q;
    while (q < N && (int64_t)h.starts.size() < max_records) {
        if (q + 4 > N) {
            if (partial_ok) break;
            return fail(BCIO_E_FORMAT, "truncated record length");
        }
        uint32_t bs = rd32(p + q);
        if (bs < 32) return fail(BCIO_E_FORMAT, "truncated BAM record");
        if (q + 4 + bs > N) {
            if (partial_ok) break;
            return fail(BCIO_E_FORMAT, "truncated BAM record");
        }
        const uint64_t pf_end = std::min(N, q + 4 + bs + kPf);
        for (h.pf = std::max(h.pf, q + kPf); h.pf < pf_end; h.pf += 64) __builtin_prefetch(p + h.pf);
        const uint8_t* r = p + q + 4;
        int32_t ls = rd32s(r + 16);
        if (ls < 0) return fail(BCIO_E_FORMAT, "negative l_seq");
        // the fields must fit the record before their sizes feed the output allocations
        if (32ull + r[8] + 4ull * rd16(r + 12) + (((uint64_t)ls + 1) / 2) + (uint64_t)ls > bs)
            return fail(BCIO_E_FORMAT, "BAM record shorter than its fields");
        h.starts.push_back(q);
        h.cig_tot += rd16(r + 12);
        h.seq_tot += (((uint64_t)ls + 1) / 2);
        h.cig_off.push_back(h.cig_tot);
        h.seq_off.push_back(h.seq_tot);
        q += 4 + (uint64_t)bs;
    }
    h.q = q;
    return BCIO_OK;
}

int fill_records(bcio_file* f, const uint8_t* p, Hop& h, int nthreads, PhaseTimer* pt);

// Records from p[q0, N) into f's struct of arrays: at most max_records complete records (see
// hop_records), then a parallel fill; *q_end = the offset after the last one.
int decode_records(bcio_file* f, const uint8_t* p, uint64_t q0, uint64_t N, int64_t max_records, bool partial_ok,
                   int nthreads, uint64_t* q_end, PhaseTimer* pt) {
    Hop h;
    h.q = h.pf = q0;
    const uint64_t guess = std::max<uint64_t>(16, std::min<uint64_t>((N - q0) / 256, (uint64_t)std::max<int64_t>(16, max_records)));
    h.starts.reserve(guess);
    h.cig_off.reserve(guess + 1);
    h.seq_off.reserve(guess + 1);
    int rc = hop_records(h, p, N, max_records, partial_ok);
    if (rc != BCIO_OK) return rc;
    *q_end = h.q;
    return fill_records(f, p, h, nthreads, pt);
}

int fill_records(bcio_file* f, const uint8_t* p, Hop& h, int nthreads, PhaseTimer* pt) {
    uvec<uint64_t>& starts = h.starts;
    const uint64_t cig_tot = h.cig_tot, seq_tot = h.seq_tot;
    f->cig_off.swap(h.cig_off);
    f->seq_off.swap(h.seq_off);
    const int64_t n = (int64_t)starts.size();
    f->tid.resize(n);
    f->pos.resize(n);
    f->l_seq.resize(n);
    f->qstart.resize(n);
    f->qend.resize(n);
    f->ref_span.resize(n);
    f->flag.resize(n);
    f->mapq.resize(n);
    f->rec_err.resize(n);
    f->cigar.resize(cig_tot);
    f->seq.resize(seq_tot);
    f->seq_ev.resize(seq_event_bytes(seq_tot));
    std::memset(f->seq_ev.data() + seq_tot, 0, f->seq_ev.size() - seq_tot);
    f->qual.resize(2 * seq_tot);
    if (pt) pt->mark("starts");
    std::atomic<int> ferr{0};
    parallel_for(n, nthreads, [&](int64_t b0, int64_t b1) {
        for (int64_t i = b0; i < b1; ++i) {
            const uint8_t* r = p + starts[i] + 4;
            uint32_t bs = rd32(p + starts[i]);
            int32_t t = rd32s(r + 0), ps = rd32s(r + 4);
            uint8_t lrn = r[8], mq = r[9];
            uint16_t nc = rd16(r + 12), fl = rd16(r + 14);
            int32_t ls = rd32s(r + 16);
            uint64_t need = 32 + (uint64_t)lrn + 4ull * nc + (((uint64_t)ls + 1) / 2) + (uint64_t)ls;
            if (need > bs) {
                ferr = 1;
                continue;
            }
            f->tid[i] = t;
            f->pos[i] = ps;
            f->mapq[i] = mq;
            f->flag[i] = fl;
            f->l_seq[i] = ls;
            const uint8_t* c = r + 32 + lrn;
            uint32_t* cd = f->cigar.data() + f->cig_off[i];
            int64_t span = 0;  // reference-consuming ops M D N = X
            for (uint16_t k = 0; k < nc; ++k) {
                uint32_t w = rd32(c + 4 * k);
                cd[k] = w;
                if ((0x18Du >> (w & 0xf)) & 1) span += w >> 4;
            }
            f->ref_span[i] = span;
            const uint8_t* s = c + 4ull * nc;
            uint64_t sb = (((uint64_t)ls + 1) / 2);
            std::memcpy(f->seq.data() + f->seq_off[i], s, sb);
            seq_to_event(s, sb, f->seq_ev.data() + f->seq_off[i]);
            const uint8_t* ql = s + sb;
            uint8_t* qd = f->qual.data() + 2 * f->seq_off[i];
            std::memcpy(qd, ql, (size_t)ls);
            if (ls & 1) qd[ls] = 0xFF;  // pad byte of an odd-length read
            uint32_t err = 0;
            if (nc == 0) err |= BCIO_REC_NO_CIGAR;
            if (ls == 0) err |= BCIO_REC_NO_SEQ;
            if (ls == 0 || ql[0] == 0xFF) err |= BCIO_REC_NO_QUAL;
            bool badclip = false;
            f->qstart[i] = query_start(cd, nc, ls, &badclip);
            f->qend[i] = query_end(cd, nc, ls, &badclip);
            if (badclip) err |= BCIO_REC_BAD_CLIP;
            if (ps < 0) err |= BCIO_REC_NEG_POS;
            f->rec_err[i] = err;
        }
    });
    if (ferr) return fail(BCIO_E_FORMAT, "BAM record shorter than its fields");
    if (pt) pt->mark("fill");
    return BCIO_OK;
}

extern "C" int bcio_open(const char* path, int nthreads, bcio_file** out) {
    if (!path || !out) return fail(BCIO_E_ARG, "null argument");
    PhaseTimer pt;
    nthreads = hw_threads(nthreads);
    FileMap file;
    int orc = file.open(path);
    if (orc == -1) return fail(BCIO_E_IO, std::string("cannot open ") + path);
    if (orc != 0) return fail(BCIO_E_IO, "short read");
    const uint8_t* comp = file.data();
    const uint64_t comp_n = file.size();
    pt.mark("read");
    // 1. BGZF block scan
    std::vector<Block> blocks;
    uint64_t off = 0, uoff = 0;
    while (off < comp_n) {
        Block b;
        uint64_t bsize = 0;
        int src = scan_block(comp + off, comp_n - off, &b, &bsize);
        if (src == 1) return fail(BCIO_E_FORMAT, g_err);
        if (src != BCIO_OK) return src;
        b.coff += off;
        b.uoff = uoff;
        uoff += b.isize;
        blocks.push_back(b);
        off += bsize;
    }
    pt.mark("scan");
    // 2. parallel inflate
    MapBuf raw(uoff);
    if (!raw.ok()) return fail(BCIO_E_IO, "cannot allocate the inflate buffer");
    pt.mark("alloc");
    if (!inflate_blocks(comp, blocks, raw.data(), nthreads)) return fail(BCIO_E_ZLIB, "inflate failed");
    pt.mark("inflate");
    file.release();

    // 3. BAM header, then every record
    auto* f = new bcio_file();
    const uint8_t* p = raw.data();
    const uint64_t N = raw.size();
    uint64_t q = 0;
    int hrc = parse_header(p, N, f->names, f->lens, &q);
    if (hrc != BCIO_OK) {
        delete f;
        return hrc > 0 ? fail(BCIO_E_FORMAT, g_err) : hrc;
    }
    uint64_t q_end = q;
    int drc = decode_records(f, p, q, N, INT64_MAX, false, nthreads, &q_end, &pt);
    if (drc != BCIO_OK) {
        delete f;
        return drc;
    }
    raw.release();
    *out = f;
    return BCIO_OK;
}

// Returning a few hundred MB of decoded arrays to the kernel takes tens of ms; nothing waits for
// it, so it happens on a detached thread (synchronously if a thread cannot be started).
extern "C" void bcio_close(bcio_file* f) {
    if (!f) return;
    try {
        std::thread([f] { delete f; }).detach();
    } catch (...) {
        delete f;
    }
}
extern "C" int32_t bcio_n_refs(const bcio_file* f) { return f ? (int32_t)f->names.size() : 0; }
extern "C" const char* bcio_ref_name(const bcio_file* f, int32_t i) {
    return (f && i >= 0 && i < (int32_t)f->names.size()) ? f->names[i].c_str() : nullptr;
}
extern "C" int64_t bcio_ref_len(const bcio_file* f, int32_t i) {
    return (f && i >= 0 && i < (int32_t)f->lens.size()) ? f->lens[i] : -1;
}

extern "C" int bcio_get_records(const bcio_file* f, bcio_records* o) {
    if (!f || !o) return fail(BCIO_E_ARG, "null argument");
    o->n = (int64_t)f->tid.size();
    o->tid = f->tid.data();
    o->pos = f->pos.data();
    o->flag = f->flag.data();
    o->mapq = f->mapq.data();
    o->l_seq = f->l_seq.data();
    o->qstart = f->qstart.data();
    o->qend = f->qend.data();
    o->rec_err = f->rec_err.data();
    o->cig_off = f->cig_off.data();
    o->cigar = f->cigar.data();
    o->seq_off = f->seq_off.data();
    o->seq = f->seq.data();
    o->qual = f->qual.data();
    o->seq_bytes = f->seq_off.empty() ? 0 : f->seq_off.back();
    o->ref_span = f->ref_span.data();
    o->seq_event = f->seq_ev.data();
    o->seq_event_bytes = (uint64_t)f->seq_ev.size();
    return BCIO_OK;
}

extern "C" int bcio_select(bcio_file* f, int64_t min_mapq, const uint8_t* ref_sel, bcio_selection* o) {
    if (!f || !o || !ref_sel) return fail(BCIO_E_ARG, "null argument");
    f->sels.emplace_back(new bcio_file::Sel());
    bcio_file::Sel& S = *f->sels.back();
    const int64_t n = (int64_t)f->tid.size();
    const int32_t nr = (int32_t)f->names.size();
    // accepted = mapped and mapq >= mmq (main.py:165); is_unmapped is flag bit 4 only.
    // Two parallel passes over fixed record chunks: count per (chunk, reference), then scatter
    // at offsets that keep file order within each reference.
    auto accepted = [&](int64_t i) { return !(f->flag[i] & 4) && (int64_t)f->mapq[i] >= min_mapq; };
    auto wanted = [&](int32_t t) { return t >= 0 && t < nr && ref_sel[t]; };
    const int64_t per = 1 << 16;
    const int64_t nch = (n + per - 1) / per;
    const int cols = nr + 1;  // per-reference counts + accepted ordinals of the chunk
    std::vector<int64_t> cc((size_t)(nch * cols), 0);
    std::vector<int64_t> ke_rec((size_t)nch, -1), ke_ord((size_t)nch, -1);
    const int nthreads = hw_threads(0);
    parallel_for(nch, nthreads, [&](int64_t c0, int64_t c1) {
        for (int64_t c = c0; c < c1; ++c) {
            int64_t* row = &cc[(size_t)(c * cols)];
            int64_t ord = 0;
            for (int64_t i = c * per, e = std::min(n, i + per); i < e; ++i) {
                if (!accepted(i)) continue;
                int32_t t = f->tid[i];
                if (wanted(t))
                    row[t]++;
                else if (ke_rec[c] < 0) {
                    ke_rec[c] = i;
                    ke_ord[c] = ord;
                }
                ord++;
            }
            row[nr] = ord;
        }
    });
    S.ref_beg.assign(nr + 1, 0);
    for (int64_t c = 0; c < nch; ++c)
        for (int32_t t = 0; t < nr; ++t) S.ref_beg[t + 1] += cc[(size_t)(c * cols + t)];
    for (int32_t t = 0; t < nr; ++t) S.ref_beg[t + 1] += S.ref_beg[t];
    // chunk c's first slot per reference, and its first ordinal
    std::vector<int64_t> ord0((size_t)nch + 1, 0);
    std::vector<int64_t> run(S.ref_beg.begin(), S.ref_beg.end() - 1);
    o->keyerror_ordinal = -1;
    o->keyerror_rec = -1;
    for (int64_t c = 0; c < nch; ++c) {
        int64_t* row = &cc[(size_t)(c * cols)];
        for (int32_t t = 0; t < nr; ++t) {
            int64_t k = row[t];
            row[t] = run[t];
            run[t] += k;
        }
        if (o->keyerror_rec < 0 && ke_rec[c] >= 0) {
            o->keyerror_rec = ke_rec[c];
            o->keyerror_ordinal = ord0[c] + ke_ord[c];
        }
        ord0[c + 1] = ord0[c] + row[nr];
    }
    o->n_accepted = ord0[nch];
    const int64_t m = S.ref_beg[nr];
    S.pos.resize(m);
    S.cig_beg.resize(m);
    S.cig_n.resize(m);
    S.seq_nib.resize(m);
    S.qlen.resize(m);
    S.ordinal.resize(m);
    S.rec.resize(m);
    S.span.resize(m);
    parallel_for(nch, nthreads, [&](int64_t c0, int64_t c1) {
        for (int64_t c = c0; c < c1; ++c) {
            int64_t* slot = &cc[(size_t)(c * cols)];
            int64_t ordinal = ord0[c];
            for (int64_t i = c * per, e = std::min(n, i + per); i < e; ++i) {
                if (!accepted(i)) continue;
                int32_t t = f->tid[i];
                if (wanted(t)) {
                    int64_t j = slot[t]++;
                    S.pos[j] = f->pos[i];
                    S.cig_beg[j] = (uint32_t)f->cig_off[i];
                    S.cig_n[j] = (uint32_t)(f->cig_off[i + 1] - f->cig_off[i]);
                    S.seq_nib[j] = (uint32_t)(2 * f->seq_off[i] + (uint64_t)std::max(0, f->qstart[i]));
                    int32_t ql = f->qend[i] - f->qstart[i];
                    S.qlen[j] = (uint32_t)std::max(0, ql);
                    S.ordinal[j] = ordinal;
                    S.rec[j] = i;
                    S.span[j] = f->ref_span[i];
                }
                ordinal++;
            }
        }
    });
    o->ref_beg = S.ref_beg.data();
    o->pos = S.pos.data();
    o->cig_beg = S.cig_beg.data();
    o->cig_n = S.cig_n.data();
    o->seq_nib = S.seq_nib.data();
    o->qlen = S.qlen.data();
    o->ordinal = S.ordinal.data();
    o->rec = S.rec.data();
    o->span = S.span.data();
    if (f->cig_off.back() > 0xFFFFFFFFull || 2 * f->seq_off.back() > 0xFFFFFFFFull)
        return fail(BCIO_E_ARG, "file too large for 32-bit batch offsets; split it");
    return BCIO_OK;
}

// ------------------------------------------------------------------------------------------
// streaming decode (bounded memory).  The file is mapped read-only; each fill scans BGZF block
// headers ahead until the blocks hold the bytes the batch is estimated to need (from the
// records' mean size so far), inflates all of them in ONE parallel pass into a buffer sized
// once (the carried partial record first), and drops the consumed part of the mapping
// (MADV_DONTNEED), so resident memory is one batch plus its inflated bytes, never the file.
struct bcio_stream {
    FileMap file;
    uint64_t coff = 0;  // next block to scan
    int nthreads = 1;
    std::vector<std::string> names;
    std::vector<int64_t> lens;
    std::unique_ptr<MapBuf> pend;  // inflated bytes (anonymous mapping: no zero fill)
    uint64_t pend_n = 0;           // bytes used in pend; [pbeg, pend_n) not handed out yet
    uint64_t pbeg = 0;
    Hop hop;  // the next batch's records counted so far (offsets from pbeg)
    uint64_t dropped = 0;  // mapping bytes already given back
    double rec_bytes = 0.0;  // mean inflated bytes per record so far
    int64_t returned = 0;
    // range streams (bcio_stream_open_range): blocks are scanned below cend only, and the block at
    // tail_block (if any) keeps its first tail_keep inflated bytes
    uint64_t cend = UINT64_MAX, tail_block = UINT64_MAX, tail_keep = 0;
    bool all_read() const { return coff >= std::min<uint64_t>(cend, file.size()); }
    const uint8_t* base() const { return pend ? pend->data() + pbeg : nullptr; }
    uint64_t avail() const { return pend_n - pbeg; }
};

namespace {

// scan + inflate blocks from coff until they hold >= want inflated bytes (or the file ends)
int stream_fill(bcio_stream* s, uint64_t want) {
    const uint8_t* comp = s->file.data();
    const uint64_t n = s->file.size();
    std::vector<Block> blocks;
    uint64_t off = s->coff, uoff = 0, trim = 0;
    const uint64_t lim = std::min<uint64_t>(n, s->cend);
    while (off < lim && uoff < want) {
        Block b;
        uint64_t bsize = 0;
        int rc = scan_block(comp + off, n - off, &b, &bsize);
        if (rc == 1) return fail(BCIO_E_FORMAT, g_err);  // a block cut off by the end of the file
        if (rc != BCIO_OK) return rc;
        b.coff += off;
        b.uoff = uoff;
        uoff += b.isize;
        blocks.push_back(b);
        if (off == s->tail_block) {  // the range ends inside this block
            if (s->tail_keep > b.isize) return fail(BCIO_E_ARG, "range end past its block");
            trim = b.isize - s->tail_keep;
        }
        off += bsize;
    }
    // one buffer: the bytes not handed out yet, then the new blocks' bytes
    const uint64_t keep = s->avail();
    auto next = std::make_unique<MapBuf>(keep + uoff + 64);
    if (!next->ok()) return fail(BCIO_E_IO, "cannot allocate the inflate buffer");
    if (keep) std::memcpy(next->data(), s->base(), keep);
    if (!inflate_blocks(comp, blocks, next->data() + keep, s->nthreads)) return fail(BCIO_E_ZLIB, "inflate failed");
    s->pend = std::move(next);
    s->pend_n = keep + uoff - trim;
    s->pbeg = 0;
    s->coff = off;
    // give the consumed compressed pages back (whole pages below the next block)
    const uint64_t page = 4096, upto = off / page * page;
    if (upto > s->dropped) {
        s->file.drop(s->dropped, upto - s->dropped);
        s->dropped = upto;
    }
    return BCIO_OK;
}

void hop_reset(Hop& h) {
    h = Hop();
}

}  // namespace

extern "C" int bcio_stream_open(const char* path, int nthreads, bcio_stream** out) {
    if (!path || !out) return fail(BCIO_E_ARG, "null argument");
    *out = nullptr;
    auto s = std::make_unique<bcio_stream>();
    int orc = s->file.open(path, /*sequential=*/true);
    if (orc == -1) return fail(BCIO_E_IO, std::string("cannot open ") + path);
    if (orc != 0) return fail(BCIO_E_IO, "short read");
    s->nthreads = hw_threads(nthreads);
    uint64_t want = 256u << 10;
    for (;;) {  // the header, however many blocks it takes
        uint64_t q = 0;
        int rc = parse_header(s->base(), s->avail(), s->names, s->lens, &q);
        if (rc == BCIO_OK) {
            s->pbeg += q;
            break;
        }
        if (rc < 0) return rc;
        if (s->all_read()) return fail(BCIO_E_FORMAT, g_err);
        if ((rc = stream_fill(s.get(), want)) != BCIO_OK) return rc;
        want *= 2;
    }
    *out = s.release();
    return BCIO_OK;
}

extern "C" int bcio_stream_next(bcio_stream* s, int64_t max_records, bcio_file** out) {
    if (!s || !out || max_records <= 0) return fail(BCIO_E_ARG, "bad argument");
    *out = nullptr;
    // the hop over the next batch's records, continued after each fill (each byte hopped once)
    Hop& h = s->hop;
    for (;;) {
        int rc = hop_records(h, s->base(), s->avail(), max_records, /*partial_ok=*/true);
        if (rc != BCIO_OK) return rc;
        const int64_t m = (int64_t)h.starts.size();
        if (m >= max_records || s->all_read()) break;
        // the bytes the missing records should take (mean record size so far), at least 8 MiB
        const double per = m > 0 ? (double)h.q / (double)m : (s->rec_bytes > 0 ? s->rec_bytes : 512.0);
        const double need = per * (double)(max_records - m) * 1.05 + 65536.0;
        const uint64_t want = (uint64_t)std::min(std::max(need, 8.0 * (1 << 20)), 8.0 * (1ull << 30));
        if ((rc = stream_fill(s, want)) != BCIO_OK) return rc;
    }
    if (h.starts.empty()) {
        if (s->avail())  // bytes left that never make a whole record
            return fail(BCIO_E_FORMAT, s->avail() < 4 ? "truncated record length" : "truncated BAM record");
        return BCIO_OK;  // end of file
    }
    auto* f = new bcio_file();
    f->names = s->names;
    f->lens = s->lens;
    const uint64_t used = h.q;
    const int64_t got = (int64_t)h.starts.size();
    int rc = fill_records(f, s->base(), h, s->nthreads, nullptr);
    hop_reset(h);
    if (rc != BCIO_OK) {
        delete f;
        return rc;
    }
    s->rec_bytes = (double)used / (double)got;
    s->pbeg += used;
    s->returned += got;
    *out = f;
    return BCIO_OK;
}

extern "C" int64_t bcio_stream_records(const bcio_stream* s) { return s ? s->returned : -1; }
extern "C" int32_t bcio_stream_n_refs(const bcio_stream* s) { return s ? (int32_t)s->names.size() : 0; }
extern "C" const char* bcio_stream_ref_name(const bcio_stream* s, int32_t i) {
    return (s && i >= 0 && i < (int32_t)s->names.size()) ? s->names[i].c_str() : nullptr;
}
extern "C" int64_t bcio_stream_ref_len(const bcio_stream* s, int32_t i) {
    return (s && i >= 0 && i < (int32_t)s->lens.size()) ? s->lens[i] : -1;
}
// like bcio_close: unmapping a batch-sized buffer takes ms, nothing waits for it
extern "C" void bcio_stream_close(bcio_stream* s) {
    if (!s) return;
    try {
        std::thread([s] { delete s; }).detach();
    } catch (...) {
        delete s;
    }
}

// ------------------------------------------------------------------------------------------
// Record-aligned split points for decoding one file on several ranks (bcio.h: sharded decode).
// Virtual offsets as in a BAM index: (block file offset << 16) | offset in its inflated bytes.
namespace {

// Inflated bytes of consecutive blocks, with where each block lies in the file and in buf.
struct Span {
    std::vector<uint8_t> buf;
    std::vector<uint64_t> boff, ustart;
    uint64_t next = 0;  // file offset after the last block
    bool eof = false;
};

// append blocks from sp.next until buf holds >= want bytes (or the file ends); single thread
int span_grow(const uint8_t* comp, uint64_t n, Span& sp, uint64_t want) {
    while (!sp.eof && sp.buf.size() < want) {
        if (sp.next >= n) {
            sp.eof = true;
            break;
        }
        Block b;
        uint64_t bsize = 0;
        int rc = scan_block(comp + sp.next, n - sp.next, &b, &bsize);
        if (rc == 1) return fail(BCIO_E_FORMAT, g_err);
        if (rc != BCIO_OK) return rc;
        b.coff += sp.next;
        b.uoff = sp.buf.size();
        sp.boff.push_back(sp.next);
        sp.ustart.push_back(b.uoff);
        sp.buf.resize(b.uoff + b.isize);
        if (!inflate_blocks(comp, std::vector<Block>{b}, sp.buf.data(), 1)) return fail(BCIO_E_ZLIB, "inflate failed");
        sp.next += bsize;
    }
    return BCIO_OK;
}

// virtual offset of byte u of the span (a record start); u at the very end: the next block
uint64_t span_voff(const Span& sp, uint64_t u) {
    if (u >= sp.buf.size()) return sp.next << 16;
    size_t j = (size_t)(std::upper_bound(sp.ustart.begin(), sp.ustart.end(), u) - sp.ustart.begin()) - 1;
    // an empty block shares its start with the next one: take the last block starting at or before u
    return (sp.boff[j] << 16) | (u - sp.ustart[j]);
}

// the record at p[q, N) looks like a BAM record of a file with n_ref references: its size
// (4 + block_size), 0 if not (or if it is cut off by N)
uint64_t plausible_record(const uint8_t* p, uint64_t q, uint64_t N, int32_t n_ref) {
    if (q + 36 > N) return 0;
    const uint32_t bs = rd32(p + q);
    if (bs < 32 || bs > (1u << 28) || q + 4 + bs > N) return 0;
    const uint8_t* r = p + q + 4;
    const int32_t tid = rd32s(r), pos = rd32s(r + 4), ls = rd32s(r + 16), ntid = rd32s(r + 20), npos = rd32s(r + 24);
    const uint8_t lrn = r[8];
    if (tid < -1 || tid >= n_ref || ntid < -1 || ntid >= n_ref || pos < -1 || npos < -1 || ls < 0 || lrn < 1) return 0;
    if (32ull + lrn + 4ull * rd16(r + 12) + (((uint64_t)ls + 1) / 2) + (uint64_t)ls > bs) return 0;
    const uint8_t* nm = r + 32;
    if (nm[lrn - 1] != 0) return 0;
    for (int i = 0; i + 1 < lrn; ++i)
        if (nm[i] < 33 || nm[i] > 126) return 0;
    return 4ull + bs;
}

// the first offset in [0, lim) where a chain of 4 plausible records starts (or one that ends
// exactly at the end of the file's data), -1 if none
int64_t sync_records(const Span& sp, uint64_t lim, int32_t n_ref) {
    const uint8_t* p = sp.buf.data();
    const uint64_t N = sp.buf.size();
    for (uint64_t o = 0; o < lim && o < N; ++o) {
        uint64_t q = o;
        int k = 0;
        while (k < 4) {
            const uint64_t sz = plausible_record(p, q, N, n_ref);
            if (!sz) break;
            q += sz;
            ++k;
            if (q == N && sp.eof) break;
        }
        if (k >= 4 || (k >= 1 && q == N && sp.eof)) return (int64_t)o;
    }
    return -1;
}

// the first BGZF block header at or after x whose chain of three blocks parses (or reaches the
// end of the file), -1 if none
int64_t sync_block(const uint8_t* comp, uint64_t n, uint64_t x) {
    for (uint64_t o = x; o + 18 <= n; ++o) {
        if (comp[o] != 31 || comp[o + 1] != 139 || comp[o + 2] != 8 || !(comp[o + 3] & 4)) continue;
        uint64_t q = o;
        int k = 0;
        bool ok = true;
        while (k < 3 && q < n) {
            Block b;
            uint64_t bsize = 0;
            if (scan_block(comp + q, n - q, &b, &bsize) != BCIO_OK) {
                ok = false;
                break;
            }
            q += bsize;
            ++k;
        }
        if (ok && (k == 3 || q == n)) return (int64_t)o;
    }
    return -1;
}

// the header of a mapped file: reference count and the first record's virtual offset
int header_span(const uint8_t* comp, uint64_t n, int32_t* n_ref, uint64_t* first) {
    Span sp;
    std::vector<std::string> names;
    std::vector<int64_t> lens;
    for (uint64_t want = 65536;; want *= 2) {
        int rc = span_grow(comp, n, sp, want);
        if (rc != BCIO_OK) return rc;
        uint64_t q = 0;
        rc = parse_header(sp.buf.data(), sp.buf.size(), names, lens, &q);
        if (rc == BCIO_OK) {
            *n_ref = (int32_t)names.size();
            *first = span_voff(sp, q);
            return BCIO_OK;
        }
        if (rc < 0) return rc;
        if (sp.eof) return fail(BCIO_E_FORMAT, g_err);
    }
}

}  // namespace

extern "C" int bcio_find_record(const char* path, int32_t tid, int32_t pos, uint64_t* voff) {
    if (!path || !voff) return fail(BCIO_E_ARG, "null argument");
    // the first record at or past (tid, pos): refID -1 (unmapped) sorts after every reference
    auto past = [tid, pos](int32_t ref, int32_t rpos) { return ref < 0 || ref > tid || (ref == tid && rpos >= pos); };
    FileMap fm;
    const int orc = fm.open_as(path, FileMap::kRandom);  // a few probes: no readahead of the file
    if (orc == -1) return fail(BCIO_E_IO, std::string("cannot open ") + path);
    if (orc != 0) return fail(BCIO_E_IO, "short read");
    const uint8_t* comp = fm.data();
    const uint64_t n = fm.size();
    int32_t n_ref = 0;
    uint64_t first = 0;
    int rc = header_span(comp, n, &n_ref, &first);
    if (rc != BCIO_OK) return rc;
    // lo: a record start (virtual offset) whose refID is below tid; the boundary lies after it
    uint64_t lo = first;
    // hi: a file offset such that the first record synchronised in any block at or after it has
    // refID >= tid (or -1); the bisection narrows [lo's block, hi) to a few blocks
    uint64_t hi = n;
    {  // the first record itself
        Span sp;
        sp.next = first >> 16;
        const uint64_t u = first & 0xFFFF;
        if ((rc = span_grow(comp, n, sp, u + 36)) != BCIO_OK) return rc;
        if (sp.buf.size() <= u) {
            *voff = 0;  // no records
            return BCIO_OK;
        }
        if (sp.buf.size() < u + 12) return fail(BCIO_E_FORMAT, "truncated BAM record");
        if (past(rd32s(sp.buf.data() + u + 4), rd32s(sp.buf.data() + u + 8))) {
            *voff = first;
            return BCIO_OK;
        }
    }
    constexpr uint64_t kProbe = 4u << 20;
    while (hi > (lo >> 16) + 4 * 65536) {
        const uint64_t mid = (lo >> 16) + (hi - (lo >> 16)) / 2;
        const int64_t c = sync_block(comp, n, mid);
        if (c < 0 || (uint64_t)c >= hi) {
            hi = mid;
            continue;
        }
        Span sp;
        sp.next = (uint64_t)c;
        int64_t o = -1;
        for (uint64_t want = 1; o < 0 && want <= kProbe; want *= 4) {  // one block, more if a record is longer
            if ((rc = span_grow(comp, n, sp, want)) != BCIO_OK) return rc;
            o = sync_records(sp, sp.buf.size(), n_ref);
            if (sp.eof) break;
        }
        if (o < 0) {  // no record start found (a record longer than the probe): look lower
            hi = mid;
            continue;
        }
        if (!past(rd32s(sp.buf.data() + o + 4), rd32s(sp.buf.data() + o + 8))) lo = std::max(lo, span_voff(sp, (uint64_t)o));
        else hi = (uint64_t)c;
    }
    // hop records from lo to the first with refID >= tid or -1 (or the end of the file)
    Span sp;
    sp.next = lo >> 16;
    uint64_t u = lo & 0xFFFF;
    for (;;) {
        if ((rc = span_grow(comp, n, sp, u + 36)) != BCIO_OK) return rc;
        if (u >= sp.buf.size()) {
            *voff = 0;  // no such record: the range runs to the end of the file
            return BCIO_OK;
        }
        if (u + 12 > sp.buf.size()) return fail(BCIO_E_FORMAT, "truncated BAM record");
        if (past(rd32s(sp.buf.data() + u + 4), rd32s(sp.buf.data() + u + 8))) {
            *voff = span_voff(sp, u);
            return BCIO_OK;
        }
        const uint32_t bs = rd32(sp.buf.data() + u);
        if (bs < 32) return fail(BCIO_E_FORMAT, "truncated BAM record");
        u += 4ull + bs;
        // keep the span bounded: drop whole blocks before u
        if (u > (4u << 20) && sp.ustart.size() > 1) {
            size_t j = (size_t)(std::upper_bound(sp.ustart.begin(), sp.ustart.end(), u) - sp.ustart.begin()) - 1;
            const uint64_t cut = sp.ustart[j];
            sp.buf.erase(sp.buf.begin(), sp.buf.begin() + (int64_t)cut);
            sp.boff.erase(sp.boff.begin(), sp.boff.begin() + (int64_t)j);
            sp.ustart.erase(sp.ustart.begin(), sp.ustart.begin() + (int64_t)j);
            for (auto& x : sp.ustart) x -= cut;
            u -= cut;
        }
    }
}

extern "C" int bcio_find_ref_start(const char* path, int32_t tid, uint64_t* voff) {
    return bcio_find_record(path, tid, INT32_MIN, voff);
}

extern "C" int bcio_stream_open_range(const char* path, int nthreads, uint64_t voff_begin, uint64_t voff_end,
                                      bcio_stream** out) {
    int rc = bcio_stream_open(path, nthreads, out);
    if (rc != BCIO_OK) return rc;
    bcio_stream* s = *out;
    // the records of [voff_begin, voff_end): restart the block scan at voff_begin's block
    s->pend.reset();
    s->pend_n = s->pbeg = 0;
    hop_reset(s->hop);
    s->coff = voff_begin >> 16;
    if (voff_end) {
        s->tail_block = voff_end >> 16;
        s->tail_keep = voff_end & 0xFFFF;
        s->cend = s->tail_keep ? s->tail_block + 1 : s->tail_block;
        if (!s->tail_keep) s->tail_block = UINT64_MAX;
    }
    const uint64_t skip = voff_begin & 0xFFFF;
    if (voff_end && voff_end <= voff_begin) {  // an empty range
        s->coff = s->cend;
        return BCIO_OK;
    }
    if ((rc = stream_fill(s, skip + 1)) != BCIO_OK || s->avail() < skip) {
        bcio_stream_close(s);
        *out = nullptr;
        return rc != BCIO_OK ? rc : fail(BCIO_E_ARG, "range start past its block");
    }
    s->pbeg = skip;
    return BCIO_OK;
}

// ------------------------------------------------------------------------------------------
// writer
namespace {

// htslib reg2bin (SAM spec §5.3), end exclusive
int reg2bin(int64_t beg, int64_t end) {
    --end;
    if (beg >> 14 == end >> 14) return (int)(((1 << 15) - 1) / 7 + (beg >> 14));
    if (beg >> 17 == end >> 17) return (int)(((1 << 12) - 1) / 7 + (beg >> 17));
    if (beg >> 20 == end >> 20) return (int)(((1 << 9) - 1) / 7 + (beg >> 20));
    if (beg >> 23 == end >> 23) return (int)(((1 << 6) - 1) / 7 + (beg >> 23));
    if (beg >> 26 == end >> 26) return (int)(((1 << 3) - 1) / 7 + (beg >> 26));
    return 0;
}

const uint8_t kEOF[28] = {31, 139, 8, 4, 0, 0, 0, 0, 0, 255, 6, 0, 66, 67, 2, 0, 27, 0, 3, 0, 0, 0, 0, 0, 0, 0, 0, 0};

}  // namespace

extern "C" int bcio_write_bam(const char* path, const bcio_write_spec* s) {
    if (!path || !s) return fail(BCIO_E_ARG, "null argument");
    // serialize uncompressed stream
    std::string u;
    u.append("BAM\1", 4);
    std::string text = "@HD\tVN:1.6\tSO:unknown\n";
    for (int32_t i = 0; i < s->n_refs; ++i)
        text += std::string("@SQ\tSN:") + s->ref_names[i] + "\tLN:" + std::to_string(s->ref_lens[i]) + "\n";
    wr32(u, (uint32_t)text.size());
    u += text;
    wr32(u, (uint32_t)s->n_refs);
    for (int32_t i = 0; i < s->n_refs; ++i) {
        std::string nm = s->ref_names[i];
        wr32(u, (uint32_t)(nm.size() + 1));
        u += nm;
        u.push_back('\0');
        wr32(u, (uint32_t)s->ref_lens[i]);
    }
    for (int64_t i = 0; i < s->n; ++i) {
        char name[32];
        int ln = std::snprintf(name, sizeof name, "r%lld", (long long)i) + 1;
        uint32_t nc = (uint32_t)(s->cig_off[i + 1] - s->cig_off[i]);
        int32_t ls = s->l_seq[i];
        uint64_t sb = (((uint64_t)ls + 1) / 2);
        uint32_t bs = (uint32_t)(32 + ln + 4 * nc + sb + (uint64_t)ls);
        const uint32_t* cg = s->cigar + s->cig_off[i];
        int64_t span = 0;
        for (uint32_t k = 0; k < nc; ++k) {
            uint32_t op = cg[k] & 0xf;
            if (op == 0 || op == 2 || op == 3 || op == 7 || op == 8) span += cg[k] >> 4;
        }
        int64_t beg = s->pos[i] < 0 ? 0 : s->pos[i];
        int bin = reg2bin(beg, beg + (span > 0 ? span : 1));
        wr32(u, bs);
        wr32(u, (uint32_t)s->tid[i]);
        wr32(u, (uint32_t)s->pos[i]);
        u.push_back((char)ln);
        u.push_back((char)s->mapq[i]);
        wr16(u, (uint16_t)bin);
        wr16(u, (uint16_t)nc);
        wr16(u, s->flag[i]);
        wr32(u, (uint32_t)ls);
        wr32(u, 0xFFFFFFFFu);
        wr32(u, 0xFFFFFFFFu);
        wr32(u, 0);
        u.append(name, (size_t)ln);
        for (uint32_t k = 0; k < nc; ++k) wr32(u, cg[k]);
        u.append((const char*)(s->seq + s->seq_off[i]), sb);
        if (s->qual_off[i + 1] - s->qual_off[i] == (uint64_t)ls)
            u.append((const char*)(s->qual + s->qual_off[i]), (size_t)ls);
        else
            u.append((size_t)ls, (char)0xFF);
    }
    // BGZF compress in 64 KiB - 256 B input blocks, in parallel
    const size_t kIn = 65280;
    const size_t nb = (u.size() + kIn - 1) / kIn;
    std::vector<std::string> outb(nb);
    std::atomic<int> zerr{0};
    parallel_for((int64_t)nb, hw_threads(s->nthreads), [&](int64_t b0, int64_t b1) {
        for (int64_t b = b0; b < b1; ++b) {
            const uint8_t* src = (const uint8_t*)u.data() + b * kIn;
            size_t len = std::min(kIn, u.size() - b * kIn);
            z_stream zs;
            std::memset(&zs, 0, sizeof zs);
            if (deflateInit2(&zs, s->level, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK) {
                zerr = 1;
                return;
            }
            std::vector<uint8_t> cbuf(deflateBound(&zs, (uLong)len) + 64);
            zs.next_in = (Bytef*)src;
            zs.avail_in = (uInt)len;
            zs.next_out = cbuf.data();
            zs.avail_out = (uInt)cbuf.size();
            if (deflate(&zs, Z_FINISH) != Z_STREAM_END) zerr = 1;
            size_t clen = zs.total_out;
            deflateEnd(&zs);
            if (clen + 26 > 65536) {  // incompressible: store
                clen = 0;
                zerr = 2;
            }
            uint32_t crc = (uint32_t)crc32(0L, src, (uInt)len);
            std::string& o = outb[b];
            const uint8_t hdr[18] = {31, 139, 8, 4, 0, 0, 0, 0, 0, 255, 6, 0, 66, 67, 2, 0, 0, 0};
            o.assign((const char*)hdr, 18);
            uint16_t bsize = (uint16_t)(clen + 25);
            o[16] = (char)(bsize & 0xff);
            o[17] = (char)(bsize >> 8);
            o.append((const char*)cbuf.data(), clen);
            wr32(o, crc);
            wr32(o, (uint32_t)len);
        }
    });
    if (zerr) return fail(BCIO_E_ZLIB, "deflate failed (block does not fit BGZF)");
    FILE* fp = std::fopen(path, "wb");
    if (!fp) return fail(BCIO_E_IO, std::string("cannot create ") + path);
    for (auto& o : outb) std::fwrite(o.data(), 1, o.size(), fp);
    std::fwrite(kEOF, 1, sizeof kEOF, fp);
    if (std::fclose(fp) != 0) return fail(BCIO_E_IO, "write failed");
    return BCIO_OK;
}

// ------------------------------------------------------------------------------------------
// formatter: str(round(x, dp)) exactly as CPython 3.10 (Objects/floatobject.c double_round +
// Python/pystrtod.c format_float_short 'r').  round(): correctly rounded decimal with dp digits
// (half-even on the exact binary value) parsed back to the nearest double; glibc printf and
// strtod are both exact, so printf("%.*f") + strtod is the same map.  repr(): shortest digits
// that round-trip (std::to_chars), fixed notation for 1e-4 <= |y| < 1e16, else d.ddde+XX.
namespace {

int py_repr(double y, char* out) {
    char buf[64];
    auto r = std::to_chars(buf, buf + sizeof buf, y, std::chars_format::scientific);
    *r.ptr = 0;
    // parse [-]d[.ddd]e[+-]xx
    const char* s = buf;
    char* o = out;
    if (*s == '-') {
        *o++ = '-';
        ++s;
    }
    char digits[40];
    int nd = 0;
    while (*s && *s != 'e') {
        if (*s != '.') digits[nd++] = *s;
        ++s;
    }
    int e10 = 0;
    if (*s == 'e') e10 = std::atoi(s + 1);
    // strip trailing zeros (to_chars shortest never emits them except for "0")
    while (nd > 1 && digits[nd - 1] == '0') --nd;
    int decpt = e10 + 1;
    if (nd == 1 && digits[0] == '0') decpt = 1;  // zero
    if (decpt <= -4 || decpt > 16) {
        *o++ = digits[0];
        if (nd > 1) {
            *o++ = '.';
            for (int i = 1; i < nd; ++i) *o++ = digits[i];
        }
        o += std::sprintf(o, "e%+.02d", decpt - 1);
    } else if (decpt <= 0) {
        *o++ = '0';
        *o++ = '.';
        for (int i = 0; i < -decpt; ++i) *o++ = '0';
        for (int i = 0; i < nd; ++i) *o++ = digits[i];
    } else if (decpt >= nd) {
        for (int i = 0; i < nd; ++i) *o++ = digits[i];
        for (int i = nd; i < decpt; ++i) *o++ = '0';
        *o++ = '.';
        *o++ = '0';
    } else {
        for (int i = 0; i < decpt; ++i) *o++ = digits[i];
        *o++ = '.';
        for (int i = decpt; i < nd; ++i) *o++ = digits[i];
    }
    *o = 0;
    return (int)(o - out);
}

// Fast path for dp <= 4: x * 10^dp is exact in x87 long double (53 + at most 10 significant bits
// of 5^dp <= 64), rintl rounds that exact value half-even like printf does, and for |n| < 2^53 the
// quotient n / 10^dp is the double nearest the decimal n·10^-dp, which is what strtod returns.
inline bool round_fast(double x, int dp, double* y) {
    static const long double kP10[5] = {1.0L, 10.0L, 100.0L, 1000.0L, 10000.0L};
    if (dp > 4 || !std::isfinite(x)) return false;
    long double prod = (long double)x * kP10[dp];
    if (!(std::fabs(prod) < 9007199254740992.0L)) return false;
    long double n = rintl(prod);
    *y = (double)n / (double)kP10[dp];
    return true;
}

inline int py_round_float(double x, int dp, char* out) {
    double y = x;
    if (round_fast(x, dp, &y)) return py_repr(y, out);
    if (std::isfinite(x) && dp <= 323) {
        char b[400];
        std::snprintf(b, sizeof b, "%.*f", dp, x);
        y = std::strtod(b, nullptr);
    }
    return py_repr(y, out);
}

inline int py_int(int64_t v, char* out) {
    auto r = std::to_chars(out, out + 24, v);
    *r.ptr = 0;
    return (int)(r.ptr - out);
}

inline char* put_int(char* w, int64_t v) { return std::to_chars(w, w + 24, v).ptr; }

inline char* put_str(char* w, const char* s, size_t n) {
    std::memcpy(w, s, n);
    return w + n;
}

// str(round(x, dp)) written at w.  With dp <= 4 and |n| < 10^15 (n = x·10^dp rounded, see
// round_fast) the decimal n·10^-dp has <= 15 significant digits, so it is the only decimal of
// that length mapping to the rounded double and repr() prints exactly it (trailing zeros
// stripped, ".0" if integral; fixed notation since 1e-4 <= |y| < 1e16 or y == 0).
inline char* put_round(char* w, double x, int dp) {
    static const long double kP10[5] = {1.0L, 10.0L, 100.0L, 1000.0L, 10000.0L};
    static const int64_t kI10[5] = {1, 10, 100, 1000, 10000};
    if (dp <= 4 && std::isfinite(x)) {
        long double r = rintl((long double)x * kP10[dp]);
        if (std::fabs(r) < 1e15L) {
            if (std::signbit(r)) *w++ = '-';
            int64_t n = (int64_t)std::fabs(r);
            w = put_int(w, n / kI10[dp]);
            *w++ = '.';
            int64_t fr = n % kI10[dp];
            if (fr == 0) {
                *w++ = '0';
                return w;
            }
            int nd = dp;
            while (fr % 10 == 0) {
                fr /= 10;
                --nd;
            }
            for (int i = nd - 1; i >= 0; --i) {
                w[i] = (char)('0' + fr % 10);
                fr /= 10;
            }
            return w + nd;
        }
    }
    return w + py_round_float(x, dp, w);
}

}  // namespace

struct bcio_fmt {
    std::string buf;
    bool taken = false;
};

extern "C" int bcio_fmt_new(bcio_fmt** out) {
    if (!out) return fail(BCIO_E_ARG, "null");
    *out = new bcio_fmt();
    return BCIO_OK;
}
extern "C" void bcio_fmt_free(bcio_fmt* b) { delete b; }
extern "C" int bcio_fmt_take(bcio_fmt* b, const char** data, int64_t* size) {
    if (!b) return fail(BCIO_E_ARG, "null");
    *data = b->buf.data();
    *size = (int64_t)b->buf.size();
    b->taken = true;
    return BCIO_OK;
}
extern "C" int bcio_fmt_pyround_float(double x, int dp, char* out, int cap) {
    if (cap < 400 || dp < 0 || dp > 323) return fail(BCIO_E_ARG, "bad dp/cap");
    return py_round_float(x, dp, out);
}
extern "C" int bcio_fmt_pyround_int(int64_t v, int dp, char* out, int cap) {
    if (cap < 24 || dp < 0) return fail(BCIO_E_ARG, "bad dp/cap");
    return py_int(v, out);
}

extern "C" int bcio_fmt_rows(bcio_fmt* b, const char* ref, int64_t L, int k, const int32_t* counts,
                             const double* pc, const double* ent, const double* sec, int dp,
                             int long_format, int nthreads) {
    if (!b || !ref || (k != 5 && k != 6) || dp < 0 || dp > 323 || L < 0)
        return fail(BCIO_E_ARG, "bad formatter arguments");
    if (b->taken) {
        b->buf.clear();
        b->taken = false;
    }
    static const char* kBase[6] = {"A", "C", "G", "T", "DS", "N"};
    const std::string refs(ref);
    const size_t rl = refs.size();
    nthreads = hw_threads(nthreads);
    const int64_t per = std::max<int64_t>(256, std::min<int64_t>(1 << 14, L / (8 * nthreads) + 1));
    const int64_t nchunks = (L + per - 1) / per;
    // worst case per position: k rows of ref + 4 ints + 3 floats (repr <= 25 chars) + separators
    const size_t row_max = (size_t)k * (rl + 4 * 24 + 3 * 32 + 16);
    std::vector<uvec<char>> parts((size_t)nchunks);
    parallel_for(nchunks, nthreads, [&](int64_t c0, int64_t c1) {
        for (int64_t c = c0; c < c1; ++c) {
            uvec<char>& s = parts[(size_t)c];
            const int64_t p0 = c * per, p1 = std::min(L, p0 + per);
            s.resize((size_t)(p1 - p0) * row_max);
            char* w = s.data();
            for (int64_t p = p0; p < p1; ++p) {
                int64_t cov = 0;
                int nz = 0;
                for (int j = 0; j < k; ++j) {
                    cov += counts[(int64_t)j * L + p];
                    nz += counts[(int64_t)j * L + p] != 0;
                }
                // entropy / secondary text, shared by all k long rows
                char et[64], st[64];
                size_t etn = 1, stn = 1;
                et[0] = st[0] = '1';
                if (cov != 0) {
                    etn = (size_t)(put_round(et, ent[p], dp) - et);
                    if (nz > 1) stn = (size_t)(put_round(st, sec[p], dp) - st);
                }
                char head[64];
                char* h = head;
                *h++ = '\t';
                h = put_int(h, p + 1);
                *h++ = '\t';
                h = put_int(h, cov);
                const size_t hn = (size_t)(h - head);
                if (!long_format) {
                    w = put_str(w, refs.data(), rl);
                    w = put_str(w, head, hn);
                    for (int j = 0; j < k; ++j) {
                        *w++ = '\t';
                        w = put_int(w, counts[(int64_t)j * L + p]);
                    }
                    for (int j = 0; j < k; ++j) {
                        *w++ = '\t';
                        if (cov == 0)
                            w = put_str(w, "-1", 2);
                        else
                            w = put_round(w, pc[(int64_t)j * L + p], dp);
                    }
                    *w++ = '\t';
                    w = put_str(w, et, etn);
                    *w++ = '\t';
                    w = put_str(w, st, stn);
                    *w++ = '\n';
                } else {
                    for (int j = 0; j < k; ++j) {
                        w = put_str(w, refs.data(), rl);
                        w = put_str(w, head, hn);
                        *w++ = '\t';
                        w = put_str(w, kBase[j], j == 4 ? 2 : 1);
                        *w++ = '\t';
                        w = put_int(w, counts[(int64_t)j * L + p]);
                        *w++ = '\t';
                        if (cov == 0)
                            w = put_str(w, "-1", 2);
                        else
                            w = put_round(w, pc[(int64_t)j * L + p], dp);
                        *w++ = '\t';
                        w = put_str(w, et, etn);
                        *w++ = '\t';
                        w = put_str(w, st, stn);
                        *w++ = '\n';
                    }
                }
            }
            s.resize((size_t)(w - s.data()));
        }
    });
    size_t tot = b->buf.size();
    for (auto& s : parts) tot += s.size();
    b->buf.reserve(tot);
    for (auto& s : parts) b->buf.append(s.data(), s.size());
    return BCIO_OK;
}

extern "C" int bcio_seq_to_event(const uint8_t* bam, int64_t nbytes, uint8_t* out, int64_t out_bytes, int nthreads) {
    if (nbytes < 0 || (nbytes > 0 && (!bam || !out))) return fail(BCIO_E_ARG, "null argument");
    if ((uint64_t)out_bytes < seq_event_bytes((uint64_t)nbytes))
        return fail(BCIO_E_ARG, "out_bytes smaller than the padded event layout");
    const int64_t chunk = 1 << 20;
    parallel_for((nbytes + chunk - 1) / chunk, hw_threads(nthreads), [&](int64_t c0, int64_t c1) {
        const int64_t a = c0 * chunk, b = std::min(nbytes, c1 * chunk);
        seq_to_event(bam + a, (uint64_t)(b - a), out + a);
    });
    std::memset(out + nbytes, 0, (size_t)(out_bytes - nbytes));
    return BCIO_OK;
}
