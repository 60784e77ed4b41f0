// bc_comm.hip — multi-GPU exchange of the C-ABI (include/basecount_hip.h, "Multi-GPU"): one
// process per GPU, RCCL over xGMI, every collective on the context's stream.
//
// The pileup itself needs no communication: references are independent, so each
// rank owns whole references and runs the single-GPU path on them.  What travels is small:
//   * the per-reference results the reference prints (main.py:469-595: summary numbers and
//     amplicon vectors), gathered to rank 0 — bc_gather_bytes (host payloads, the CLI) and
//     bc_gather_dev (payloads already in HBM, the bench's timed step);
//   * control data: the reference order chosen by rank 0 (main.py:92's set order is per process,
//     so one rank decides: bc_broadcast_bytes), the first out-of-range read of every reference
//     (bc_allgather_i64: every rank must raise the reference's first error), a barrier.
// Ragged sizes are exchanged first (bc_allgather_i64) and laid out by bc_gather_layout, the one
// piece that is pure host arithmetic (tested on the CPU).  The gather is a grouped set of
// point-to-point receives at the root, which is what xGMI's point-to-point links carry best: no
// ring, no padding of every payload to the largest.
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "bc_internal.h"

struct bc_comm {
    bc_ctx* ctx = nullptr;
    ncclComm_t nc = nullptr;
    int rank = 0, world = 1;
    void* dbuf = nullptr;  // device staging for host-buffer collectives (grows)
    size_t dbuf_bytes = 0;
};

// the C-ABI's thread-local message (bc_capi.hip) is what bc_last_error() returns
namespace bc {
int set_error(int code, const std::string& m);
}

namespace {

int cfail(int code, const std::string& m) { return bc::set_error(code, m); }

int nccl_fail(ncclResult_t r, const char* where) {
    return cfail(BC_E_COMM, std::string(where) + ": " + ncclGetErrorString(r));
}

#define NCCL_TRY(expr)                                        \
    do {                                                      \
        ncclResult_t _r = (expr);                             \
        if (_r != ncclSuccess) return nccl_fail(_r, #expr);   \
    } while (0)

#define HIPC_TRY(expr)                                                                          \
    do {                                                                                        \
        hipError_t _e = (expr);                                                                 \
        if (_e != hipSuccess) return cfail(BC_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
    } while (0)

struct Dev {
    int prev = -1;
    explicit Dev(int d) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != d) (void)hipSetDevice(d);
    }
    ~Dev() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

int staging(bc_comm* c, size_t bytes) {
    if (bytes <= c->dbuf_bytes) return BC_OK;
    if (c->dbuf) {
        HIPC_TRY(hipStreamSynchronize(c->ctx->stream));
        HIPC_TRY(hipFree(c->dbuf));
        c->dbuf = nullptr;
        c->dbuf_bytes = 0;
    }
    const size_t sz = std::max<size_t>(bytes, 4096);
    HIPC_TRY(hipMalloc(&c->dbuf, sz));
    c->dbuf_bytes = sz;
    return BC_OK;
}

}  // namespace

extern "C" {

int bc_gather_layout(const int64_t* sizes, int world, int64_t* offsets) {
    if (!sizes || !offsets || world <= 0) return cfail(BC_E_ARG, "bc_gather_layout: bad argument");
    int64_t off = 0;
    for (int r = 0; r < world; ++r) {
        if (sizes[r] < 0) return cfail(BC_E_ARG, "bc_gather_layout: negative size from rank " + std::to_string(r));
        offsets[r] = off;
        if (sizes[r] > INT64_MAX - off) return cfail(BC_E_ARG, "bc_gather_layout: total overflows");
        off += sizes[r];
    }
    offsets[world] = off;
    return BC_OK;
}

int bc_comm_unique_id(uint8_t* id) {
    if (!id) return cfail(BC_E_ARG, "id is NULL");
    ncclUniqueId u;
    NCCL_TRY(ncclGetUniqueId(&u));
    static_assert(sizeof(u) == BC_COMM_ID_BYTES, "RCCL unique id size");
    std::memcpy(id, &u, sizeof u);
    return BC_OK;
}

int bc_comm_init(bc_ctx* ctx, const uint8_t* id, int rank, int world, bc_comm** out) {
    if (!ctx || !id || !out) return cfail(BC_E_ARG, "NULL argument");
    if (world < 1 || rank < 0 || rank >= world) return cfail(BC_E_ARG, "rank / world out of range");
    *out = nullptr;
    Dev g(ctx->device);
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof u);
    auto* c = new bc_comm();
    c->ctx = ctx;
    c->rank = rank;
    c->world = world;
    ncclResult_t r = ncclCommInitRank(&c->nc, world, u, rank);
    if (r != ncclSuccess) {
        delete c;
        return nccl_fail(r, "ncclCommInitRank");
    }
    *out = c;
    return BC_OK;
}

int bc_comm_destroy(bc_comm* c) {
    if (!c) return BC_OK;
    Dev g(c->ctx->device);
    (void)hipStreamSynchronize(c->ctx->stream);
    if (c->nc) (void)ncclCommDestroy(c->nc);
    if (c->dbuf) (void)hipFree(c->dbuf);
    delete c;
    return BC_OK;
}

int bc_comm_rank(const bc_comm* c, int* rank, int* world) {
    if (!c || !rank || !world) return cfail(BC_E_ARG, "NULL argument");
    *rank = c->rank;
    *world = c->world;
    return BC_OK;
}

int bc_comm_barrier(bc_comm* c) {
    if (!c) return cfail(BC_E_ARG, "comm is NULL");
    Dev g(c->ctx->device);
    if (int rc = staging(c, 8)) return rc;
    NCCL_TRY(ncclAllReduce(c->dbuf, c->dbuf, 1, ncclInt32, ncclSum, c->nc, c->ctx->stream));
    HIPC_TRY(hipStreamSynchronize(c->ctx->stream));
    return BC_OK;
}

int bc_allgather_i64(bc_comm* c, const int64_t* h_send, int64_t n, int64_t* h_recv) {
    if (!c || n < 0 || (n > 0 && (!h_send || !h_recv))) return cfail(BC_E_ARG, "bad argument");
    if (n == 0) return BC_OK;
    Dev g(c->ctx->device);
    const size_t one = (size_t)n * 8;
    if (int rc = staging(c, one * (size_t)(c->world + 1))) return rc;
    uint8_t* send = (uint8_t*)c->dbuf;
    uint8_t* recv = send + one;
    HIPC_TRY(hipMemcpyAsync(send, h_send, one, hipMemcpyHostToDevice, c->ctx->stream));
    NCCL_TRY(ncclAllGather(send, recv, (size_t)n, ncclInt64, c->nc, c->ctx->stream));
    HIPC_TRY(hipMemcpyAsync(h_recv, recv, one * (size_t)c->world, hipMemcpyDeviceToHost, c->ctx->stream));
    HIPC_TRY(hipStreamSynchronize(c->ctx->stream));
    return BC_OK;
}

int bc_broadcast_bytes(bc_comm* c, void* h_buf, int64_t n, int root) {
    if (!c || n < 0 || (n > 0 && !h_buf) || root < 0 || root >= c->world) return cfail(BC_E_ARG, "bad argument");
    if (n == 0) return BC_OK;
    Dev g(c->ctx->device);
    if (int rc = staging(c, (size_t)n)) return rc;
    if (c->rank == root) HIPC_TRY(hipMemcpyAsync(c->dbuf, h_buf, (size_t)n, hipMemcpyHostToDevice, c->ctx->stream));
    NCCL_TRY(ncclBroadcast(c->dbuf, c->dbuf, (size_t)n, ncclUint8, root, c->nc, c->ctx->stream));
    if (c->rank != root) HIPC_TRY(hipMemcpyAsync(h_buf, c->dbuf, (size_t)n, hipMemcpyDeviceToHost, c->ctx->stream));
    HIPC_TRY(hipStreamSynchronize(c->ctx->stream));
    return BC_OK;
}

int bc_gather_dev(bc_comm* c, const void* d_send, int64_t n, void* d_recv, const int64_t* sizes, int root) {
    if (!c || !sizes || n < 0 || root < 0 || root >= c->world) return cfail(BC_E_ARG, "bad argument");
    if (sizes[c->rank] != n) return cfail(BC_E_ARG, "bc_gather_dev: sizes[rank] differs from n");
    if (n > 0 && !d_send) return cfail(BC_E_ARG, "d_send is NULL");
    std::vector<int64_t> off((size_t)c->world + 1);
    if (int rc = bc_gather_layout(sizes, c->world, off.data())) return rc;
    if (c->rank == root && off[c->world] > 0 && !d_recv) return cfail(BC_E_ARG, "d_recv is NULL on the root");
    Dev g(c->ctx->device);
    hipStream_t s = c->ctx->stream;
    if (c->rank == root && n > 0)
        HIPC_TRY(hipMemcpyAsync((uint8_t*)d_recv + off[root], d_send, (size_t)n, hipMemcpyDeviceToDevice, s));
    NCCL_TRY(ncclGroupStart());
    if (c->rank == root) {
        for (int r = 0; r < c->world; ++r)
            if (r != root && sizes[r] > 0) {
                ncclResult_t e = ncclRecv((uint8_t*)d_recv + off[r], (size_t)sizes[r], ncclUint8, r, c->nc, s);
                if (e != ncclSuccess) {
                    (void)ncclGroupEnd();
                    return nccl_fail(e, "ncclRecv");
                }
            }
    } else if (n > 0) {
        ncclResult_t e = ncclSend(d_send, (size_t)n, ncclUint8, root, c->nc, s);
        if (e != ncclSuccess) {
            (void)ncclGroupEnd();
            return nccl_fail(e, "ncclSend");
        }
    }
    NCCL_TRY(ncclGroupEnd());
    return BC_OK;
}

int bc_reduce_i32_dev(bc_comm* c, const int32_t* d_send, int32_t* d_recv, int64_t n, int root) {
    if (!c || n < 0 || root < 0 || root >= c->world) return cfail(BC_E_ARG, "bad argument");
    if (n > 0 && !d_send) return cfail(BC_E_ARG, "d_send is NULL");
    if (c->rank == root && n > 0 && !d_recv) return cfail(BC_E_ARG, "d_recv is NULL on the root");
    if (n == 0) return BC_OK;
    Dev g(c->ctx->device);
    // (the receive buffer is only written on the root; elsewhere RCCL takes the send buffer)
    NCCL_TRY(ncclReduce(d_send, c->rank == root ? (void*)d_recv : (void*)d_send, (size_t)n, ncclInt32, ncclSum,
                        root, c->nc, c->ctx->stream));
    return BC_OK;
}

int bc_gather_bytes(bc_comm* c, const void* h_send, int64_t n, void* h_recv, const int64_t* sizes, int root) {
    if (!c || !sizes || n < 0 || (n > 0 && !h_send) || root < 0 || root >= c->world)
        return cfail(BC_E_ARG, "bad argument");
    std::vector<int64_t> off((size_t)c->world + 1);
    if (int rc = bc_gather_layout(sizes, c->world, off.data())) return rc;
    const int64_t total = off[c->world];
    if (c->rank == root && total > 0 && !h_recv) return cfail(BC_E_ARG, "h_recv is NULL on the root");
    Dev g(c->ctx->device);
    // staging: [own payload | the root's receive area]
    const size_t own = ((size_t)n + 255) / 256 * 256;
    if (int rc = staging(c, own + (c->rank == root ? (size_t)total : 0) + 16)) return rc;
    uint8_t* send = (uint8_t*)c->dbuf;
    uint8_t* recv = send + own;
    if (n > 0) HIPC_TRY(hipMemcpyAsync(send, h_send, (size_t)n, hipMemcpyHostToDevice, c->ctx->stream));
    if (int rc = bc_gather_dev(c, send, n, recv, sizes, root)) return rc;
    if (c->rank == root && total > 0)
        HIPC_TRY(hipMemcpyAsync(h_recv, recv, (size_t)total, hipMemcpyDeviceToHost, c->ctx->stream));
    HIPC_TRY(hipStreamSynchronize(c->ctx->stream));
    return BC_OK;
}

}  // extern "C"
