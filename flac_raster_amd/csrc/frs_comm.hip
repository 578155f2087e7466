// frs_comm.hip -- RCCL over xGMI for the multi-GPU create-streaming.
//
// Tiles shard by contiguous tile rows with no data-path collective; the one exchange of the sharded path is an
// all-gather of per-tile byte sizes (a few KB) so every rank knows every tile's offset in the streaming file.
// librccl.so is loaded at run time (dlopen), so the codec library itself has no hard RCCL dependency; the
// ncclUniqueId of rank 0 reaches the other ranks through the host's bootstrap (flac_raster_amd/distributed.py).
#include <dlfcn.h>
#include <string.h>

#include <chrono>
#include <mutex>
#include <string>
#include <thread>

#include <rccl/rccl.h>

#include "frs_internal.h"

struct frs_comm {
    ncclComm_t comm = nullptr;
    int rank = 0, nranks = 1;
    frs_ctx *ctx = nullptr;
    DevBuf buf;  // send | recv staging of the all-gathers
    bool aborted = false;  // a collective failed or timed out and the communicator was aborted
};

namespace {
struct RcclApi {
    void *h = nullptr;
    ncclResult_t (*get_unique_id)(ncclUniqueId *) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*all_gather)(const void *, void *, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    const char *(*error_string)(ncclResult_t) = nullptr;
    ncclResult_t (*comm_abort)(ncclComm_t) = nullptr;  // required: the bounded wait of an all-gather needs it
    ncclResult_t (*get_async_error)(ncclComm_t, ncclResult_t *) = nullptr;  // optional
    std::string err;
};
RcclApi g_api;
std::once_flag g_once;

bool load_rccl() {
    std::call_once(g_once, [] {
        const char *names[] = {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"};
        for (const char *n : names)
            if ((g_api.h = dlopen(n, RTLD_NOW | RTLD_LOCAL))) break;
        if (!g_api.h) {
            g_api.err = std::string("cannot load librccl.so: ") + dlerror();
            return;
        }
        g_api.get_unique_id = (decltype(g_api.get_unique_id))dlsym(g_api.h, "ncclGetUniqueId");
        g_api.comm_init_rank = (decltype(g_api.comm_init_rank))dlsym(g_api.h, "ncclCommInitRank");
        g_api.comm_destroy = (decltype(g_api.comm_destroy))dlsym(g_api.h, "ncclCommDestroy");
        g_api.all_gather = (decltype(g_api.all_gather))dlsym(g_api.h, "ncclAllGather");
        g_api.error_string = (decltype(g_api.error_string))dlsym(g_api.h, "ncclGetErrorString");
        g_api.comm_abort = (decltype(g_api.comm_abort))dlsym(g_api.h, "ncclCommAbort");
        g_api.get_async_error = (decltype(g_api.get_async_error))dlsym(g_api.h, "ncclCommGetAsyncError");
        if (!g_api.get_unique_id || !g_api.comm_init_rank || !g_api.comm_destroy || !g_api.all_gather ||
            !g_api.comm_abort)
            g_api.err = "librccl.so lacks the nccl* entry points (incl. ncclCommAbort, which bounds a hung collective)";
    });
    return g_api.h && g_api.err.empty();
}

std::string nccl_msg(ncclResult_t r) {
    return g_api.error_string ? g_api.error_string(r) : ("ncclResult " + std::to_string((int)r));
}
}  // namespace

extern "C" {

int frs_comm_unique_id(uint8_t *id_out) {
    if (!id_out) return FRS_E_ARG;
    if (!load_rccl()) return FRS_E_UNSUPPORTED;
    ncclUniqueId id;
    if (g_api.get_unique_id(&id) != ncclSuccess) return FRS_E_HIP;
    memcpy(id_out, id.internal, NCCL_UNIQUE_ID_BYTES);
    return FRS_OK;
}

int frs_comm_init(frs_ctx *ctx, const uint8_t *id, int32_t nranks, int32_t rank, frs_comm **out) {
    if (!ctx || !id || !out || nranks < 1 || rank < 0 || rank >= nranks) return FRS_E_ARG;
    *out = nullptr;
    if (!load_rccl()) {
        ctx->err = g_api.err;
        return FRS_E_UNSUPPORTED;
    }
    FRS_HIP(hipSetDevice(ctx->device));
    ncclUniqueId uid;
    memcpy(uid.internal, id, NCCL_UNIQUE_ID_BYTES);
    frs_comm *c = new frs_comm();
    const ncclResult_t r = g_api.comm_init_rank(&c->comm, nranks, uid, rank);
    if (r != ncclSuccess) {
        ctx->err = "ncclCommInitRank: " + nccl_msg(r);
        delete c;
        return FRS_E_HIP;
    }
    c->rank = rank;
    c->nranks = nranks;
    c->ctx = ctx;
    *out = c;
    return FRS_OK;
}

void frs_comm_destroy(frs_comm *c) {
    if (!c) return;
    if (c->ctx && !c->aborted) {  // (after an abort the stream may hold work that never drains: no sync)
        hipSetDevice(c->ctx->device);
        hipStreamSynchronize(c->ctx->stream);
    }
    if (c->comm) g_api.comm_destroy(c->comm);
    c->buf.release();
    delete c;
}

int frs_comm_allgather_i64(frs_comm *c, const int64_t *send_host, int64_t count, int64_t *recv_host) {
    if (!c || count < 0 || (count && (!send_host || !recv_host))) return FRS_E_ARG;
    frs_ctx *ctx = c->ctx;
    if (c->aborted || !c->comm) {
        ctx->err = "communicator was aborted after a failed all-gather";
        return FRS_E_HIP;
    }
    if (count == 0) return FRS_OK;
    FRS_HIP(hipSetDevice(ctx->device));
    const size_t sb = sizeof(int64_t) * (size_t)count;
    FRS_HIP(c->buf.ensure(sb * (size_t)(c->nranks + 1)));
    int64_t *dsend = c->buf.as<int64_t>(), *drecv = dsend + count;
    FRS_HIP(hipMemcpyAsync(dsend, send_host, sb, hipMemcpyHostToDevice, ctx->stream));
    const ncclResult_t r = g_api.all_gather(dsend, drecv, (size_t)count, ncclInt64, c->comm, ctx->stream);
    if (r != ncclSuccess) {
        ctx->err = "ncclAllGather: " + nccl_msg(r);
        return FRS_E_HIP;
    }
    FRS_HIP(hipMemcpyAsync(recv_host, drecv, sb * (size_t)c->nranks, hipMemcpyDeviceToHost, ctx->stream));
    // bounded wait: a dead or hung peer would leave the collective pending for good.  Poll an event, check the
    // communicator's asynchronous error, and abort it after $FRS_COMM_TIMEOUT seconds (default 120).
    hipEvent_t done;
    FRS_HIP(hipEventCreateWithFlags(&done, hipEventDisableTiming));
    FRS_HIP(hipEventRecord(done, ctx->stream));
    double limit_s = 120.0;
    if (const char *e = getenv("FRS_COMM_TIMEOUT")) limit_s = atof(e);
    const auto t0 = std::chrono::steady_clock::now();
    int rc = FRS_OK;
    for (int spin = 0;; spin++) {
        const hipError_t q = hipEventQuery(done);
        if (q == hipSuccess) break;
        if (q != hipErrorNotReady) {
            ctx->err = std::string("all-gather: ") + hipGetErrorString(q);
            rc = FRS_E_HIP;
            break;
        }
        ncclResult_t ae = ncclSuccess;
        if (g_api.get_async_error && g_api.get_async_error(c->comm, &ae) == ncclSuccess && ae != ncclSuccess &&
            ae != ncclInProgress) {
            ctx->err = "ncclAllGather: " + nccl_msg(ae);
            rc = FRS_E_HIP;
            break;
        }
        const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (el > limit_s) {
            ctx->err = "ncclAllGather did not complete within FRS_COMM_TIMEOUT (a peer rank died or hung)";
            rc = FRS_E_HIP;
            break;
        }
        std::this_thread::sleep_for(std::chrono::microseconds(spin < 1000 ? 5 : 200));
    }
    hipEventDestroy(done);
    if (rc != FRS_OK && c->comm) {
        g_api.comm_abort(c->comm);  // frees the pending collective; the communicator is unusable afterwards
        c->comm = nullptr;
        c->aborted = true;
    }
    return rc;
}

}  // extern "C"
