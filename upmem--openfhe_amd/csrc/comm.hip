// comm.hip -- multi-GPU evaluation-key broadcast over RCCL (xGMI).
//
// the only collective of the path is a broadcast of the
// key-switching keys from a root GPU, once per key, before any ciphertext is
// switched; the polynomial work itself is sharded by ciphertext batch with no
// exchange.  The reference has no multi-device path (its PimManager drives
// one DPU set per process, PimManager.h:21-127); this is the MI355X
// equivalent of loading the key into every device's memory.
//
// One communicator per (process, device): ranks exchange the 128-byte
// unique id out of band (the caller's launcher: torch.distributed, MPI, a
// file), then each calls ofhe_hip_comm_init.  ncclBroadcast runs in place on
// the caller's stream, so a broadcast orders with the caller's kernels like
// every other entry point; nothing here synchronises.
#include <rccl/rccl.h>

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <thread>

#include "internal.hpp"

static_assert(OFHE_COMM_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "unique id size");

struct ofhe_comm_s {
    ofhe_ctx_t ctx = nullptr;
    ncclComm_t comm = nullptr;
    int nranks = 0, rank = 0;
};

namespace {
int rccl_fail(const char* what, ncclResult_t r) {
    return ofhe::fail(OFHE_ERR_HIP, std::string(what) + ": " + ncclGetErrorString(r));
}

// The communicator is created non-blocking and polled against a deadline
// (OFHE_COMM_INIT_TIMEOUT_S, default 120 s): a peer that never arrives makes
// ofhe_hip_comm_init fail with an error instead of hanging the job, and the
// caller falls back (shard.key_broadcaster agrees on the fallback across ranks).
double init_timeout_s() {
    const char* e = getenv("OFHE_COMM_INIT_TIMEOUT_S");
    const double v = e ? atof(e) : 120.0;
    return v > 0 ? v : 120.0;
}
// wait for a non-blocking communicator's pending call; ncclInProgress -> done or error
ncclResult_t settle(ncclComm_t c, double timeout_s) {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        ncclResult_t st = ncclInProgress;
        const ncclResult_t r = ncclCommGetAsyncError(c, &st);
        if (r != ncclSuccess) return r;
        if (st != ncclInProgress) return st;
        const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (dt > timeout_s) return ncclInProgress;
        std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
}
}  // namespace

int ofhe_hip_comm_unique_id(void* id) {
    if (!id) return ofhe::fail(OFHE_ERR_ARG, "unique id buffer is NULL");
    ncclUniqueId u;
    const ncclResult_t r = ncclGetUniqueId(&u);
    if (r != ncclSuccess) return rccl_fail("ncclGetUniqueId", r);
    std::memcpy(id, u.internal, sizeof(u.internal));
    return OFHE_OK;
}

int ofhe_hip_comm_init(ofhe_ctx_t ctx, int nranks, int rank, const void* id, ofhe_comm_t* out) {
    if (!ctx || !id || !out) return ofhe::fail(OFHE_ERR_ARG, "NULL argument");
    if (!ctx->live.load()) return ofhe::fail(OFHE_ERR_STATE, "context was finalized");
    if (nranks < 1 || rank < 0 || rank >= nranks) return ofhe::fail(OFHE_ERR_ARG, "rank must be in [0, nranks)");
    HIPCHK(hipSetDevice(ctx->device));
    ncclUniqueId u;
    std::memcpy(u.internal, id, sizeof(u.internal));
    ncclComm_t c = nullptr;
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    ncclResult_t r = ncclCommInitRankConfig(&c, nranks, u, rank, &cfg);
    if (r == ncclInProgress) r = settle(c, init_timeout_s());
    if (r != ncclSuccess) {
        if (c) (void)ncclCommAbort(c);
        if (r == ncclInProgress) return ofhe::fail(OFHE_ERR_HIP, "ncclCommInitRankConfig: timed out waiting for the peer ranks");
        return rccl_fail("ncclCommInitRankConfig", r);
    }
    ofhe_comm_s* s = new (std::nothrow) ofhe_comm_s();
    if (!s) {
        (void)ncclCommDestroy(c);
        return ofhe::fail(OFHE_ERR_NOMEM, "communicator allocation failed");
    }
    s->ctx = ctx;
    s->comm = c;
    s->nranks = nranks;
    s->rank = rank;
    *out = s;
    return OFHE_OK;
}

int ofhe_hip_comm_destroy(ofhe_comm_t c) {
    if (!c) return ofhe::fail(OFHE_ERR_ARG, "communicator is NULL");
    (void)hipSetDevice(c->ctx->device);
    const ncclResult_t r = c->comm ? ncclCommDestroy(c->comm) : ncclSuccess;
    delete c;
    if (r != ncclSuccess) return rccl_fail("ncclCommDestroy", r);
    return OFHE_OK;
}

int ofhe_hip_bcast_evalkey(ofhe_comm_t c, uint64_t* key, size_t words, int root, void* stream) {
    if (!c || !c->comm) return ofhe::fail(OFHE_ERR_STATE, "communicator is NULL or destroyed");
    if (root < 0 || root >= c->nranks) return ofhe::fail(OFHE_ERR_ARG, "root must be in [0, nranks)");
    if (words == 0) return OFHE_OK;
    if (!key) return ofhe::fail(OFHE_ERR_ARG, "key is NULL");
    HIPCHK(hipSetDevice(c->ctx->device));
    // u64 words as ncclUint64: in place (sendbuff == recvbuff), the root's
    // buffer is read, every other rank's is overwritten
    ncclResult_t r = ncclBroadcast(key, key, words, ncclUint64, root, c->comm, ofhe::pick(stream));
    if (r == ncclInProgress) r = settle(c->comm, init_timeout_s());  // enqueue of a non-blocking comm
    if (r != ncclSuccess) return rccl_fail("ncclBroadcast", r);
    return OFHE_OK;
}
