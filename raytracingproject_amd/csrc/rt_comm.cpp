// rt_comm.cpp -- RCCL behind the C ABI (include/rt_hip.h, "RCCL"): the one exchange
// step of the multi-GPU frame, the gather of finished shard buffers to
// rank 0 over xGMI.  Rendering itself never communicates: tiles t -> rank t mod N.
//
// Two ways to get a communicator: one process per GPU (ncclCommInitRank with an id rank
// 0 made and shared out of band) or one process driving all GPUs (ncclCommInitAll,
// rccl.h:236).  The gather is ncclGather (rccl.h:745): rank r's W*H*3/N-ish shard lands at
// offset r of rank 0's buffer, which rt_unshard / rt_finish_frame_u8 then un-interleave.
#include <rccl/rccl.h>

#include <chrono>
#include <cstring>
#include <thread>
#include <vector>

#include "rt_ctx.h"

using namespace rtx_abi;

namespace {

#define NCCLCHK(ctx, expr)                                                                              \
    do {                                                                                                \
        ncclResult_t r_ = (expr);                                                                       \
        if (r_ != ncclSuccess) return fail(ctx, RT_ERR_COMM, "%s: %s", #expr, ncclGetErrorString(r_)); \
    } while (0)

ncclDataType_t dtype_of(const rt_ctx* c) { return c->precision == RT_PREC_F64 ? ncclFloat64 : ncclFloat32; }

// elements of one rank's shard buffer for a W x H frame over n ranks
size_t shard_elems(int W, int H, int n) {
    rt_shard_info si;
    if (rt_shard_layout(W, H, 0, n, &si) != RT_OK) return 0;
    return (size_t)si.max_shard_tiles * 64 * 3;
}

// A non-blocking communicator's pending operation (init, or an enqueue that returned
// ncclInProgress): poll its async state until it settles or `timeout_ms` passes.
ncclResult_t wait_comm(ncclComm_t comm, int timeout_ms) {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        ncclResult_t st = ncclSuccess;
        const ncclResult_t r = ncclCommGetAsyncError(comm, &st);
        if (r != ncclSuccess) return r;
        if (st != ncclInProgress) return st;
        if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(timeout_ms)) return ncclInProgress;
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
}

}  // namespace

void rt_comm_release(rt_ctx* c) {
    if (c && c->comm) {
        (void)ncclCommDestroy((ncclComm_t)c->comm);
        c->comm = nullptr;
        c->comm_rank = c->comm_size = 0;
        c->comm_nonblocking = false;
    }
}

extern "C" {

int rt_comm_unique_id(char id[RT_COMM_ID_BYTES]) {
    static_assert(sizeof(ncclUniqueId) == RT_COMM_ID_BYTES, "ncclUniqueId size");
    if (!id) return RT_ERR_INVALID;
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return RT_ERR_COMM;
    std::memcpy(id, &u, sizeof(u));
    return RT_OK;
}

int rt_comm_init_rank(rt_ctx* c, int nranks, int rank, const char id[RT_COMM_ID_BYTES]) {
    return rt_comm_init_rank_timeout(c, nranks, rank, id, RT_COMM_INIT_TIMEOUT_MS);
}

// Non-blocking ncclCommInitRankConfig polled against a deadline: a rank whose peers never
// join (one of them failed before reaching the init) gets RT_ERR_COMM back instead of
// blocking forever, and the half-built communicator is aborted.
int rt_comm_init_rank_timeout(rt_ctx* c, int nranks, int rank, const char id[RT_COMM_ID_BYTES], int timeout_ms) {
    if (!c) return RT_ERR_INVALID;
    if (!id || nranks < 1 || rank < 0 || rank >= nranks || timeout_ms < 1)
        return fail(c, RT_ERR_INVALID, "rank %d of %d (id %s, timeout %d ms)", rank, nranks, id ? "given" : "NULL",
                    timeout_ms);
    if (c->comm) return fail(c, RT_ERR_INVALID, "context already has a communicator (rt_comm_destroy first)");
    HIPCHK(c, hipSetDevice(c->device));
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    ncclComm_t comm = nullptr;
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    ncclResult_t r = ncclCommInitRankConfig(&comm, nranks, u, rank, &cfg);
    if (r == ncclInProgress || r == ncclSuccess) r = comm ? wait_comm(comm, timeout_ms) : r;
    if (r != ncclSuccess) {
        if (comm) (void)ncclCommAbort(comm);
        return fail(c, RT_ERR_COMM, "ncclCommInitRankConfig (rank %d of %d): %s", rank, nranks,
                    r == ncclInProgress ? "timed out waiting for the other ranks" : ncclGetErrorString(r));
    }
    c->comm = comm;
    c->comm_rank = rank;
    c->comm_size = nranks;
    c->comm_nonblocking = true;
    return RT_OK;
}

int rt_comm_init_all(rt_ctx** cs, int n) {
    if (!cs || n < 1) return RT_ERR_INVALID;
    for (int r = 0; r < n; ++r) {
        if (!cs[r]) return RT_ERR_INVALID;
        if (cs[r]->comm) return fail(cs[0], RT_ERR_INVALID, "context %d already has a communicator", r);
        for (int q = 0; q < r; ++q)
            if (cs[q] == cs[r]) return fail(cs[0], RT_ERR_INVALID, "context %d is listed twice", r);
    }
    std::vector<int> devs(n);
    for (int r = 0; r < n; ++r) devs[r] = cs[r]->device;
    std::vector<ncclComm_t> comms(n, nullptr);
    NCCLCHK(cs[0], ncclCommInitAll(comms.data(), n, devs.data()));
    for (int r = 0; r < n; ++r) {
        cs[r]->comm = comms[r];
        cs[r]->comm_rank = r;
        cs[r]->comm_size = n;
    }
    return RT_OK;
}

int rt_comm_rank(rt_ctx* c, int* rank, int* nranks) {
    if (!c || !rank || !nranks) return RT_ERR_INVALID;
    if (!c->comm) return fail(c, RT_ERR_INVALID, "no communicator");
    *rank = c->comm_rank;
    *nranks = c->comm_size;
    return RT_OK;
}

int rt_comm_destroy(rt_ctx* c) {
    if (!c) return RT_ERR_INVALID;
    (void)hipSetDevice(c->device);
    rt_comm_release(c);
    return RT_OK;
}

int rt_gather_shards(rt_ctx* c, const void* shard, void* gathered, int W, int H, void* stream) {
    if (!c) return RT_ERR_INVALID;
    if (!c->comm) return fail(c, RT_ERR_INVALID, "rt_gather_shards without a communicator");
    const size_t n = shard_elems(W, H, c->comm_size);
    if (!shard || n == 0 || (c->comm_rank == 0 && !gathered))
        return fail(c, RT_ERR_INVALID, "gather of a %dx%d frame: shard %p, gathered %p", W, H, shard, gathered);
    HIPCHK(c, hipSetDevice(c->device));
    ncclResult_t r = ncclGather(shard, gathered, n, dtype_of(c), 0, (ncclComm_t)c->comm,
                                stream ? (hipStream_t)stream : c->stream);
    if (r == ncclInProgress && c->comm_nonblocking) r = wait_comm((ncclComm_t)c->comm, RT_COMM_INIT_TIMEOUT_MS);
    if (r != ncclSuccess) return fail(c, RT_ERR_COMM, "ncclGather: %s", ncclGetErrorString(r));
    return RT_OK;
}

}  // extern "C"

// rt_render_frame_multi's gather when its contexts share a communicator from
// rt_comm_init_all: one grouped ncclGather, each rank on its own context's stream (after
// its render); `gathered` is on cs[0]'s device.
int rt_comm_gather_group(rt_ctx** cs, int n, size_t elems, void* gathered) {
    for (int r = 0; r < n; ++r)
        if (!cs[r]->comm || cs[r]->comm_size != n || cs[r]->comm_rank != r)
            return fail(cs[0], RT_ERR_INVALID, "context %d is not rank %d of an %d-rank communicator", r, r, n);
    NCCLCHK(cs[0], ncclGroupStart());
    for (int r = 0; r < n; ++r) {
        const ncclResult_t e = ncclGather(cs[r]->d_shard, r == 0 ? gathered : nullptr, elems, dtype_of(cs[r]), 0,
                                          (ncclComm_t)cs[r]->comm, cs[r]->stream);
        if (e != ncclSuccess) {
            (void)ncclGroupEnd();
            return fail(cs[0], RT_ERR_COMM, "ncclGather (rank %d): %s", r, ncclGetErrorString(e));
        }
    }
    NCCLCHK(cs[0], ncclGroupEnd());
    return RT_OK;
}
