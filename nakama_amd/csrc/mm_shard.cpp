// nakama_amd/csrc/mm_shard.cpp — the exchange of the row-sharded mode
// (include/nakama_cluster.h): each rank evaluates one block of a batch's
// searches and the blocks are all-gathered in place, over RCCL between device
// buffers (xGMI) or through a host-memory all-gather the caller supplies.
#include <rccl/rccl.h>

#include <cstring>

#include "mm_core.h"

namespace nkm {

namespace {
void nccl_check(ncclResult_t r, int line) {
    if (r != ncclSuccess) throw DeviceError{hipErrorUnknown, ncclGetErrorString(r), line};
}
#define NKM_NCCL(x) nccl_check((x), __LINE__)
}  // namespace

int Core::set_row_shard(int world, int rank, mm_allgather_fn fn, void* ctx) {
    std::lock_guard<std::mutex> pl(process_mu_);
    std::lock_guard<std::mutex> lk(mu_);
    if (world < 1 || rank < 0 || rank >= world) return MM_ERR_ARG;
    shard_release();
    shard_world_ = world;
    shard_rank_ = rank;
    shard_fn_ = fn;
    shard_ctx_ = ctx;
    return MM_OK;
}

int Core::set_row_shard_rccl(int world, int rank, const uint8_t* uid, int len) {
    std::lock_guard<std::mutex> pl(process_mu_);
    std::lock_guard<std::mutex> lk(mu_);
    if (world < 1 || rank < 0 || rank >= world || !uid || len != NCCL_UNIQUE_ID_BYTES) return MM_ERR_ARG;
    shard_release();
    NKM_HIP(hipSetDevice(device_));
    ncclUniqueId id;
    std::memcpy(id.internal, uid, NCCL_UNIQUE_ID_BYTES);
    ncclComm_t comm = nullptr;
    NKM_NCCL(ncclCommInitRank(&comm, world, id, rank));
    nccl_comm_ = comm;
    shard_world_ = world;
    shard_rank_ = rank;
    return MM_OK;
}

void Core::shard_release() {
    if (nccl_comm_) {
        (void)ncclCommDestroy(static_cast<ncclComm_t>(nccl_comm_));
        nccl_comm_ = nullptr;
    }
    shard_world_ = 1;
    shard_rank_ = 0;
    shard_fn_ = nullptr;
    shard_ctx_ = nullptr;
}

// One in-place broadcast per rank (rooted at its segment) in one group: the
// all-gather-v RCCL has no single call for; each link carries every segment once.
void Core::shard_gather_device(void* dbuf, const std::vector<int64_t>& off) {
    auto* comm = static_cast<ncclComm_t>(nccl_comm_);
    char* b = static_cast<char*>(dbuf);
    NKM_NCCL(ncclGroupStart());
    for (int q = 0; q < shard_world_; q++) {
        const int64_t n = off[q + 1] - off[q];
        if (n > 0) NKM_NCCL(ncclBroadcast(b + off[q], b + off[q], (size_t)n, ncclChar, q, comm, stream_));
    }
    NKM_NCCL(ncclGroupEnd());
}

void Core::shard_gather_host(void* hbuf, const std::vector<int64_t>& off) {
    if (shard_fn_(shard_ctx_, hbuf, off.data()) != 0)
        throw DeviceError{hipErrorUnknown, "row-shard all-gather callback failed", __LINE__};
}

bool Core::shard_any(bool v) {
    if (!row_shard()) return v;
    std::vector<int64_t> off(shard_world_ + 1);
    for (int q = 0; q <= shard_world_; q++) off[q] = q;
    if (nccl_comm_) {
        DevArray<uint8_t>& d = d_pair_out_;
        d.reserve(shard_world_, false);
        uint8_t mine = v ? 1 : 0;
        NKM_HIP(hipMemcpyAsync(d.p + shard_rank_, &mine, 1, hipMemcpyHostToDevice, stream_));
        shard_gather_device(d.p, off);
        std::vector<uint8_t> all(shard_world_);
        NKM_HIP(hipMemcpyAsync(all.data(), d.p, shard_world_, hipMemcpyDeviceToHost, stream_));
        NKM_HIP(hipStreamSynchronize(stream_));
        for (uint8_t x : all) v |= x != 0;
        return v;
    }
    std::vector<uint8_t> all(shard_world_, 0);
    all[shard_rank_] = v ? 1 : 0;
    shard_gather_host(all.data(), off);
    for (uint8_t x : all) v |= x != 0;
    return v;
}

}  // namespace nkm

extern "C" {

int mm_rccl_unique_id(uint8_t* out, int32_t cap) {
    if (!out || cap < NCCL_UNIQUE_ID_BYTES) return MM_ERR_ARG;
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return MM_ERR_DEVICE;
    std::memcpy(out, id.internal, NCCL_UNIQUE_ID_BYTES);
    return MM_OK;
}

}  // extern "C"
