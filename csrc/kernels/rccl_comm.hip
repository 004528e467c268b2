// RCCL controller: one communicator per cluster version, bootstrapped with a
// unique id broadcast over the kungfu host transport (like the reference's
// NCCL bootstrap, srcs/cpp/src/nccl/gpu_collective.cpp:130-152), issuing
// collectives on a caller-chosen HIP stream with NO host synchronisation
// (the reference syncs the stream after every op, gpu_collective.cpp:104,115,126;
// here completion is tracked with hipEvents by the Python scheduler).
//
// Covers every NCCL call of the reference (AllReduce / Reduce / Broadcast,
// gpu_collective.cpp:102-126) plus AllGather / ReduceScatter / Send / Recv used
// by the bucketed DP engine and the device-side graph strategies.
#include "rccl_comm.hpp"

#include <rccl/rccl.h>

#include <cstring>
#include <stdexcept>
#include <string>

namespace kfk {

namespace {

void check(ncclResult_t r, const char *what) {
    if (r != ncclSuccess && r != ncclInProgress)
        throw std::runtime_error(std::string("rccl ") + what + ": " + ncclGetErrorString(r));
}

void hcheck(hipError_t e, const char *what) {
    if (e != hipSuccess) throw std::runtime_error(std::string("hip ") + what + ": " + hipGetErrorString(e));
}

ncclDataType_t nccl_dtype(int dt) {
    switch (dt) {
    case 0: return ncclUint8;
    case 2: return ncclUint32;
    case 3: return ncclUint64;
    case 4: return ncclInt8;
    case 6: return ncclInt32;
    case 7: return ncclInt64;
    case 8: return ncclFloat16;
    case 9: return ncclBfloat16;
    case 10: return ncclFloat32;
    case 11: return ncclFloat64;
    case 12: return ncclUint8;  // bool
    }
    throw std::invalid_argument("rccl: unsupported dtype code " + std::to_string(dt));
}

ncclRedOp_t nccl_op(int op) {
    switch (op) {
    case 0: return ncclSum;
    case 1: return ncclMin;
    case 2: return ncclMax;
    case 3: return ncclProd;
    case 4: return ncclAvg;
    }
    throw std::invalid_argument("rccl: unsupported op code " + std::to_string(op));
}

}  // namespace

std::string RcclComm::unique_id() {
    ncclUniqueId id;
    check(ncclGetUniqueId(&id), "GetUniqueId");
    return std::string(reinterpret_cast<const char *>(&id), sizeof(id));
}

int RcclComm::version() {
    int v = 0;
    ncclGetVersion(&v);
    return v;
}

RcclComm::RcclComm(const std::string &id, int rank, int size, int device) : rank_(rank), size_(size) {
    if (id.size() != sizeof(ncclUniqueId)) throw std::invalid_argument("rccl: bad unique id length");
    hcheck(hipSetDevice(device), "SetDevice");
    ncclUniqueId uid;
    std::memcpy(&uid, id.data(), sizeof(uid));
    ncclComm_t c = nullptr;
    check(ncclCommInitRank(&c, size, uid, rank), "CommInitRank");
    comm_ = c;
}

RcclComm::~RcclComm() { destroy(); }

void RcclComm::destroy() {
    if (comm_) {
        ncclCommDestroy(static_cast<ncclComm_t>(comm_));
        comm_ = nullptr;
    }
}

void RcclComm::abort() {
    if (comm_) {
        ncclCommAbort(static_cast<ncclComm_t>(comm_));
        comm_ = nullptr;
    }
}

#define KFK_COMM static_cast<ncclComm_t>(comm_)
#define KFK_NEED_COMM \
    if (!comm_) throw std::runtime_error("rccl: communicator destroyed")

void RcclComm::all_reduce(const void *send, void *recv, size_t count, int dtype, int op, hipStream_t s) {
    KFK_NEED_COMM;
    check(ncclAllReduce(send, recv, count, nccl_dtype(dtype), nccl_op(op), KFK_COMM, s), "AllReduce");
}

void RcclComm::reduce(const void *send, void *recv, size_t count, int dtype, int op, int root, hipStream_t s) {
    KFK_NEED_COMM;
    check(ncclReduce(send, recv, count, nccl_dtype(dtype), nccl_op(op), root, KFK_COMM, s), "Reduce");
}

void RcclComm::broadcast(const void *send, void *recv, size_t count, int dtype, int root, hipStream_t s) {
    KFK_NEED_COMM;
    check(ncclBroadcast(send, recv, count, nccl_dtype(dtype), root, KFK_COMM, s), "Broadcast");
}

void RcclComm::all_gather(const void *send, void *recv, size_t count, int dtype, hipStream_t s) {
    KFK_NEED_COMM;
    check(ncclAllGather(send, recv, count, nccl_dtype(dtype), KFK_COMM, s), "AllGather");
}

void RcclComm::reduce_scatter(const void *send, void *recv, size_t count, int dtype, int op, hipStream_t s) {
    KFK_NEED_COMM;
    check(ncclReduceScatter(send, recv, count, nccl_dtype(dtype), nccl_op(op), KFK_COMM, s), "ReduceScatter");
}

void RcclComm::send(const void *buf, size_t count, int dtype, int peer, hipStream_t s) {
    KFK_NEED_COMM;
    check(ncclSend(buf, count, nccl_dtype(dtype), peer, KFK_COMM, s), "Send");
}

void RcclComm::recv(void *buf, size_t count, int dtype, int peer, hipStream_t s) {
    KFK_NEED_COMM;
    check(ncclRecv(buf, count, nccl_dtype(dtype), peer, KFK_COMM, s), "Recv");
}

void RcclComm::group_start() { check(ncclGroupStart(), "GroupStart"); }
void RcclComm::group_end() { check(ncclGroupEnd(), "GroupEnd"); }

}  // namespace kfk
