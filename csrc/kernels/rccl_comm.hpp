// RCCL communicator wrapper (see rccl_comm.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <string>

namespace kfk {

class RcclComm {
  public:
    static std::string unique_id();  // 128-byte ncclUniqueId
    static int version();
    RcclComm(const std::string &id, int rank, int size, int device);
    ~RcclComm();
    RcclComm(const RcclComm &) = delete;
    RcclComm &operator=(const RcclComm &) = delete;

    int rank() const { return rank_; }
    int size() const { return size_; }
    bool valid() const { return comm_ != nullptr; }

    // dtype / op codes follow kungfu::DType / ReduceOp (op 4 = average).
    void all_reduce(const void *send, void *recv, size_t count, int dtype, int op, hipStream_t s);
    void reduce(const void *send, void *recv, size_t count, int dtype, int op, int root, hipStream_t s);
    void broadcast(const void *send, void *recv, size_t count, int dtype, int root, hipStream_t s);
    void all_gather(const void *send, void *recv, size_t count, int dtype, hipStream_t s);
    void reduce_scatter(const void *send, void *recv, size_t count, int dtype, int op, hipStream_t s);
    void send(const void *buf, size_t count, int dtype, int peer, hipStream_t s);
    void recv(void *buf, size_t count, int dtype, int peer, hipStream_t s);
    static void group_start();
    static void group_end();
    void destroy();
    void abort();

  private:
    void *comm_ = nullptr;
    int rank_, size_;
};

}  // namespace kfk
