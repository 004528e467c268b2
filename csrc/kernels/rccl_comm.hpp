// RCCL communicator wrapper + device-plane watchdog (see rccl_comm.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <string>

namespace kfk {

class RcclComm {
  public:
    static std::string unique_id();  // 128-byte ncclUniqueId
    static int version();
    // Non-blocking init (ncclCommInitRankConfig, blocking=0) polled against a deadline
    // of `init_timeout_s` seconds (<= 0: KUNGFU_RCCL_INIT_TIMEOUT_S, default 300); on
    // expiry the half-built communicator is aborted and std::runtime_error is thrown.
    // CTA budget (ncclConfig_t.minCTAs / maxCTAs): how many workgroups -- RCCL channels --
    // one collective of this communicator may occupy; <= 0 = KUNGFU_RCCL_MIN_CTAS /
    // KUNGFU_RCCL_MAX_CTAS, unset = RCCL's own choice.  Bounds the CUs the gradient
    // all-reduces take from the overlapped backward (and lets two communicators driven
    // concurrently -- the hierarchical local reduce / broadcast -- stay co-resident).
    RcclComm(const std::string &id, int rank, int size, int device, double init_timeout_s = 0, int min_ctas = 0,
             int max_ctas = 0);
    ~RcclComm();
    RcclComm(const RcclComm &) = delete;
    RcclComm &operator=(const RcclComm &) = delete;

    int rank() const { return rank_; }
    int size() const { return size_; }
    bool valid() const { return comm_ != nullptr; }
    bool blocking() const { return blocking_; }
    int min_ctas() const { return min_ctas_; }  // 0 = RCCL default
    int max_ctas() const { return max_ctas_; }

    // dtype / op codes follow kungfu::DType / ReduceOp (op 4 = average).  `tag` names the
    // operation for the watchdog (e.g. "bucket 3/5"); every op is registered with it.
    void all_reduce(const void *send, void *recv, size_t count, int dtype, int op, hipStream_t s,
                    const char *tag = "");
    void reduce(const void *send, void *recv, size_t count, int dtype, int op, int root, hipStream_t s,
                const char *tag = "");
    void broadcast(const void *send, void *recv, size_t count, int dtype, int root, hipStream_t s,
                   const char *tag = "");
    void all_gather(const void *send, void *recv, size_t count, int dtype, hipStream_t s, const char *tag = "");
    void reduce_scatter(const void *send, void *recv, size_t count, int dtype, int op, hipStream_t s,
                        const char *tag = "");
    // point-to-point: no watchdog entry of their own (callers group them and call watch())
    void send(const void *buf, size_t count, int dtype, int peer, hipStream_t s);
    void recv(void *buf, size_t count, int dtype, int peer, hipStream_t s);
    void group_start();
    void group_end();  // polls this communicator when it is non-blocking
    // register "everything issued on s so far" with the watchdog under `what`
    void watch(hipStream_t s, const std::string &what);
    // ncclCommGetAsyncError as an int (0 = success, 7 = in progress)
    int async_error();
    void destroy();  // finalize (bounded) + destroy; aborts if finalize does not finish
    void abort();

  private:
    void wait_ready(const char *what, double timeout_s);
    void enq(int r, const char *what);
    void *comm_ = nullptr;
    int rank_, size_;
    bool blocking_ = true;
    int min_ctas_ = 0, max_ctas_ = 0;
    unsigned long long seq_ = 0;
};

// Process-wide device-plane watchdog (parity: the reference's synchronous NCCL error
// check after every op, srcs/cpp/src/nccl/gpu_collective.cpp:96-128, and its stall
// detector around every op, srcs/go/libkungfu-comm/main.go:163-179).  A host thread
// polls the completion event of every registered collective and every live
// communicator's async error; when an op is older than KUNGFU_RCCL_TIMEOUT_S (default
// 600, 0 disables) or a communicator reports an error, it prints which op stalled on
// which rank, aborts every communicator (RCCL kernels leave their spin loops) and
// terminates the process with exit code 3 (never re-execs).
struct WatchdogInfo {
    long long registered = 0, completed = 0, pending = 0;
    double oldest_s = 0, timeout_s = 0;
    bool abort_on_stall = false;  // false: a stall past timeout_s is logged, not fatal
    long long stalls_logged = 0;
};
WatchdogInfo watchdog_info();
void watchdog_set_label(const std::string &label);  // e.g. "rank 3/8"
void watchdog_set_timeout(double seconds);
// Called (on a helper thread) before the communicators are aborted: the Python binding
// takes the GIL there and never releases it, so no Python thread runs on with results
// of the aborted collectives during the few ms until the process exits.
void watchdog_set_freeze_hook(void (*fn)());

}  // namespace kfk
