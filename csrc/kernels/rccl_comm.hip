// RCCL controller: one communicator per cluster version, bootstrapped with a
// unique id broadcast over the kungfu host transport (like the reference's
// NCCL bootstrap, srcs/cpp/src/nccl/gpu_collective.cpp:130-152), issuing
// collectives on a caller-chosen HIP stream with NO host synchronisation
// (the reference syncs the stream after every op, gpu_collective.cpp:104,115,126;
// here completion is tracked with hipEvents).
//
// Covers every NCCL call of the reference (AllReduce / Reduce / Broadcast,
// gpu_collective.cpp:102-126) plus AllGather / ReduceScatter / Send / Recv used
// by the bucketed DP engine and the device-side graph strategies.
//
// Failure detection (the reference checks every NCCL result and syncs, and wraps
// every op in a stall detector, srcs/go/libkungfu-comm/main.go:163-179):
//  * communicators are created NON-BLOCKING (ncclCommInitRankConfig, blocking=0)
//    and polled against a deadline, so a rank whose peers never arrive fails
//    with a message instead of hanging in ncclCommInitRank;
//  * every collective registers a completion event with a process-wide watchdog
//    thread which also polls ncclCommGetAsyncError of every live communicator;
//    an async error is reported by name and rank, every communicator is aborted
//    and the process exits with status 3.  A stalled op (older than the timeout)
//    is only LOGGED by default (600 s; like the reference's stall detector,
//    srcs/go/utils/stalldetector.go, which never kills): a peer may legitimately
//    spend long in an evaluation or checkpoint while the others wait in the next
//    bucket.  Setting KUNGFU_RCCL_TIMEOUT_S explicitly (bench.py does) makes a
//    stall fatal as well (abort + exit 3); KUNGFU_RCCL_STALL_ACTION=log|abort
//    overrides either default.
#include "rccl_comm.hpp"

#include <rccl/rccl.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <set>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace kfk {

namespace {

double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

double env_double(const char *k, double def) {
    const char *v = std::getenv(k);
    if (!v || !*v) return def;
    char *end = nullptr;
    double d = std::strtod(v, &end);
    return end == v ? def : d;
}

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

const char *dtype_name(int dt) {
    switch (dt) {
    case 0: return "u8";
    case 2: return "u32";
    case 3: return "u64";
    case 4: return "i8";
    case 6: return "i32";
    case 7: return "i64";
    case 8: return "f16";
    case 9: return "bf16";
    case 10: return "f32";
    case 11: return "f64";
    case 12: return "bool";
    }
    return "?";
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

// ---------------------------------------------------------------- watchdog
class Watchdog {
  public:
    static Watchdog &get() {
        static Watchdog *w = new Watchdog();  // never destroyed: usable from atexit paths
        return *w;
    }

    void add(hipStream_t s, std::string what) {
        if (timeout_ <= 0) return;
        hipEvent_t ev = nullptr;
        {
            std::lock_guard<std::mutex> lk(mu_);
            if (!pool_.empty()) {
                ev = pool_.back();
                pool_.pop_back();
            }
        }
        if (!ev && hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) return;
        if (hipEventRecord(ev, s) != hipSuccess) {
            std::lock_guard<std::mutex> lk(mu_);
            pool_.push_back(ev);
            return;
        }
        std::lock_guard<std::mutex> lk(mu_);
        q_.push_back(Entry{ev, std::move(what), now_s()});
        ++registered_;
        start_locked();
    }

    void add_comm(void *c) {
        std::lock_guard<std::mutex> lk(mu_);
        comms_.insert(c);
        if (timeout_ > 0) start_locked();
    }

    void remove_comm(void *c) {
        std::lock_guard<std::mutex> lk(mu_);
        comms_.erase(c);
    }

    void set_label(const std::string &l) {
        std::lock_guard<std::mutex> lk(mu_);
        label_ = l;
    }

    void set_timeout(double t) { timeout_ = t; }
    void set_freeze(void (*fn)()) { freeze_ = fn; }

    WatchdogInfo info() {
        std::lock_guard<std::mutex> lk(mu_);
        WatchdogInfo i;
        i.registered = registered_;
        i.completed = completed_;
        i.pending = static_cast<long long>(q_.size());
        double t = now_s();
        for (const auto &e : q_) i.oldest_s = std::max(i.oldest_s, t - e.t0);
        i.timeout_s = timeout_;
        i.abort_on_stall = abort_on_stall_;
        i.stalls_logged = stalls_logged_;
        return i;
    }

  private:
    struct Entry {
        hipEvent_t ev;
        std::string what;
        double t0;
        double warned = 0;  // log-only mode: time of the last stall warning
    };

    Watchdog() : timeout_(env_double("KUNGFU_RCCL_TIMEOUT_S", 600.0)) {
        const char *t = std::getenv("KUNGFU_RCCL_TIMEOUT_S");
        abort_on_stall_ = t && *t;
        const char *a = std::getenv("KUNGFU_RCCL_STALL_ACTION");
        if (a && std::string(a) == "abort") abort_on_stall_ = true;
        if (a && std::string(a) == "log") abort_on_stall_ = false;
    }

    void start_locked() {
        if (started_) return;
        started_ = true;
        std::thread([this] { loop(); }).detach();
    }

    void loop() {
        const double period = std::min(0.05, std::max(0.005, timeout_ / 20));
        for (;;) {
            std::this_thread::sleep_for(std::chrono::duration<double>(period));
            std::string fail;
            {
                std::lock_guard<std::mutex> lk(mu_);
                const double t = now_s();
                for (auto it = q_.begin(); it != q_.end();) {
                    hipError_t r = hipEventQuery(it->ev);
                    if (r == hipSuccess) {
                        pool_.push_back(it->ev);
                        it = q_.erase(it);
                        ++completed_;
                        continue;
                    }
                    if (r == hipErrorCapturedEvent || r == hipErrorStreamCaptureUnsupported ||
                        r == hipErrorStreamCaptureImplicit || r == hipErrorStreamCaptureWrongThread) {
                        // the op's stream joined a hipGraph capture after the op was enqueued: its
                        // event cannot be queried until the capture ends -- look again later
                        ++it;
                        continue;
                    }
                    if (r != hipErrorNotReady) {
                        fail = "device error while waiting for " + it->what + ": " + hipGetErrorString(r);
                        break;
                    }
                    if (timeout_ > 0 && t - it->t0 > timeout_) {
                        char buf[160];
                        std::snprintf(buf, sizeof(buf), " has not completed after %.1f s (KUNGFU_RCCL_TIMEOUT_S=%g)",
                                      t - it->t0, timeout_.load());
                        if (abort_on_stall_) {
                            fail = "collective " + it->what + buf;
                            break;
                        }
                        if (t - it->warned > timeout_) {  // log-only: warn again every timeout period
                            it->warned = t;
                            ++stalls_logged_;
                            std::fprintf(stderr, "[W] kungfu rccl watchdog (%s): collective %s%s; still waiting "
                                         "(set KUNGFU_RCCL_TIMEOUT_S or KUNGFU_RCCL_STALL_ACTION=abort to fail)\n",
                                         label_.empty() ? "?" : label_.c_str(), it->what.c_str(), buf);
                            std::fflush(stderr);
                        }
                    }
                    ++it;
                }
                if (fail.empty()) {
                    for (void *c : comms_) {
                        ncclResult_t st = ncclSuccess;
                        if (ncclCommGetAsyncError(static_cast<ncclComm_t>(c), &st) == ncclSuccess &&
                            st != ncclSuccess && st != ncclInProgress) {
                            fail = std::string("communicator async error: ") + ncclGetErrorString(st);
                            break;
                        }
                    }
                }
                if (!fail.empty()) die_locked(fail);
            }
        }
    }

    [[noreturn]] void die_locked(const std::string &why) {
        std::fprintf(stderr, "[F] kungfu rccl watchdog (%s): %s\n", label_.empty() ? "?" : label_.c_str(),
                     why.c_str());
        int shown = 0;
        const double t = now_s();
        for (const auto &e : q_) {
            if (shown++ == 8) {
                std::fprintf(stderr, "[F]   ... %zu pending ops in total\n", q_.size());
                break;
            }
            std::fprintf(stderr, "[F]   pending: %s (enqueued %.1f s ago)\n", e.what.c_str(), t - e.t0);
        }
        std::fprintf(stderr, "[F] aborting %zu communicator(s) and exiting with status 3\n", comms_.size());
        std::fflush(stderr);
        std::fflush(stdout);
        if (freeze_) {  // stop the application's threads first (bounded: 2 s)
            auto frozen = std::make_shared<std::atomic<bool>>(false);
            void (*f)() = freeze_;
            std::thread([f, frozen] {
                f();
                frozen->store(true);
                for (;;) std::this_thread::sleep_for(std::chrono::seconds(1));
            }).detach();
            const double t_frz = now_s() + 2.0;
            while (!frozen->load() && now_s() < t_frz) std::this_thread::sleep_for(std::chrono::milliseconds(5));
        }
        // ncclCommAbort makes the RCCL kernels leave their wait loops, so the process
        // does not exit with waves spinning on the device; bounded, it runs detached.
        std::vector<void *> cs(comms_.begin(), comms_.end());
        auto done = std::make_shared<std::atomic<bool>>(false);
        std::thread([cs, done] {
            for (void *c : cs) ncclCommAbort(static_cast<ncclComm_t>(c));
            done->store(true);
        }).detach();
        const double t_end = now_s() + 15.0;
        while (!done->load() && now_s() < t_end) std::this_thread::sleep_for(std::chrono::milliseconds(20));
        ::_exit(3);
    }

    std::mutex mu_;
    std::deque<Entry> q_;
    std::vector<hipEvent_t> pool_;
    std::set<void *> comms_;
    std::string label_;
    std::atomic<double> timeout_;
    void (*freeze_)() = nullptr;
    bool started_ = false;
    bool abort_on_stall_ = false;
    long long registered_ = 0, completed_ = 0, stalls_logged_ = 0;
};

}  // namespace

WatchdogInfo watchdog_info() { return Watchdog::get().info(); }
void watchdog_set_label(const std::string &label) { Watchdog::get().set_label(label); }
void watchdog_set_timeout(double seconds) { Watchdog::get().set_timeout(seconds); }
void watchdog_set_freeze_hook(void (*fn)()) { Watchdog::get().set_freeze(fn); }

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

RcclComm::RcclComm(const std::string &id, int rank, int size, int device, double init_timeout_s, int min_ctas,
                   int max_ctas)
    : rank_(rank), size_(size) {
    if (id.size() != sizeof(ncclUniqueId)) throw std::invalid_argument("rccl: bad unique id length");
    hcheck(hipSetDevice(device), "SetDevice");
    ncclUniqueId uid;
    std::memcpy(&uid, id.data(), sizeof(uid));
    if (init_timeout_s <= 0) init_timeout_s = env_double("KUNGFU_RCCL_INIT_TIMEOUT_S", 300.0);
    blocking_ = env_double("KUNGFU_RCCL_BLOCKING", 0) != 0;
    if (min_ctas <= 0) min_ctas = static_cast<int>(env_double("KUNGFU_RCCL_MIN_CTAS", 0));
    if (max_ctas <= 0) max_ctas = static_cast<int>(env_double("KUNGFU_RCCL_MAX_CTAS", 0));
    if (min_ctas > 0 && max_ctas > 0 && min_ctas > max_ctas) min_ctas = max_ctas;
    if (min_ctas > 0 && max_ctas <= 0)  // RCCL rejects a minCTAs without a maxCTAs ("invalid argument")
        throw std::invalid_argument("rccl: KUNGFU_RCCL_MIN_CTAS needs KUNGFU_RCCL_MAX_CTAS as well");
    min_ctas_ = min_ctas > 0 ? min_ctas : 0;
    max_ctas_ = max_ctas > 0 ? max_ctas : 0;
    if (blocking_ && (min_ctas_ || max_ctas_))
        throw std::invalid_argument("rccl: a CTA budget needs the config init (KUNGFU_RCCL_BLOCKING=0)");
    ncclComm_t c = nullptr;
    if (!blocking_) {
        ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
        cfg.version = static_cast<unsigned int>(version());  // the loaded library's, not the header's
        cfg.blocking = 0;
        if (min_ctas_) cfg.minCTAs = min_ctas_;
        if (max_ctas_) cfg.maxCTAs = max_ctas_;
        ncclResult_t r = ncclCommInitRankConfig(&c, size, uid, rank, &cfg);
        if (r != ncclSuccess && r != ncclInProgress) {
            if (c) ncclCommAbort(c);
            throw std::runtime_error(std::string("rccl CommInitRankConfig: ") + ncclGetErrorString(r));
        }
        comm_ = c;
        try {
            wait_ready("CommInitRankConfig", init_timeout_s);
        } catch (...) {
            ncclCommAbort(c);
            comm_ = nullptr;
            throw;
        }
    } else {
        check(ncclCommInitRank(&c, size, uid, rank), "CommInitRank");
        comm_ = c;
    }
    Watchdog::get().add_comm(comm_);
}

RcclComm::~RcclComm() { destroy(); }

void RcclComm::wait_ready(const char *what, double timeout_s) {
    if (blocking_ || !comm_) return;
    const double t_end = now_s() + timeout_s;
    int sleep_us = 20;
    for (;;) {
        ncclResult_t st = ncclSuccess;
        ncclResult_t r = ncclCommGetAsyncError(static_cast<ncclComm_t>(comm_), &st);
        if (r != ncclSuccess) throw std::runtime_error(std::string("rccl CommGetAsyncError: ") + ncclGetErrorString(r));
        if (st == ncclSuccess) return;
        if (st != ncclInProgress)
            throw std::runtime_error(std::string("rccl ") + what + " (rank " + std::to_string(rank_) + " of " +
                                     std::to_string(size_) + "): " + ncclGetErrorString(st));
        if (now_s() > t_end) {
            char buf[64];
            std::snprintf(buf, sizeof(buf), "%.0f", timeout_s);
            throw std::runtime_error(std::string("rccl ") + what + " timed out after " + buf + " s on rank " +
                                     std::to_string(rank_) + " of " + std::to_string(size_) +
                                     " (a peer never joined, or the bootstrap address is unreachable)");
        }
        std::this_thread::sleep_for(std::chrono::microseconds(sleep_us));
        sleep_us = std::min(sleep_us * 2, 20000);
    }
}

void RcclComm::enq(int r, const char *what) {
    check(static_cast<ncclResult_t>(r), what);
    if (static_cast<ncclResult_t>(r) == ncclInProgress)
        wait_ready(what, env_double("KUNGFU_RCCL_INIT_TIMEOUT_S", 300.0));
}

void RcclComm::watch(hipStream_t s, const std::string &what) {
    // inside a hipGraph capture the collective is a graph node, not work in flight: an event
    // recorded now would never complete as such (and querying it from the watchdog thread is
    // not allowed during capture) -- graph replays are not watched
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone) return;
    char buf[64];
    std::snprintf(buf, sizeof(buf), " #%llu on rank %d/%d", ++seq_, rank_, size_);
    Watchdog::get().add(s, what + buf);
}

int RcclComm::async_error() {
    if (!comm_) return 0;
    ncclResult_t st = ncclSuccess;
    ncclCommGetAsyncError(static_cast<ncclComm_t>(comm_), &st);
    return static_cast<int>(st);
}

void RcclComm::destroy() {
    if (!comm_) return;
    ncclComm_t c = static_cast<ncclComm_t>(comm_);
    Watchdog::get().remove_comm(comm_);
    bool ok = true;
    if (!blocking_) {
        // finalize flushes outstanding work; bounded, then destroy (or abort on expiry)
        ncclResult_t r = ncclCommFinalize(c);
        if (r == ncclSuccess || r == ncclInProgress) {
            try {
                wait_ready("CommFinalize", env_double("KUNGFU_RCCL_INIT_TIMEOUT_S", 300.0));
            } catch (const std::exception &e) {
                std::fprintf(stderr, "[W] %s; aborting the communicator\n", e.what());
                ok = false;
            }
        } else {
            ok = false;
        }
    }
    if (ok)
        ncclCommDestroy(c);
    else
        ncclCommAbort(c);
    comm_ = nullptr;
}

void RcclComm::abort() {
    if (comm_) {
        Watchdog::get().remove_comm(comm_);
        ncclCommAbort(static_cast<ncclComm_t>(comm_));
        comm_ = nullptr;
    }
}

#define KFK_COMM static_cast<ncclComm_t>(comm_)
#define KFK_NEED_COMM \
    if (!comm_) throw std::runtime_error("rccl: communicator destroyed")

namespace {
std::string opname(const char *op, const char *tag, size_t count, int dtype) {
    std::string s(op);
    s += "(";
    if (tag && *tag) {
        s += tag;
        s += ", ";
    }
    s += std::to_string(count) + " x " + dtype_name(dtype) + ")";
    return s;
}
}  // namespace

void RcclComm::all_reduce(const void *send, void *recv, size_t count, int dtype, int op, hipStream_t s,
                          const char *tag) {
    KFK_NEED_COMM;
    enq(ncclAllReduce(send, recv, count, nccl_dtype(dtype), nccl_op(op), KFK_COMM, s), "AllReduce");
    watch(s, opname("AllReduce", tag, count, dtype));
}

void RcclComm::reduce(const void *send, void *recv, size_t count, int dtype, int op, int root, hipStream_t s,
                      const char *tag) {
    KFK_NEED_COMM;
    enq(ncclReduce(send, recv, count, nccl_dtype(dtype), nccl_op(op), root, KFK_COMM, s), "Reduce");
    watch(s, opname("Reduce", tag, count, dtype));
}

void RcclComm::broadcast(const void *send, void *recv, size_t count, int dtype, int root, hipStream_t s,
                         const char *tag) {
    KFK_NEED_COMM;
    enq(ncclBroadcast(send, recv, count, nccl_dtype(dtype), root, KFK_COMM, s), "Broadcast");
    watch(s, opname("Broadcast", tag, count, dtype));
}

void RcclComm::all_gather(const void *send, void *recv, size_t count, int dtype, hipStream_t s, const char *tag) {
    KFK_NEED_COMM;
    enq(ncclAllGather(send, recv, count, nccl_dtype(dtype), KFK_COMM, s), "AllGather");
    watch(s, opname("AllGather", tag, count, dtype));
}

void RcclComm::reduce_scatter(const void *send, void *recv, size_t count, int dtype, int op, hipStream_t s,
                              const char *tag) {
    KFK_NEED_COMM;
    enq(ncclReduceScatter(send, recv, count, nccl_dtype(dtype), nccl_op(op), KFK_COMM, s), "ReduceScatter");
    watch(s, opname("ReduceScatter", tag, count, dtype));
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

void RcclComm::group_end() {
    ncclResult_t r = ncclGroupEnd();
    enq(r, "GroupEnd");
}

}  // namespace kfk
