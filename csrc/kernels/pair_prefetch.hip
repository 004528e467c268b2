// Native prefetch of the pair-averaging peer model (PairAveragingOptimizer, GPU path).
//
// Parity: the reference's AsyncModelAveraging / AsyncRequestModel keep a prefetch buffer filled by
// a native callback (srcs/cpp/src/tensorflow/ops/cpu/peer_to_peer.cpp:166-238,424-510).  Here one
// C++ thread per optimizer does, per step and off the training thread (no Python, no GIL):
//   1. advertise: host-wait the event of the snapshot published at the end of the step, then save
//      the 16-byte (slot, version) record (and, with peers on other hosts, the host copy) in this
//      peer's store through the runtime's C API (libkungfu_amd: kungfu_save / kungfu_request);
//   2. pull: request the target's record, copy its advertised ring slot into the destination on a
//      dedicated HIP stream -- from the peer's IPC-mapped slot (same host, one-sided over xGMI) or
//      through the host store (other hosts: TCP into a pinned staging buffer, then H2D) -- after
//      the event of the kernel that consumed the previous pull, host-wait that copy, and fetch the
//      record again: a version that advanced by >= slots - 1 means the copy may overlap a rewrite,
//      and the pull is dropped (the torn-read-free protocol of optimizers/pair_avg.py).
// finish(stream) joins the step's work and makes `stream` wait on the copy (no host wait there).
#include <hip/hip_runtime.h>

#include <dlfcn.h>

#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "kernels.hpp"

namespace kfk {

namespace {

void hcheck(hipError_t e, const char *what) {
    if (e != hipSuccess) throw std::runtime_error(std::string("pair prefetch: ") + what + ": " + hipGetErrorString(e));
}

}  // namespace

struct PairPrefetcher::Impl {
    using SaveFn = int (*)(const char *, const void *, size_t);
    using RequestFn = int (*)(int, const char *, const char *, void *, size_t, int *);
    SaveFn save = nullptr;
    RequestFn request = nullptr;
    int device = 0, self_rank = 0, slots = 3;
    std::string rec_name, model_name;
    int64_t nbytes = 0;
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;

    std::mutex mu;
    std::condition_variable cv;
    std::thread worker;
    bool busy = false, have_job = false, stop = false;
    Job job;
    Result result;

    bool record(int target, int64_t own_ver, int64_t out[2]) {
        if (target == self_rank) {
            if (own_ver <= 0) return false;
            out[0] = own_ver % slots, out[1] = own_ver;
            return true;
        }
        int found = 0;
        if (request(target, "", rec_name.c_str(), out, 16, &found) != 0 || !found) return false;
        return true;
    }

    void run(const Job &j, Result &r) {
        hcheck(hipSetDevice(device), "SetDevice");
        int64_t own_ver = j.own_ver;
        if (j.pending_ev) {  // advertise the snapshot published at the end of the previous step
            hcheck(hipEventSynchronize(reinterpret_cast<hipEvent_t>(j.pending_ev)), "EventSynchronize(snapshot)");
            own_ver = j.pending_ver;
            const int64_t rec[2] = {own_ver % slots, own_ver};
            if (save(rec_name.c_str(), rec, 16) != 0) throw std::runtime_error("pair prefetch: saving the record failed");
            if (j.host_copy && save(model_name.c_str(), reinterpret_cast<const void *>(j.host_copy),
                                    static_cast<size_t>(nbytes)) != 0)
                throw std::runtime_error("pair prefetch: saving the host copy failed");
        }
        r = Result{};
        r.own_ver = own_ver;
        int64_t rec[2];
        if (!record(j.target, own_ver, rec)) return;
        const int64_t slot = rec[0], ver = rec[1];
        if (j.after_ev) hcheck(hipStreamWaitEvent(stream, reinterpret_cast<hipEvent_t>(j.after_ev), 0), "StreamWaitEvent");
        void *dst = reinterpret_cast<void *>(j.dst);
        if (!j.src_slots.empty()) {
            if (slot < 0 || slot >= static_cast<int64_t>(j.src_slots.size())) return;
            hcheck(hipMemcpyAsync(dst, reinterpret_cast<const void *>(j.src_slots[slot]), static_cast<size_t>(nbytes),
                                  hipMemcpyDeviceToDevice, stream),
                   "MemcpyAsync(peer slot)");
        } else {
            int found = 0;
            if (request(j.target, "", model_name.c_str(), reinterpret_cast<void *>(j.host_stage),
                        static_cast<size_t>(nbytes), &found) != 0 || !found)
                return;
            hcheck(hipMemcpyAsync(dst, reinterpret_cast<const void *>(j.host_stage), static_cast<size_t>(nbytes),
                                  hipMemcpyHostToDevice, stream),
                   "MemcpyAsync(host stage)");
        }
        hcheck(hipEventRecord(done, stream), "EventRecord");
        hcheck(hipEventSynchronize(done), "EventSynchronize(copy)");
        if (!j.src_slots.empty()) {
            int64_t after[2];
            if (!record(j.target, own_ver, after) || after[1] - ver >= slots - 1) {
                r.status = 2;  // the owner may have started rewriting the slot during the copy
                r.version = ver;
                return;
            }
        }
        r.status = 1;
        r.version = ver;
    }

    void loop() {
        for (;;) {
            Job j;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return have_job || stop; });
                if (stop && !have_job) return;
                j = job;
                have_job = false;
            }
            Result r;
            try {
                run(j, r);
            } catch (const std::exception &e) {
                r = Result{};
                r.error = e.what();
            }
            {
                std::lock_guard<std::mutex> lk(mu);
                result = r;
                busy = false;
            }
            cv.notify_all();
        }
    }
};

PairPrefetcher::PairPrefetcher(const std::string &libpath, int device, int self_rank, const std::string &rec_name,
                               const std::string &model_name, int64_t nbytes, int slots)
    : d_(new Impl) {
    void *h = dlopen(libpath.c_str(), RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen(libpath.c_str(), RTLD_NOW);
    if (!h) throw std::runtime_error("pair prefetch: cannot open " + libpath);
    d_->save = reinterpret_cast<Impl::SaveFn>(dlsym(h, "kungfu_save"));
    d_->request = reinterpret_cast<Impl::RequestFn>(dlsym(h, "kungfu_request"));
    if (!d_->save || !d_->request) throw std::runtime_error("pair prefetch: runtime C API not found in " + libpath);
    d_->device = device, d_->self_rank = self_rank, d_->slots = slots;
    d_->rec_name = rec_name, d_->model_name = model_name, d_->nbytes = nbytes;
    hcheck(hipSetDevice(device), "SetDevice");
    hcheck(hipStreamCreateWithFlags(&d_->stream, hipStreamNonBlocking), "StreamCreate");
    hcheck(hipEventCreateWithFlags(&d_->done, hipEventDisableTiming), "EventCreate");
    d_->worker = std::thread([this] { d_->loop(); });
}

PairPrefetcher::~PairPrefetcher() {
    {
        std::unique_lock<std::mutex> lk(d_->mu);
        d_->cv.wait(lk, [&] { return !d_->busy; });
        d_->stop = true;
    }
    d_->cv.notify_all();
    if (d_->worker.joinable()) d_->worker.join();
    (void)hipStreamSynchronize(d_->stream);
    (void)hipEventDestroy(d_->done);
    (void)hipStreamDestroy(d_->stream);
    delete d_;
}

void PairPrefetcher::start(const Job &j) {
    std::unique_lock<std::mutex> lk(d_->mu);
    d_->cv.wait(lk, [&] { return !d_->busy; });
    d_->job = j;
    d_->have_job = true;
    d_->busy = true;
    lk.unlock();
    d_->cv.notify_all();
}

bool PairPrefetcher::busy() {
    std::lock_guard<std::mutex> lk(d_->mu);
    return d_->busy;
}

PairPrefetcher::Result PairPrefetcher::finish(uintptr_t wait_stream) {
    std::unique_lock<std::mutex> lk(d_->mu);
    d_->cv.wait(lk, [&] { return !d_->busy; });
    Result r = d_->result;
    d_->result = Result{};
    lk.unlock();
    if (r.error.empty() && r.status == 1 && wait_stream)
        hcheck(hipStreamWaitEvent(reinterpret_cast<hipStream_t>(wait_stream), d_->done, 0), "StreamWaitEvent(done)");
    return r;
}

}  // namespace kfk
