// Ordered collective scheduler: every rank must issue its RCCL collectives in
// the SAME order, whatever order its backward pass produces the gradient
// buckets in.
//
// Parity: NCCLScheduler / LinearExecutor (srcs/cpp/include/kungfu/nccl/scheduler.hpp:15-80,
// srcs/cpp/src/nccl/scheduler.cpp:9-131): ops start in a fixed order; after the
// first step rank 0's observed arrival order is broadcast and becomes the
// order of later steps (auto_order).  Here the scheduler only DECIDES the
// launch order (ready() returns the ops that may start now); the launches are
// enqueued by the caller on its comm stream, so no dedicated NCCL thread and
// no host synchronisation are needed.
#pragma once

#include <kungfu/session.hpp>

#include <mutex>
#include <vector>

namespace kungfu {

class OrderedScheduler {
  public:
    explicit OrderedScheduler(int n);

    // Begin a step: nothing launched, arrivals cleared.
    void reset();
    // Op i became ready; returns the ops that may be launched now, in order.
    std::vector<int> ready(int i);
    // Remaining ops in order (end of step: unused / late ops).
    std::vector<int> flush();
    // Adopt rank 0's arrival order of the last step (broadcast over the session).
    // Ops that never arrived keep their relative order at the end.
    void auto_order(Session &s);
    void set_order(const std::vector<int> &order);

    std::vector<int> order() const;
    std::vector<int> arrivals() const;
    int size() const { return n_; }

  private:
    int n_;
    mutable std::mutex mu_;
    std::vector<int> order_;   // launch order (op ids)
    std::vector<char> ready_;  // per op
    std::vector<char> done_;   // per op
    std::vector<int> arrivals_;
    size_t next_ = 0;          // position in order_
};

// Gradient-bucket accounting of the S-SGD engine (kungfu_amd/parallel/ddp.py GradReducer): the
// per-parameter gradient hook is ONE call, mark(param), which counts the parameter's gradient
// arrival, decrements its bucket's pending count and, when the bucket is complete, asks the
// ordered scheduler which buckets may be launched now -- the bookkeeping the reference's
// NCCLScheduler does on its own thread (srcs/cpp/src/nccl/scheduler.cpp:9-131), done inline in
// the autograd hook with no Python per arrival.
//
// The first step after construction only learns how many gradients each parameter receives per
// backward (expected = fires of that step, set by learn()); later steps count down.
class BucketTracker {
  public:
    static constexpr int kLate = -1;  // mark(): this parameter's bucket was already launched

    // bucket_of[p] = bucket index of parameter p (0 .. n_buckets-1)
    BucketTracker(int n_buckets, const std::vector<int> &bucket_of);

    // A gradient of parameter p arrived.  Returns the buckets to launch now, in launch order
    // (marked launched), {kLate} if p's bucket was already launched, {} otherwise.
    std::vector<int> mark(int p);
    // End of backward: every bucket not launched yet, in launch order (marked launched).
    std::vector<int> flush();
    // Begin a step: pending counts from the expected fires (1 per bucket while learning).
    void reset();
    // Adopt the fires of the step just finished as the expected counts (end of the first step).
    void learn();
    bool learned() const;
    bool launched(int bucket) const;
    std::vector<int> fires() const;
    std::vector<int> expected() const;

    OrderedScheduler &scheduler() { return sched_; }

  private:
    mutable std::mutex mu_;
    OrderedScheduler sched_;
    std::vector<int> bucket_of_;
    std::vector<int> expected_;  // per parameter (empty until learned)
    std::vector<int> fires_;     // per parameter, this step
    std::vector<int> pending_;   // per bucket
    std::vector<char> launched_; // per bucket
};

}  // namespace kungfu
