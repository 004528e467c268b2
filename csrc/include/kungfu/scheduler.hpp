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

}  // namespace kungfu
