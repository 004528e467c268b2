// Ordered collective scheduler (see kungfu/scheduler.hpp).
#include <kungfu/scheduler.hpp>

#include <algorithm>
#include <stdexcept>

namespace kungfu {

OrderedScheduler::OrderedScheduler(int n) : n_(n), order_(n), ready_(n, 0), done_(n, 0) {
    if (n < 0) throw std::invalid_argument("OrderedScheduler: negative size");
    for (int i = 0; i < n; ++i) order_[i] = i;
}

void OrderedScheduler::reset() {
    std::lock_guard<std::mutex> l(mu_);
    std::fill(ready_.begin(), ready_.end(), 0);
    std::fill(done_.begin(), done_.end(), 0);
    arrivals_.clear();
    next_ = 0;
}

std::vector<int> OrderedScheduler::ready(int i) {
    std::lock_guard<std::mutex> l(mu_);
    if (i < 0 || i >= n_) throw std::out_of_range("OrderedScheduler::ready: bad op id");
    std::vector<int> go;
    if (ready_[i]) return go;
    ready_[i] = 1;
    arrivals_.push_back(i);
    while (next_ < order_.size() && ready_[order_[next_]]) {
        int op = order_[next_++];
        done_[op] = 1;
        go.push_back(op);
    }
    return go;
}

std::vector<int> OrderedScheduler::flush() {
    std::lock_guard<std::mutex> l(mu_);
    std::vector<int> go;
    for (; next_ < order_.size(); ++next_) {
        int op = order_[next_];
        if (!done_[op]) {
            done_[op] = 1;
            go.push_back(op);
        }
    }
    return go;
}

void OrderedScheduler::set_order(const std::vector<int> &order) {
    std::lock_guard<std::mutex> l(mu_);
    std::vector<char> seen(n_, 0);
    std::vector<int> o;
    for (int i : order)
        if (i >= 0 && i < n_ && !seen[i]) {
            seen[i] = 1;
            o.push_back(i);
        }
    for (int i : order_)
        if (!seen[i]) o.push_back(i);  // ops absent from `order` keep their relative order
    order_ = o;
}

void OrderedScheduler::auto_order(Session &s) {
    std::vector<int32_t> buf(n_, -1);
    {
        std::lock_guard<std::mutex> l(mu_);
        for (size_t k = 0; k < arrivals_.size() && k < buf.size(); ++k) buf[k] = arrivals_[k];
    }
    s.broadcast(Workspace{buf.data(), buf.data(), buf.size(), DType::I32, ReduceOp::SUM, "kf:sched:order"});
    set_order(std::vector<int>(buf.begin(), buf.end()));
}

std::vector<int> OrderedScheduler::order() const {
    std::lock_guard<std::mutex> l(mu_);
    return order_;
}

std::vector<int> OrderedScheduler::arrivals() const {
    std::lock_guard<std::mutex> l(mu_);
    return arrivals_;
}

BucketTracker::BucketTracker(int n_buckets, const std::vector<int> &bucket_of)
    : sched_(n_buckets), bucket_of_(bucket_of), fires_(bucket_of.size(), 0), pending_(n_buckets, 1),
      launched_(n_buckets, 0) {
    for (int b : bucket_of_)
        if (b < 0 || b >= n_buckets) throw std::invalid_argument("BucketTracker: bucket index out of range");
}

std::vector<int> BucketTracker::mark(int p) {
    std::lock_guard<std::mutex> l(mu_);
    if (p < 0 || p >= static_cast<int>(bucket_of_.size())) throw std::out_of_range("BucketTracker::mark: bad param");
    ++fires_[p];
    if (expected_.empty()) return {};  // learning step: buckets launch at flush()
    const int b = bucket_of_[p];
    if (launched_[b]) return {kLate};
    if (--pending_[b] > 0) return {};
    std::vector<int> go = sched_.ready(b);
    for (int j : go) launched_[j] = 1;
    return go;
}

std::vector<int> BucketTracker::flush() {
    std::lock_guard<std::mutex> l(mu_);
    std::vector<int> go;
    for (int j : sched_.flush())
        if (!launched_[j]) {
            launched_[j] = 1;
            go.push_back(j);
        }
    return go;
}

void BucketTracker::reset() {
    std::lock_guard<std::mutex> l(mu_);
    std::fill(fires_.begin(), fires_.end(), 0);
    std::fill(launched_.begin(), launched_.end(), 0);
    if (expected_.empty()) {
        std::fill(pending_.begin(), pending_.end(), 1);
    } else {
        std::fill(pending_.begin(), pending_.end(), 0);
        for (size_t p = 0; p < bucket_of_.size(); ++p) pending_[bucket_of_[p]] += expected_[p];
    }
    sched_.reset();
}

void BucketTracker::learn() {
    std::lock_guard<std::mutex> l(mu_);
    expected_ = fires_;
}

bool BucketTracker::learned() const {
    std::lock_guard<std::mutex> l(mu_);
    return !expected_.empty();
}

bool BucketTracker::launched(int bucket) const {
    std::lock_guard<std::mutex> l(mu_);
    return bucket >= 0 && bucket < static_cast<int>(launched_.size()) && launched_[bucket];
}

std::vector<int> BucketTracker::fires() const {
    std::lock_guard<std::mutex> l(mu_);
    return fires_;
}

std::vector<int> BucketTracker::expected() const {
    std::lock_guard<std::mutex> l(mu_);
    return expected_;
}

}  // namespace kungfu
