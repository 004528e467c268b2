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

}  // namespace kungfu
