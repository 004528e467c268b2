// Model-averaging engine (see kungfu/model_avg.hpp).
#include <kungfu/log.hpp>
#include <kungfu/model_avg.hpp>

#include <immintrin.h>

#include <stdexcept>

namespace kungfu {

PeerSelector::PeerSelector(const std::string &kind, std::vector<int> ranks, uint64_t seed)
    : ranks_(std::move(ranks)), rng_(seed) {
    if (kind == "random") random_ = true;
    else if (kind == "roundrobin" || kind == "round_robin") random_ = false;
    else throw std::invalid_argument("unsupported peer selection strategy: " + kind);
}

int PeerSelector::next() {
    if (ranks_.empty()) return -1;
    if (random_) return ranks_[std::uniform_int_distribution<size_t>(0, ranks_.size() - 1)(rng_)];
    int r = ranks_[t_];
    t_ = (t_ + 1) % ranks_.size();
    return r;
}

void average_f32(float *dst, const float *a, const float *b, size_t n) {
    size_t i = 0;
    const __m256 half = _mm256_set1_ps(0.5f);
    for (; i + 8 <= n; i += 8)
        _mm256_storeu_ps(dst + i, _mm256_mul_ps(_mm256_add_ps(_mm256_loadu_ps(a + i), _mm256_loadu_ps(b + i)), half));
    for (; i < n; ++i) dst[i] = 0.5f * (a[i] + b[i]);
}

namespace {
std::vector<int> others(Peer &p) {
    auto s = p.session();
    std::vector<int> r;
    if (!s) return r;
    for (int i = 0; i < s->size(); ++i)
        if (i != s->rank()) r.push_back(i);
    return r;
}
}  // namespace

ModelAverager::ModelAverager(Peer *peer, size_t count, const std::string &name, const std::string &selection)
    : peer_(peer), count_(count), name_(name),
      sel_(selection, others(*peer), static_cast<uint64_t>(peer->uid())), model_buf_(count), prefetch_buf_(count) {}

ModelAverager::~ModelAverager() { wait(); }

void ModelAverager::save(const float *model) { peer_->save(name_, model, count_ * sizeof(float)); }

int ModelAverager::request(float *out) {
    int target;
    {
        std::lock_guard<std::mutex> l(mu_);
        target = sel_.next();
    }
    if (target < 0) return -1;
    if (!peer_->request(target, "", name_, out, count_ * sizeof(float))) return -1;
    pulls_.fetch_add(1);
    return target;
}

int ModelAverager::average(float *model) {
    int t = request(model_buf_.data());
    if (t < 0) return -1;
    average_f32(model, model, model_buf_.data(), count_);
    return t;
}

void ModelAverager::start_prefetch() {
    bool expect = false;
    if (!requesting_.compare_exchange_strong(expect, true)) return;
    if (worker_.joinable()) worker_.join();
    worker_ = std::thread([this] {
        TraceScope ts("ModelAverager::prefetch");
        int t = request(prefetch_buf_.data());
        if (t >= 0) {
            std::lock_guard<std::mutex> l(mu_);
            model_buf_.swap(prefetch_buf_);
            have_model_ = true;
            last_peer_ = t;
        }
        requesting_.store(false);
    });
}

int ModelAverager::async_average(float *model) {
    bool have;
    {
        std::lock_guard<std::mutex> l(mu_);
        have = have_model_;
    }
    if (!have) {  // first call: one synchronous pull so there is something to average with
        wait();
        int t = request(model_buf_.data());
        std::lock_guard<std::mutex> l(mu_);
        if (t >= 0) {
            have_model_ = true;
            last_peer_ = t;
        }
    }
    start_prefetch();
    std::lock_guard<std::mutex> l(mu_);
    if (!have_model_) return -1;
    average_f32(model, model, model_buf_.data(), count_);
    return last_peer_;
}

void ModelAverager::wait() {
    if (worker_.joinable()) worker_.join();
}

}  // namespace kungfu
