// Model-averaging engine over the peer's one-sided P2P store: peer selection,
// model save, synchronous and prefetching (asynchronous) pull-and-average.
//
// Parity: the reference's legacy fused-model pair-averaging TF ops
//   ModelAveraging / AsyncModelAveraging / SaveModel / RequestModel /
//   AsyncRequestModel and the random / round-robin SelectionStrategy
//   (srcs/cpp/src/tensorflow/ops/cpu/peer_to_peer.cpp:8-523) and the
//   ModelBuffer (srcs/cpp/include/kungfu/tensorflow/model_buffer.hpp:13-53).
//
// Here the "model" is one contiguous f32 buffer (the flat parameter space of
// kungfu_amd), so the buffer never needs per-variable copy loops: averaging is
// one AVX pass v = (v + peer) / 2 and the store entry is the buffer itself.
#pragma once

#include <kungfu/peer.hpp>

#include <atomic>
#include <cstdint>
#include <memory>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <vector>

namespace kungfu {

class PeerSelector {
  public:
    // kind: "random" (uniform over ranks) or "roundrobin"
    PeerSelector(const std::string &kind, std::vector<int> ranks, uint64_t seed);
    int next();
    const std::vector<int> &ranks() const { return ranks_; }

  private:
    bool random_;
    std::vector<int> ranks_;
    size_t t_ = 0;
    std::mt19937_64 rng_;
};

class ModelAverager {
  public:
    // count: number of f32 elements of the model; name: store key.
    ModelAverager(Peer *peer, size_t count, const std::string &name, const std::string &selection);
    ~ModelAverager();

    // Put the model into the local store (other peers pull it).
    void save(const float *model);
    // Pull a selected peer's model into out; returns the peer rank or -1 if it had none.
    int request(float *out);
    // Synchronous pair averaging: model = (model + peer_model) / 2.  Returns the peer or -1.
    int average(float *model);
    // Prefetching variant: averages with the most recently completed pull (the first call
    // pulls synchronously) and starts the next pull in the background if none is in flight.
    int async_average(float *model);
    // Waits for an in-flight background pull.
    void wait();

    size_t count() const { return count_; }
    int64_t pulls() const { return pulls_.load(); }

  private:
    void start_prefetch();

    Peer *peer_;
    size_t count_;
    std::string name_;
    PeerSelector sel_;
    std::mutex mu_;  // guards model_buf_ / have_model_ / sel_
    std::vector<float> model_buf_, prefetch_buf_;
    bool have_model_ = false;
    int last_peer_ = -1;
    std::atomic<bool> requesting_{false};
    std::thread worker_;
    std::atomic<int64_t> pulls_{0};
};

// dst = (a + b) / 2 over n floats (AVX2).
void average_f32(float *dst, const float *a, const float *b, size_t n);

}  // namespace kungfu
