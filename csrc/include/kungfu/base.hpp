// Base types of the kungfu-amd host runtime: dtypes, reduce ops, strategies,
// workspaces and the CPU reduction kernel.
//
// Parity map (reference paths relative to /root/reference):
//   DType codes       srcs/cpp/include/kungfu/dtype.h:21-39, srcs/go/kungfu/base/dtype.go:6-46
//   ReduceOp          srcs/cpp/include/kungfu/op.h:8-19
//   transform2        srcs/go/kungfu/base/op.cpp:22-93 (+ f16 AVX path f16.c:16-50)
//   Strategy          srcs/cpp/include/kungfu/strategy.h:7-17, srcs/go/kungfu/base/strategy.go
//   Workspace/Split   srcs/go/kungfu/base/workspace.go:10-50
//
// Differences by design: bf16 is a first-class dtype (the reference mis-maps
// it to f16), f16 and bf16 reductions accumulate in f32, and all dtypes x ops
// are supported (the reference only reduces f16 with SUM).
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>
#include <utility>
#include <vector>

namespace kungfu {

enum class DType : int32_t {
    U8 = 0, U16 = 1, U32 = 2, U64 = 3,
    I8 = 4, I16 = 5, I32 = 6, I64 = 7,
    F16 = 8, BF16 = 9, F32 = 10, F64 = 11,
    BOOL = 12,
};

enum class ReduceOp : int32_t { SUM = 0, MIN = 1, MAX = 2, PROD = 3 };

enum class Strategy : int32_t {
    STAR = 0,
    MULTI_STAR = 1,
    RING = 2,
    CLIQUE = 3,
    TREE = 4,
    BINARY_TREE = 5,
    BINARY_TREE_STAR = 6,
    MULTI_BINARY_TREE_STAR = 7,
    AUTO = 8,
};

size_t dtype_size(DType t);
const char *dtype_name(DType t);
bool parse_dtype(const std::string &s, DType *t);

const char *op_name(ReduceOp op);
bool parse_op(const std::string &s, ReduceOp *op);

const char *strategy_name(Strategy s);
bool parse_strategy(const std::string &s, Strategy *out);
Strategy default_strategy();  // BINARY_TREE_STAR (reference default)
std::vector<Strategy> all_strategies();

// z[i] = op(x[i], y[i]) for i < n.  z may alias x or y.  Vectorised (AVX2/F16C
// where compiled in); f16/bf16 computed in f32 and rounded to nearest-even.
void transform2(void *z, const void *x, const void *y, size_t n, DType dt, ReduceOp op);

// Half-precision helpers (host).
uint16_t f32_to_f16(float f);
float f16_to_f32(uint16_t h);
uint16_t f32_to_bf16(float f);
float bf16_to_f32(uint16_t h);

// Half-open element interval [begin, end).
struct Interval {
    size_t begin = 0, end = 0;
    size_t len() const { return end - begin; }
};

// Split [0, n) into k near-equal parts (first n%k parts get one more).
std::vector<Interval> even_partition(size_t n, size_t k);

// A (possibly in-place) buffer pair for one collective call.
struct Workspace {
    const void *send = nullptr;
    void *recv = nullptr;
    size_t count = 0;
    DType dtype = DType::U8;
    ReduceOp op = ReduceOp::SUM;
    std::string name;

    size_t bytes() const { return count * dtype_size(dtype); }
    bool empty() const { return count == 0; }
    bool inplace() const { return send == recv; }
    // Copy send -> recv (no-op when in-place).
    void forward() const;
    // Chunk i of k: element range given by even_partition; name gets a suffix.
    std::vector<Workspace> split(size_t k) const;
};

}  // namespace kungfu
