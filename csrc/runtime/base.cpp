// CPU reduction kernel + dtype/op/strategy tables.  See base.hpp for parity.
#include <kungfu/base.hpp>

#include <algorithm>
#include <type_traits>
#include <cstring>
#include <stdexcept>

#if defined(__AVX2__) || defined(__F16C__)
#include <immintrin.h>
#endif

namespace kungfu {

size_t dtype_size(DType t) {
    switch (t) {
    case DType::U8: case DType::I8: case DType::BOOL: return 1;
    case DType::U16: case DType::I16: case DType::F16: case DType::BF16: return 2;
    case DType::U32: case DType::I32: case DType::F32: return 4;
    case DType::U64: case DType::I64: case DType::F64: return 8;
    }
    return 0;
}

static const char *kDTypeNames[] = {"u8", "u16", "u32", "u64", "i8", "i16", "i32",
                                    "i64", "f16", "bf16", "f32", "f64", "bool"};

const char *dtype_name(DType t) {
    int i = static_cast<int>(t);
    return (i >= 0 && i <= 12) ? kDTypeNames[i] : "?";
}

bool parse_dtype(const std::string &s, DType *t) {
    for (int i = 0; i <= 12; ++i)
        if (s == kDTypeNames[i]) { *t = static_cast<DType>(i); return true; }
    return false;
}

const char *op_name(ReduceOp op) {
    switch (op) {
    case ReduceOp::SUM: return "sum";
    case ReduceOp::MIN: return "min";
    case ReduceOp::MAX: return "max";
    case ReduceOp::PROD: return "prod";
    }
    return "?";
}

bool parse_op(const std::string &s, ReduceOp *op) {
    static const std::pair<const char *, ReduceOp> t[] = {
        {"sum", ReduceOp::SUM}, {"min", ReduceOp::MIN}, {"max", ReduceOp::MAX}, {"prod", ReduceOp::PROD}};
    for (auto &p : t)
        if (s == p.first) { *op = p.second; return true; }
    return false;
}

static const char *kStrategyNames[] = {"STAR", "MULTI_STAR", "RING", "CLIQUE", "TREE",
                                       "BINARY_TREE", "BINARY_TREE_STAR",
                                       "MULTI_BINARY_TREE_STAR", "AUTO"};

const char *strategy_name(Strategy s) {
    int i = static_cast<int>(s);
    return (i >= 0 && i <= 8) ? kStrategyNames[i] : "?";
}

bool parse_strategy(const std::string &s, Strategy *out) {
    for (int i = 0; i <= 8; ++i)
        if (s == kStrategyNames[i]) { *out = static_cast<Strategy>(i); return true; }
    return false;
}

Strategy default_strategy() { return Strategy::BINARY_TREE_STAR; }

std::vector<Strategy> all_strategies() {
    std::vector<Strategy> v;
    for (int i = 0; i <= 8; ++i) v.push_back(static_cast<Strategy>(i));
    return v;
}

// ---- half precision -------------------------------------------------------

uint16_t f32_to_bf16(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    if ((u & 0x7fffffffu) > 0x7f800000u) return static_cast<uint16_t>((u >> 16) | 0x40);  // NaN
    u += 0x7fffu + ((u >> 16) & 1u);
    return static_cast<uint16_t>(u >> 16);
}

float bf16_to_f32(uint16_t h) {
    uint32_t u = static_cast<uint32_t>(h) << 16;
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}

uint16_t f32_to_f16(float f) {
#if defined(__F16C__)
    return _cvtss_sh(f, _MM_FROUND_TO_NEAREST_INT);
#else
    uint32_t x;
    std::memcpy(&x, &f, 4);
    uint32_t sign = (x >> 16) & 0x8000u;
    int32_t exp = static_cast<int32_t>((x >> 23) & 0xff) - 127 + 15;
    uint32_t mant = x & 0x7fffffu;
    if (((x >> 23) & 0xff) == 0xff) return static_cast<uint16_t>(sign | 0x7c00u | (mant ? 0x200u : 0));
    if (exp >= 31) return static_cast<uint16_t>(sign | 0x7c00u);
    if (exp <= 0) {
        if (exp < -10) return static_cast<uint16_t>(sign);
        mant |= 0x800000u;
        uint32_t shift = static_cast<uint32_t>(14 - exp);
        uint32_t h = mant >> shift;
        uint32_t rem = mant & ((1u << shift) - 1), half = 1u << (shift - 1);
        if (rem > half || (rem == half && (h & 1))) ++h;
        return static_cast<uint16_t>(sign | h);
    }
    uint32_t h = sign | (static_cast<uint32_t>(exp) << 10) | (mant >> 13);
    uint32_t rem = mant & 0x1fffu;
    if (rem > 0x1000u || (rem == 0x1000u && (h & 1))) ++h;
    return static_cast<uint16_t>(h);
#endif
}

float f16_to_f32(uint16_t h) {
#if defined(__F16C__)
    return _cvtsh_ss(h);
#else
    uint32_t sign = (h & 0x8000u) << 16;
    uint32_t exp = (h >> 10) & 0x1f, mant = h & 0x3ffu, u;
    if (exp == 0) {
        if (mant == 0) u = sign;
        else {
            exp = 127 - 15 + 1;
            while (!(mant & 0x400u)) { mant <<= 1; --exp; }
            mant &= 0x3ffu;
            u = sign | (exp << 23) | (mant << 13);
        }
    } else if (exp == 31) u = sign | 0x7f800000u | (mant << 13);
    else u = sign | ((exp + 127 - 15) << 23) | (mant << 13);
    float f;
    std::memcpy(&f, &u, 4);
    return f;
#endif
}

// ---- reduction --------------------------------------------------------------

namespace {

template <typename T> struct OpSum { static T ap(T a, T b) { return a + b; } };
template <typename T> struct OpMin { static T ap(T a, T b) { return b < a ? b : a; } };
template <typename T> struct OpMax { static T ap(T a, T b) { return a < b ? b : a; } };
template <typename T> struct OpProd { static T ap(T a, T b) { return a * b; } };

template <typename T, template <typename> class Op>
void apply(T *__restrict z, const T *x, const T *y, size_t n) {
    // Simple loop: -O3 -mavx2 vectorises it when z does not alias (checked by
    // the compiler with a runtime overlap test).
    for (size_t i = 0; i < n; ++i) z[i] = Op<T>::ap(x[i], y[i]);
}

template <typename T>
void apply_op(T *z, const T *x, const T *y, size_t n, ReduceOp op) {
    switch (op) {
    case ReduceOp::SUM: apply<T, OpSum>(z, x, y, n); break;
    case ReduceOp::MIN: apply<T, OpMin>(z, x, y, n); break;
    case ReduceOp::MAX: apply<T, OpMax>(z, x, y, n); break;
    case ReduceOp::PROD: apply<T, OpProd>(z, x, y, n); break;
    }
}

template <template <typename> class Op>
void half_f16(uint16_t *z, const uint16_t *x, const uint16_t *y, size_t n) {
    size_t i = 0;
#if defined(__F16C__) && defined(__AVX__)
    for (; i + 8 <= n; i += 8) {
        __m256 a = _mm256_cvtph_ps(_mm_loadu_si128(reinterpret_cast<const __m128i *>(x + i)));
        __m256 b = _mm256_cvtph_ps(_mm_loadu_si128(reinterpret_cast<const __m128i *>(y + i)));
        __m256 c;
        if (std::is_same<Op<float>, OpSum<float>>::value) c = _mm256_add_ps(a, b);
        else if (std::is_same<Op<float>, OpMin<float>>::value) c = _mm256_min_ps(b, a);
        else if (std::is_same<Op<float>, OpMax<float>>::value) c = _mm256_max_ps(b, a);
        else c = _mm256_mul_ps(a, b);
        _mm_storeu_si128(reinterpret_cast<__m128i *>(z + i), _mm256_cvtps_ph(c, _MM_FROUND_TO_NEAREST_INT));
    }
#endif
    for (; i < n; ++i) z[i] = f32_to_f16(Op<float>::ap(f16_to_f32(x[i]), f16_to_f32(y[i])));
}

template <template <typename> class Op>
void half_bf16(uint16_t *z, const uint16_t *x, const uint16_t *y, size_t n) {
    size_t i = 0;
#if defined(__AVX2__)
    const __m256i rnd = _mm256_set1_epi32(0x7fff);
    const __m256i one = _mm256_set1_epi32(1);
    for (; i + 8 <= n; i += 8) {
        __m256i xa = _mm256_cvtepu16_epi32(_mm_loadu_si128(reinterpret_cast<const __m128i *>(x + i)));
        __m256i ya = _mm256_cvtepu16_epi32(_mm_loadu_si128(reinterpret_cast<const __m128i *>(y + i)));
        __m256 a = _mm256_castsi256_ps(_mm256_slli_epi32(xa, 16));
        __m256 b = _mm256_castsi256_ps(_mm256_slli_epi32(ya, 16));
        __m256 c;
        if (std::is_same<Op<float>, OpSum<float>>::value) c = _mm256_add_ps(a, b);
        else if (std::is_same<Op<float>, OpMin<float>>::value) c = _mm256_min_ps(b, a);
        else if (std::is_same<Op<float>, OpMax<float>>::value) c = _mm256_max_ps(b, a);
        else c = _mm256_mul_ps(a, b);
        __m256i u = _mm256_castps_si256(c);
        // round-to-nearest-even (NaNs are quieted by the scalar tail rule
        // only; vector path keeps the payload's top bits which stay NaN).
        __m256i lsb = _mm256_and_si256(_mm256_srli_epi32(u, 16), one);
        u = _mm256_add_epi32(u, _mm256_add_epi32(rnd, lsb));
        u = _mm256_srli_epi32(u, 16);
        __m128i lo = _mm256_castsi256_si128(u), hi = _mm256_extracti128_si256(u, 1);
        _mm_storeu_si128(reinterpret_cast<__m128i *>(z + i), _mm_packus_epi32(lo, hi));
    }
#endif
    for (; i < n; ++i) z[i] = f32_to_bf16(Op<float>::ap(bf16_to_f32(x[i]), bf16_to_f32(y[i])));
}

template <template <typename> class Op>
void half_dispatch(DType dt, void *z, const void *x, const void *y, size_t n) {
    auto *zz = static_cast<uint16_t *>(z);
    auto *xx = static_cast<const uint16_t *>(x);
    auto *yy = static_cast<const uint16_t *>(y);
    if (dt == DType::F16) half_f16<Op>(zz, xx, yy, n);
    else half_bf16<Op>(zz, xx, yy, n);
}

}  // namespace

void transform2(void *z, const void *x, const void *y, size_t n, DType dt, ReduceOp op) {
    switch (dt) {
#define KF_CASE(D, T) \
    case DType::D: apply_op<T>(static_cast<T *>(z), static_cast<const T *>(x), static_cast<const T *>(y), n, op); return;
        KF_CASE(U8, uint8_t)
        KF_CASE(U16, uint16_t)
        KF_CASE(U32, uint32_t)
        KF_CASE(U64, uint64_t)
        KF_CASE(I8, int8_t)
        KF_CASE(I16, int16_t)
        KF_CASE(I32, int32_t)
        KF_CASE(I64, int64_t)
        KF_CASE(F32, float)
        KF_CASE(F64, double)
#undef KF_CASE
    case DType::BOOL: {
        // bool: SUM/MAX = or, MIN/PROD = and.
        auto *zz = static_cast<uint8_t *>(z);
        auto *xx = static_cast<const uint8_t *>(x);
        auto *yy = static_cast<const uint8_t *>(y);
        bool is_or = (op == ReduceOp::SUM || op == ReduceOp::MAX);
        for (size_t i = 0; i < n; ++i) zz[i] = is_or ? (xx[i] || yy[i]) : (xx[i] && yy[i]);
        return;
    }
    case DType::F16:
    case DType::BF16:
        switch (op) {
        case ReduceOp::SUM: half_dispatch<OpSum>(dt, z, x, y, n); return;
        case ReduceOp::MIN: half_dispatch<OpMin>(dt, z, x, y, n); return;
        case ReduceOp::MAX: half_dispatch<OpMax>(dt, z, x, y, n); return;
        case ReduceOp::PROD: half_dispatch<OpProd>(dt, z, x, y, n); return;
        }
    }
    throw std::invalid_argument("transform2: bad dtype");
}

// ---- partition / workspace ---------------------------------------------------

std::vector<Interval> even_partition(size_t n, size_t k) {
    std::vector<Interval> out;
    if (k == 0) return out;
    size_t q = n / k, r = n % k, off = 0;
    for (size_t i = 0; i < k; ++i) {
        size_t len = q + (i < r ? 1 : 0);
        out.push_back({off, off + len});
        off += len;
    }
    return out;
}

void Workspace::forward() const {
    if (!inplace() && count > 0) std::memmove(recv, send, bytes());
}

std::vector<Workspace> Workspace::split(size_t k) const {
    std::vector<Workspace> out;
    size_t es = dtype_size(dtype);
    auto parts = even_partition(count, k);
    for (size_t i = 0; i < parts.size(); ++i) {
        Workspace w = *this;
        w.send = static_cast<const char *>(send) + parts[i].begin * es;
        w.recv = static_cast<char *>(recv) + parts[i].begin * es;
        w.count = parts[i].len();
        if (k > 1) w.name = name + "#" + std::to_string(i);
        out.push_back(w);
    }
    return out;
}

}  // namespace kungfu
