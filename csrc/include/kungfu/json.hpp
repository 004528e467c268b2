// Minimal JSON value + parser/serializer for the control plane (cluster specs,
// config-server bodies, runner stages, monitor dumps).  Header-only.
#pragma once

#include <cctype>
#include <cstdint>
#include <cstdio>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace kungfu {
namespace json {

struct Value {
    enum Kind { NUL, BOOL, NUM, STR, ARR, OBJ } kind = NUL;
    bool b = false;
    double n = 0;
    std::string s;
    std::vector<Value> a;
    std::vector<std::pair<std::string, Value>> o;  // insertion-ordered

    Value() = default;
    static Value null() { return Value(); }
    static Value boolean(bool v) { Value x; x.kind = BOOL; x.b = v; return x; }
    static Value number(double v) { Value x; x.kind = NUM; x.n = v; return x; }
    static Value string(const std::string &v) { Value x; x.kind = STR; x.s = v; return x; }
    static Value array() { Value x; x.kind = ARR; return x; }
    static Value object() { Value x; x.kind = OBJ; return x; }

    Value &push(const Value &v) { a.push_back(v); return a.back(); }
    Value &set(const std::string &k, const Value &v) {
        for (auto &kv : o)
            if (kv.first == k) { kv.second = v; return kv.second; }
        o.emplace_back(k, v);
        return o.back().second;
    }
    const Value *get(const std::string &k) const {
        for (auto &kv : o)
            if (kv.first == k) return &kv.second;
        return nullptr;
    }
    const Value &at(const std::string &k) const {
        auto *v = get(k);
        if (!v) throw std::runtime_error("json: missing key " + k);
        return *v;
    }
    int64_t as_int() const { return static_cast<int64_t>(n); }
};

inline void escape(const std::string &s, std::string &out) {
    out.push_back('"');
    for (char c : s) {
        switch (c) {
        case '"': out += "\\\""; break;
        case '\\': out += "\\\\"; break;
        case '\n': out += "\\n"; break;
        case '\t': out += "\\t"; break;
        case '\r': out += "\\r"; break;
        default:
            if (static_cast<unsigned char>(c) < 0x20) {
                char buf[8];
                std::snprintf(buf, sizeof(buf), "\\u%04x", c);
                out += buf;
            } else out.push_back(c);
        }
    }
    out.push_back('"');
}

inline void dump(const Value &v, std::string &out) {
    switch (v.kind) {
    case Value::NUL: out += "null"; break;
    case Value::BOOL: out += v.b ? "true" : "false"; break;
    case Value::NUM: {
        char buf[64];
        if (v.n == static_cast<double>(static_cast<int64_t>(v.n)))
            std::snprintf(buf, sizeof(buf), "%lld", static_cast<long long>(v.n));
        else std::snprintf(buf, sizeof(buf), "%.17g", v.n);
        out += buf;
        break;
    }
    case Value::STR: escape(v.s, out); break;
    case Value::ARR:
        out.push_back('[');
        for (size_t i = 0; i < v.a.size(); ++i) {
            if (i) out.push_back(',');
            dump(v.a[i], out);
        }
        out.push_back(']');
        break;
    case Value::OBJ:
        out.push_back('{');
        for (size_t i = 0; i < v.o.size(); ++i) {
            if (i) out.push_back(',');
            escape(v.o[i].first, out);
            out.push_back(':');
            dump(v.o[i].second, out);
        }
        out.push_back('}');
        break;
    }
}

inline std::string dump(const Value &v) {
    std::string s;
    dump(v, s);
    return s;
}

class Parser {
  public:
    explicit Parser(const std::string &s) : s_(s) {}
    Value parse() {
        Value v = value();
        ws();
        if (i_ != s_.size()) fail("trailing characters");
        return v;
    }

  private:
    const std::string &s_;
    size_t i_ = 0;

    [[noreturn]] void fail(const char *m) { throw std::runtime_error(std::string("json: ") + m); }
    void ws() {
        while (i_ < s_.size() && std::isspace(static_cast<unsigned char>(s_[i_]))) ++i_;
    }
    bool lit(const char *w) {
        size_t n = std::char_traits<char>::length(w);
        if (s_.compare(i_, n, w) == 0) { i_ += n; return true; }
        return false;
    }
    Value value() {
        ws();
        if (i_ >= s_.size()) fail("unexpected end");
        char c = s_[i_];
        if (c == '{') return object();
        if (c == '[') return array();
        if (c == '"') return Value::string(str());
        if (lit("true")) return Value::boolean(true);
        if (lit("false")) return Value::boolean(false);
        if (lit("null")) return Value::null();
        return number();
    }
    std::string str() {
        if (s_[i_] != '"') fail("expected string");
        ++i_;
        std::string out;
        while (i_ < s_.size() && s_[i_] != '"') {
            char c = s_[i_++];
            if (c == '\\') {
                if (i_ >= s_.size()) fail("bad escape");
                char e = s_[i_++];
                switch (e) {
                case 'n': out.push_back('\n'); break;
                case 't': out.push_back('\t'); break;
                case 'r': out.push_back('\r'); break;
                case 'b': out.push_back('\b'); break;
                case 'f': out.push_back('\f'); break;
                case 'u': {
                    if (i_ + 4 > s_.size()) fail("bad \\u");
                    unsigned cp = std::stoul(s_.substr(i_, 4), nullptr, 16);
                    i_ += 4;
                    if (cp < 0x80) out.push_back(static_cast<char>(cp));
                    else if (cp < 0x800) {
                        out.push_back(static_cast<char>(0xc0 | (cp >> 6)));
                        out.push_back(static_cast<char>(0x80 | (cp & 0x3f)));
                    } else {
                        out.push_back(static_cast<char>(0xe0 | (cp >> 12)));
                        out.push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3f)));
                        out.push_back(static_cast<char>(0x80 | (cp & 0x3f)));
                    }
                    break;
                }
                default: out.push_back(e);
                }
            } else out.push_back(c);
        }
        if (i_ >= s_.size()) fail("unterminated string");
        ++i_;
        return out;
    }
    Value number() {
        size_t st = i_;
        if (s_[i_] == '-' || s_[i_] == '+') ++i_;
        while (i_ < s_.size() && (std::isdigit(static_cast<unsigned char>(s_[i_])) || s_[i_] == '.' ||
                                  s_[i_] == 'e' || s_[i_] == 'E' || s_[i_] == '-' || s_[i_] == '+'))
            ++i_;
        if (st == i_) fail("unexpected character");
        return Value::number(std::stod(s_.substr(st, i_ - st)));
    }
    Value array() {
        ++i_;
        Value v = Value::array();
        ws();
        if (i_ < s_.size() && s_[i_] == ']') { ++i_; return v; }
        for (;;) {
            v.a.push_back(value());
            ws();
            if (i_ >= s_.size()) fail("unterminated array");
            if (s_[i_] == ',') { ++i_; continue; }
            if (s_[i_] == ']') { ++i_; return v; }
            fail("expected , or ]");
        }
    }
    Value object() {
        ++i_;
        Value v = Value::object();
        ws();
        if (i_ < s_.size() && s_[i_] == '}') { ++i_; return v; }
        for (;;) {
            ws();
            std::string k = str();
            ws();
            if (i_ >= s_.size() || s_[i_] != ':') fail("expected :");
            ++i_;
            v.o.emplace_back(k, value());
            ws();
            if (i_ >= s_.size()) fail("unterminated object");
            if (s_[i_] == ',') { ++i_; continue; }
            if (s_[i_] == '}') { ++i_; return v; }
            fail("expected , or }");
        }
    }
};

inline Value parse(const std::string &s) { return Parser(s).parse(); }

}  // namespace json
}  // namespace kungfu
