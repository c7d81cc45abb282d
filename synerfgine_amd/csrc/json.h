// json.h -- minimal JSON / msgpack value tree for scene files and .ingp snapshots.
// (The reference uses nlohmann::json; only the subset its scene JSON and
// snapshot reader need is implemented: engine.cu:21-228, testbed.cu:236-270.)
#pragma once
#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace sng {

struct JValue {
    enum Type { Null, Bool, Number, String, Array, Object, Binary } type = Null;
    bool b = false;
    double num = 0.0;
    std::string str;   // String or Binary payload
    std::vector<JValue> arr;
    std::vector<std::pair<std::string, JValue>> obj;

    bool is_number() const { return type == Number || type == Bool; }
    bool contains(const std::string& k) const {
        if (type != Object) return false;
        for (auto& kv : obj) if (kv.first == k) return true;
        return false;
    }
    const JValue& operator[](const std::string& k) const {
        if (type == Object)
            for (auto& kv : obj) if (kv.first == k) return kv.second;
        throw std::runtime_error("json: missing key '" + k + "'");
    }
    const JValue& operator[](size_t i) const {
        if (type != Array || i >= arr.size()) throw std::runtime_error("json: bad array index");
        return arr[i];
    }
    size_t size() const { return type == Array ? arr.size() : (type == Object ? obj.size() : 0); }
    double as_num() const {
        if (type == Number) return num;
        if (type == Bool) return b ? 1.0 : 0.0;
        throw std::runtime_error("json: value is not a number");
    }
    float as_float() const { return (float)as_num(); }
    bool as_bool() const {
        if (type == Bool) return b;
        if (type == Number) return num != 0.0;
        throw std::runtime_error("json: value is not a bool");
    }
    const std::string& as_str() const {
        if (type != String) throw std::runtime_error("json: value is not a string");
        return str;
    }
};

class JsonParser {
public:
    explicit JsonParser(const std::string& s) : s_(s) {}
    JValue parse() {
        JValue v = value();
        ws();
        if (i_ != s_.size()) fail("trailing characters");
        return v;
    }

private:
    const std::string& s_;
    size_t i_ = 0;
    [[noreturn]] void fail(const char* m) { throw std::runtime_error(std::string("json parse error: ") + m + " at offset " + std::to_string(i_)); }
    void ws() {
        while (i_ < s_.size()) {
            char c = s_[i_];
            if (c == ' ' || c == '\t' || c == '\n' || c == '\r') { ++i_; continue; }
            if (c == '/' && i_ + 1 < s_.size() && s_[i_ + 1] == '/') { while (i_ < s_.size() && s_[i_] != '\n') ++i_; continue; }
            break;
        }
    }
    JValue value() {
        ws();
        if (i_ >= s_.size()) fail("unexpected end");
        char c = s_[i_];
        JValue v;
        if (c == '{') {
            v.type = JValue::Object;
            ++i_;
            ws();
            if (s_[i_] == '}') { ++i_; return v; }
            while (true) {
                ws();
                if (s_[i_] != '"') fail("expected key");
                std::string k = string_();
                ws();
                if (s_[i_] != ':') fail("expected ':'");
                ++i_;
                JValue x = value();
                v.obj.emplace_back(std::move(k), std::move(x));
                ws();
                if (s_[i_] == ',') { ++i_; continue; }
                if (s_[i_] == '}') { ++i_; break; }
                fail("expected ',' or '}'");
            }
        } else if (c == '[') {
            v.type = JValue::Array;
            ++i_;
            ws();
            if (s_[i_] == ']') { ++i_; return v; }
            while (true) {
                v.arr.push_back(value());
                ws();
                if (s_[i_] == ',') { ++i_; continue; }
                if (s_[i_] == ']') { ++i_; break; }
                fail("expected ',' or ']'");
            }
        } else if (c == '"') {
            v.type = JValue::String;
            v.str = string_();
        } else if (s_.compare(i_, 4, "true") == 0) { v.type = JValue::Bool; v.b = true; i_ += 4; }
        else if (s_.compare(i_, 5, "false") == 0) { v.type = JValue::Bool; v.b = false; i_ += 5; }
        else if (s_.compare(i_, 4, "null") == 0) { i_ += 4; }
        else {
            size_t st = i_;
            while (i_ < s_.size() && (isdigit((unsigned char)s_[i_]) || s_[i_] == '-' || s_[i_] == '+' || s_[i_] == '.' || s_[i_] == 'e' || s_[i_] == 'E')) ++i_;
            if (st == i_) fail("unexpected character");
            v.type = JValue::Number;
            v.num = std::stod(s_.substr(st, i_ - st));
        }
        return v;
    }
    std::string string_() {
        ++i_;
        std::string r;
        while (i_ < s_.size() && s_[i_] != '"') {
            char c = s_[i_++];
            if (c == '\\') {
                char e = s_[i_++];
                switch (e) {
                    case 'n': r += '\n'; break;
                    case 't': r += '\t'; break;
                    case 'r': r += '\r'; break;
                    case 'b': r += '\b'; break;
                    case 'f': r += '\f'; break;
                    case 'u': { unsigned cp = std::stoul(s_.substr(i_, 4), nullptr, 16); i_ += 4; r += (char)(cp < 128 ? cp : '?'); break; }
                    default: r += e;
                }
            } else r += c;
        }
        if (i_ >= s_.size()) fail("unterminated string");
        ++i_;
        return r;
    }
};

// msgpack -> JValue (nlohmann::json::from_msgpack subset: bin/ext -> Binary)
class MsgpackParser {
public:
    MsgpackParser(const uint8_t* p, size_t n) : p_(p), n_(n) {}
    JValue parse() { return value(); }

private:
    const uint8_t* p_;
    size_t n_, i_ = 0;
    uint8_t u8() { if (i_ >= n_) throw std::runtime_error("msgpack: truncated"); return p_[i_++]; }
    uint64_t be(int bytes) { uint64_t v = 0; for (int k = 0; k < bytes; ++k) v = (v << 8) | u8(); return v; }
    std::string raw(size_t len) {
        if (i_ + len > n_) throw std::runtime_error("msgpack: truncated");
        std::string s((const char*)p_ + i_, len);
        i_ += len;
        return s;
    }
    JValue str_(size_t len) { JValue v; v.type = JValue::String; v.str = raw(len); return v; }
    JValue bin_(size_t len) { JValue v; v.type = JValue::Binary; v.str = raw(len); return v; }
    JValue arr_(size_t len) { JValue v; v.type = JValue::Array; for (size_t k = 0; k < len; ++k) v.arr.push_back(value()); return v; }
    JValue map_(size_t len) {
        JValue v; v.type = JValue::Object;
        for (size_t k = 0; k < len; ++k) {
            JValue key = value();
            std::string ks = key.type == JValue::String ? key.str : std::to_string((long long)key.as_num());
            v.obj.emplace_back(ks, value());
        }
        return v;
    }
    JValue num_(double d) { JValue v; v.type = JValue::Number; v.num = d; return v; }
    JValue value() {
        uint8_t c = u8();
        if (c <= 0x7f) return num_(c);
        if (c >= 0xe0) return num_((int8_t)c);
        if ((c & 0xe0) == 0xa0) return str_(c & 0x1f);
        if ((c & 0xf0) == 0x90) return arr_(c & 0x0f);
        if ((c & 0xf0) == 0x80) return map_(c & 0x0f);
        switch (c) {
            case 0xc0: return JValue{};
            case 0xc2: { JValue v; v.type = JValue::Bool; v.b = false; return v; }
            case 0xc3: { JValue v; v.type = JValue::Bool; v.b = true; return v; }
            case 0xc4: return bin_(be(1));
            case 0xc5: return bin_(be(2));
            case 0xc6: return bin_(be(4));
            case 0xc7: { size_t l = be(1); u8(); return bin_(l); }
            case 0xc8: { size_t l = be(2); u8(); return bin_(l); }
            case 0xc9: { size_t l = be(4); u8(); return bin_(l); }
            case 0xca: { uint32_t b = (uint32_t)be(4); float f; std::memcpy(&f, &b, 4); return num_(f); }
            case 0xcb: { uint64_t b = be(8); double d; std::memcpy(&d, &b, 8); return num_(d); }
            case 0xcc: return num_((double)be(1));
            case 0xcd: return num_((double)be(2));
            case 0xce: return num_((double)be(4));
            case 0xcf: return num_((double)be(8));
            case 0xd0: return num_((int8_t)be(1));
            case 0xd1: return num_((int16_t)be(2));
            case 0xd2: return num_((int32_t)be(4));
            case 0xd3: return num_((double)(int64_t)be(8));
            case 0xd4: { u8(); return bin_(1); }
            case 0xd5: { u8(); return bin_(2); }
            case 0xd6: { u8(); return bin_(4); }
            case 0xd7: { u8(); return bin_(8); }
            case 0xd8: { u8(); return bin_(16); }
            case 0xd9: return str_(be(1));
            case 0xda: return str_(be(2));
            case 0xdb: return str_(be(4));
            case 0xdc: return arr_(be(2));
            case 0xdd: return arr_(be(4));
            case 0xde: return map_(be(2));
            case 0xdf: return map_(be(4));
        }
        throw std::runtime_error("msgpack: unsupported type byte");
    }
};

// JValue-free msgpack emitter (nlohmann::json::to_msgpack's encodings: the smallest int/str/bin/map
// form; floats as float32 when exact, else float64), for Testbed::save_snapshot (testbed.cu:4812-4876).
class MsgpackWriter {
public:
    std::vector<uint8_t> out;
    void map(uint32_t n) { if (n < 16) u8(0x80 | n); else if (n < 65536) { u8(0xde); be(n, 2); } else { u8(0xdf); be(n, 4); } }
    void arr(uint32_t n) { if (n < 16) u8(0x90 | n); else if (n < 65536) { u8(0xdc); be(n, 2); } else { u8(0xdd); be(n, 4); } }
    void str(const std::string& v) {
        const size_t n = v.size();
        if (n < 32) u8(0xa0 | (uint8_t)n);
        else if (n < 256) { u8(0xd9); be(n, 1); }
        else if (n < 65536) { u8(0xda); be(n, 2); }
        else { u8(0xdb); be(n, 4); }
        out.insert(out.end(), v.begin(), v.end());
    }
    void bin(const void* p, size_t n) {
        if (n < 256) { u8(0xc4); be(n, 1); }
        else if (n < 65536) { u8(0xc5); be(n, 2); }
        else { u8(0xc6); be(n, 4); }
        const uint8_t* b = static_cast<const uint8_t*>(p);
        out.insert(out.end(), b, b + n);
    }
    void uint(uint64_t v) {
        if (v < 128) u8((uint8_t)v);
        else if (v < 256) { u8(0xcc); be(v, 1); }
        else if (v < 65536) { u8(0xcd); be(v, 2); }
        else if (v <= 0xffffffffull) { u8(0xce); be(v, 4); }
        else { u8(0xcf); be(v, 8); }
    }
    void sint(int64_t v) {
        if (v >= 0) { uint((uint64_t)v); return; }
        if (v >= -32) u8((uint8_t)(int8_t)v);
        else if (v >= -128) { u8(0xd0); be((uint64_t)(uint8_t)(int8_t)v, 1); }
        else if (v >= -32768) { u8(0xd1); be((uint64_t)(uint16_t)(int16_t)v, 2); }
        else if (v >= INT32_MIN) { u8(0xd2); be((uint64_t)(uint32_t)(int32_t)v, 4); }
        else { u8(0xd3); be((uint64_t)v, 8); }
    }
    void num(double v) {
        const float f = (float)v;
        if ((double)f == v) { uint32_t b; std::memcpy(&b, &f, 4); u8(0xca); be(b, 4); }
        else { uint64_t b; std::memcpy(&b, &v, 8); u8(0xcb); be(b, 8); }
    }
    void boolean(bool v) { u8(v ? 0xc3 : 0xc2); }
    void nil() { u8(0xc0); }
    void key(const char* k) { str(k); }
    void nums(const float* v, int n) { arr((uint32_t)n); for (int i = 0; i < n; ++i) num(v[i]); }

private:
    void u8(uint8_t v) { out.push_back(v); }
    void be(uint64_t v, int bytes) { for (int k = bytes - 1; k >= 0; --k) out.push_back((uint8_t)(v >> (8 * k))); }
};

}  // namespace sng
