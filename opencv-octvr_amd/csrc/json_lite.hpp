// json_lite.hpp — minimal JSON reader for rig configs (the reference uses vendored rapidjson:
// modules/octvr/include/rapidjson, parsed in apps/octvr/dump.cpp:71-74).  Supports the subset the
// rig schema needs: objects, arrays, numbers, strings, true/false/null.  Throws std::runtime_error.
#pragma once

#include <locale.h>

#include <cerrno>
#include <charconv>
#include <cstdint>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace octvr {

struct JsonValue {
    enum Kind { Null, Bool, Number, String, Array, Object } kind = Null;
    bool b = false;
    double num = 0;
    std::string str;
    std::vector<JsonValue> arr;
    std::vector<std::pair<std::string, JsonValue>> obj;  // insertion order kept

    bool has(const std::string& k) const {
        if (kind != Object) return false;
        for (auto& kv : obj)
            if (kv.first == k) return true;
        return false;
    }
    const JsonValue& operator[](const std::string& k) const {
        if (kind != Object) throw std::runtime_error("json: not an object when looking up '" + k + "'");
        for (auto& kv : obj)
            if (kv.first == k) return kv.second;
        throw std::runtime_error("json: missing member '" + k + "'");
    }
    const JsonValue& operator[](size_t i) const {
        if (kind != Array || i >= arr.size()) throw std::runtime_error("json: bad array index");
        return arr[i];
    }
    size_t size() const { return kind == Array ? arr.size() : obj.size(); }
    double as_double() const {
        if (kind != Number) throw std::runtime_error("json: expected a number");
        return num;
    }
    int as_int() const { return (int)as_double(); }
    bool as_bool() const {
        if (kind != Bool) throw std::runtime_error("json: expected a bool");
        return b;
    }
    const std::string& as_string() const {
        if (kind != String) throw std::runtime_error("json: expected a string");
        return str;
    }
    double get(const std::string& k, double dflt) const { return has(k) ? (*this)[k].as_double() : dflt; }
};

class JsonParser {
public:
    // exact: numbers correctly rounded (strtod) instead of rapidjson's rules — for text written from
    // doubles with 17 significant digits (the C++ API's rapidjson::Value overloads, OCTVR_JSON_EXACT)
    explicit JsonParser(const std::string& s, bool exact = false) : s_(s), i_(0), exact_(exact) {}
    JsonValue parse() {
        JsonValue v = value();
        ws();
        if (i_ != s_.size()) fail("trailing characters");
        return v;
    }

private:
    const std::string& s_;
    size_t i_;
    bool exact_;

    [[noreturn]] void fail(const char* what) {
        throw std::runtime_error(std::string("json parse error: ") + what + " at offset " + std::to_string(i_));
    }
    void ws() {
        while (i_ < s_.size() && (s_[i_] == ' ' || s_[i_] == '\n' || s_[i_] == '\r' || s_[i_] == '\t')) i_++;
    }
    bool lit(const char* t) {
        size_t n = strlen(t);
        if (s_.compare(i_, n, t) == 0) {
            i_ += n;
            return true;
        }
        return false;
    }
    JsonValue value() {
        ws();
        if (i_ >= s_.size()) fail("unexpected end");
        char c = s_[i_];
        JsonValue v;
        if (c == '{') {
            v.kind = JsonValue::Object;
            i_++;
            ws();
            if (i_ < s_.size() && s_[i_] == '}') { i_++; return v; }
            while (true) {
                ws();
                if (i_ >= s_.size() || s_[i_] != '"') fail("expected key");
                std::string k = string_lit();
                ws();
                if (i_ >= s_.size() || s_[i_] != ':') fail("expected ':'");
                i_++;
                v.obj.emplace_back(k, value());
                ws();
                if (i_ < s_.size() && s_[i_] == ',') { i_++; continue; }
                if (i_ < s_.size() && s_[i_] == '}') { i_++; break; }
                fail("expected ',' or '}'");
            }
        } else if (c == '[') {
            v.kind = JsonValue::Array;
            i_++;
            ws();
            if (i_ < s_.size() && s_[i_] == ']') { i_++; return v; }
            while (true) {
                v.arr.push_back(value());
                ws();
                if (i_ < s_.size() && s_[i_] == ',') { i_++; continue; }
                if (i_ < s_.size() && s_[i_] == ']') { i_++; break; }
                fail("expected ',' or ']'");
            }
        } else if (c == '"') {
            v.kind = JsonValue::String;
            v.str = string_lit();
        } else if (lit("true")) {
            v.kind = JsonValue::Bool;
            v.b = true;
        } else if (lit("false")) {
            v.kind = JsonValue::Bool;
        } else if (lit("null")) {
            v.kind = JsonValue::Null;
        } else {
            v.kind = JsonValue::Number;
            if (exact_) {  // std::from_chars: correctly rounded and locale-independent (strtod reads the
                           // C library's LC_NUMERIC radix: "1,5" under a comma locale)
                const char* b = s_.data() + i_;
                const char* e = s_.data() + s_.size();
                if (b < e && *b == '-' && b + 1 < e && !(b[1] >= '0' && b[1] <= '9')) fail("bad number");
                if (b < e && !(*b == '-' || (*b >= '0' && *b <= '9'))) fail("bad number");
                double x = 0.0;
                const std::from_chars_result r = std::from_chars(b, e, x, std::chars_format::general);
                if (r.ptr == b || (r.ec != std::errc() && r.ec != std::errc::result_out_of_range)) fail("bad number");
                if (r.ec == std::errc::result_out_of_range) {
                    // overflow (1e400) or underflow (subnormals on some libstdc++ versions): the value the
                    // previous strtod path gave — +-HUGE_VAL, the subnormal, or 0 — read in the C locale
                    static const locale_t c_loc = newlocale(LC_NUMERIC_MASK, "C", (locale_t)0);
                    const std::string tok(b, r.ptr);
                    x = c_loc ? strtod_l(tok.c_str(), nullptr, c_loc) : 0.0;
                }
                v.num = x;
                i_ += (size_t)(r.ptr - b);
            } else {
                v.num = number();
            }
        }
        return v;
    }
    // rapidjson 1.0.2 reader.h:1090-1276 with default flags (StrtodNormalPrecision, strtod.h:26-44): the
    // significand is gathered in a uint64 (fraction digits only while it is <= 2^53-1), converted to
    // double and scaled by one multiply/divide with an exact power of ten — NOT always correctly
    // rounded, and reproduced here so configs parse to the same doubles as in the reference.
    double number() {
        auto peek_digit = [&]() { return i_ < s_.size() && s_[i_] >= '0' && s_[i_] <= '9'; };
        bool minus = false;
        if (i_ < s_.size() && s_[i_] == '-') { minus = true; i_++; }
        unsigned i = 0;
        uint64_t i64 = 0;
        bool use64bit = false;
        int significandDigit = 0;
        if (i_ < s_.size() && s_[i_] == '0') {
            i = 0;
            i_++;
        } else if (peek_digit()) {
            i = (unsigned)(s_[i_++] - '0');
            const unsigned lim = minus ? 214748364u : 429496729u;
            const char lastd = minus ? '8' : '5';
            while (peek_digit()) {
                if (i >= lim && (i != lim || s_[i_] > lastd)) { i64 = i; use64bit = true; break; }
                i = i * 10 + (unsigned)(s_[i_++] - '0');
                significandDigit++;
            }
        } else {
            fail("bad value");
        }
        bool useDouble = false;
        double d = 0.0;
        if (use64bit) {
            const uint64_t lim = minus ? 0x0CCCCCCCCCCCCCCCULL : 0x1999999999999999ULL;
            const char lastd = minus ? '8' : '5';
            while (peek_digit()) {
                if (i64 >= lim && (i64 != lim || s_[i_] > lastd)) { d = (double)i64; useDouble = true; break; }
                i64 = i64 * 10 + (unsigned)(s_[i_++] - '0');
                significandDigit++;
            }
        }
        if (useDouble)
            while (peek_digit()) d = d * 10 + (s_[i_++] - '0');
        int expFrac = 0;
        if (i_ < s_.size() && s_[i_] == '.') {
            i_++;
            if (!peek_digit()) fail("missing fraction");
            if (!useDouble) {
                if (!use64bit) i64 = i;
                while (peek_digit()) {
                    if (i64 > 0x1FFFFFFFFFFFFFULL) break;
                    i64 = i64 * 10 + (unsigned)(s_[i_++] - '0');
                    --expFrac;
                    if (i64 != 0) significandDigit++;
                }
                d = (double)i64;
                useDouble = true;
            }
            while (peek_digit()) {
                if (significandDigit < 17) {
                    d = d * 10.0 + (s_[i_++] - '0');
                    --expFrac;
                    if (d > 0.0) significandDigit++;
                } else {
                    i_++;
                }
            }
        }
        int exp = 0;
        if (i_ < s_.size() && (s_[i_] == 'e' || s_[i_] == 'E')) {
            i_++;
            if (!useDouble) { d = (double)(use64bit ? i64 : i); useDouble = true; }
            bool expMinus = false;
            if (i_ < s_.size() && s_[i_] == '+') i_++;
            else if (i_ < s_.size() && s_[i_] == '-') { expMinus = true; i_++; }
            if (!peek_digit()) fail("missing exponent");
            exp = s_[i_++] - '0';
            while (peek_digit()) {
                exp = exp * 10 + (s_[i_++] - '0');
                if (exp > 100000) fail("exponent too large");
            }
            if (expMinus) exp = -exp;
        }
        if (useDouble) {
            int p = exp + expFrac;
            auto pow10 = [](int n) { double r = 1.0; static const double t[] = {1e0, 1e1, 1e2, 1e3, 1e4, 1e5, 1e6, 1e7, 1e8, 1e9, 1e10, 1e11, 1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22}; if (n <= 22) return t[n]; char buf[16]; const int k = snprintf(buf, sizeof buf, "1e%d", n); std::from_chars(buf, buf + k, r); return r; };
            auto fast = [&](double sig, int e) { return e < -308 ? 0.0 : e >= 0 ? sig * pow10(e) : sig / pow10(-e); };
            if (p < -308) { d = fast(d, -308); d = fast(d, p + 308); }
            else d = fast(d, p);
            return minus ? -d : d;
        }
        if (use64bit) return minus ? (double)(int64_t)(~i64 + 1) : (double)i64;
        return minus ? (double)(int32_t)(~i + 1) : (double)i;
    }
    std::string string_lit() {
        std::string out;
        i_++;  // opening quote
        while (i_ < s_.size() && s_[i_] != '"') {
            char c = s_[i_++];
            if (c == '\\') {
                if (i_ >= s_.size()) fail("bad escape");
                char e = s_[i_++];
                switch (e) {
                    case 'n': out += '\n'; break;
                    case 't': out += '\t'; break;
                    case 'r': out += '\r'; break;
                    case 'b': out += '\b'; break;
                    case 'f': out += '\f'; break;
                    case 'u': {
                        if (i_ + 4 > s_.size()) fail("bad \\u");
                        unsigned cp = (unsigned)strtoul(s_.substr(i_, 4).c_str(), nullptr, 16);
                        i_ += 4;
                        if (cp < 0x80) out += (char)cp;
                        else if (cp < 0x800) { out += (char)(0xC0 | (cp >> 6)); out += (char)(0x80 | (cp & 0x3F)); }
                        else { out += (char)(0xE0 | (cp >> 12)); out += (char)(0x80 | ((cp >> 6) & 0x3F)); out += (char)(0x80 | (cp & 0x3F)); }
                        break;
                    }
                    default: out += e;
                }
            } else {
                out += c;
            }
        }
        if (i_ >= s_.size()) fail("unterminated string");
        i_++;
        return out;
    }
};

inline JsonValue json_parse(const std::string& s, bool exact = false) { return JsonParser(s, exact).parse(); }

}  // namespace octvr
