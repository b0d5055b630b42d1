// Minimal JSON value, parser and serializer for the HTTP API (the reference vendors nlohmann/json,
// src/json.hpp; we only need objects/arrays/strings/numbers/bools with UTF-8 passthrough).
#pragma once

#include <cctype>
#include <cmath>
#include <cstdio>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace dl {
namespace json {

class Value {
  public:
    enum Type { NUL, BOOL, NUMBER, STRING, ARRAY, OBJECT };
    Value() : t_(NUL) {}
    Value(std::nullptr_t) : t_(NUL) {}
    Value(bool b) : t_(BOOL), b_(b) {}
    Value(int v) : t_(NUMBER), n_(v) {}
    Value(long v) : t_(NUMBER), n_((double)v) {}
    Value(long long v) : t_(NUMBER), n_((double)v) {}
    Value(unsigned v) : t_(NUMBER), n_(v) {}
    Value(unsigned long v) : t_(NUMBER), n_((double)v) {}
    Value(unsigned long long v) : t_(NUMBER), n_((double)v) {}
    Value(double v) : t_(NUMBER), n_(v) {}
    Value(float v) : t_(NUMBER), n_(v) {}
    Value(const char *s) : t_(STRING), s_(s) {}
    Value(std::string s) : t_(STRING), s_(std::move(s)) {}
    static Value array() {
        Value v;
        v.t_ = ARRAY;
        return v;
    }
    static Value object() {
        Value v;
        v.t_ = OBJECT;
        return v;
    }

    Type type() const { return t_; }
    bool isNull() const { return t_ == NUL; }
    bool isObject() const { return t_ == OBJECT; }
    bool isArray() const { return t_ == ARRAY; }
    bool isString() const { return t_ == STRING; }
    bool isNumber() const { return t_ == NUMBER; }
    bool isBool() const { return t_ == BOOL; }

    bool asBool() const {
        if (t_ != BOOL) throw std::runtime_error("json: not a bool");
        return b_;
    }
    double asNumber() const {
        if (t_ != NUMBER) throw std::runtime_error("json: not a number");
        return n_;
    }
    const std::string &asString() const {
        if (t_ != STRING) throw std::runtime_error("json: not a string");
        return s_;
    }
    const std::vector<Value> &items() const {
        if (t_ != ARRAY) throw std::runtime_error("json: not an array");
        return a_;
    }
    const std::vector<std::pair<std::string, Value>> &members() const {
        if (t_ != OBJECT) throw std::runtime_error("json: not an object");
        return o_;
    }

    bool contains(const std::string &k) const {
        if (t_ != OBJECT) return false;
        for (auto &m : o_)
            if (m.first == k) return true;
        return false;
    }
    const Value &operator[](const std::string &k) const {
        static const Value nul;
        if (t_ != OBJECT) return nul;
        for (auto &m : o_)
            if (m.first == k) return m.second;
        return nul;
    }
    Value &set(const std::string &k, Value v) {
        if (t_ == NUL) t_ = OBJECT;
        if (t_ != OBJECT) throw std::runtime_error("json: not an object");
        for (auto &m : o_)
            if (m.first == k) {
                m.second = std::move(v);
                return m.second;
            }
        o_.emplace_back(k, std::move(v));
        return o_.back().second;
    }
    Value &push(Value v) {
        if (t_ == NUL) t_ = ARRAY;
        if (t_ != ARRAY) throw std::runtime_error("json: not an array");
        a_.push_back(std::move(v));
        return a_.back();
    }
    size_t size() const { return t_ == ARRAY ? a_.size() : (t_ == OBJECT ? o_.size() : 0); }

    std::string dump() const {
        std::string out;
        dumpTo(out);
        return out;
    }

    static Value parse(const std::string &text) {
        size_t i = 0;
        Value v = parseValue(text, i);
        skipWs(text, i);
        if (i != text.size()) throw std::runtime_error("json: trailing characters");
        return v;
    }

  private:
    static void escape(const std::string &s, std::string &out) {
        out.push_back('"');
        for (unsigned char c : s) {
            switch (c) {
                case '"': out += "\\\""; break;
                case '\\': out += "\\\\"; break;
                case '\n': out += "\\n"; break;
                case '\r': out += "\\r"; break;
                case '\t': out += "\\t"; break;
                case '\b': out += "\\b"; break;
                case '\f': out += "\\f"; break;
                default:
                    if (c < 0x20) {
                        char buf[8];
                        std::snprintf(buf, sizeof(buf), "\\u%04x", c);
                        out += buf;
                    } else {
                        out.push_back((char)c);
                    }
            }
        }
        out.push_back('"');
    }
    void dumpTo(std::string &out) const {
        switch (t_) {
            case NUL: out += "null"; break;
            case BOOL: out += b_ ? "true" : "false"; break;
            case NUMBER: {
                char buf[32];
                if (std::isfinite(n_) && n_ == (double)(long long)n_ && std::fabs(n_) < 1e15)
                    std::snprintf(buf, sizeof(buf), "%lld", (long long)n_);
                else if (std::isfinite(n_))
                    std::snprintf(buf, sizeof(buf), "%.9g", n_);
                else
                    std::snprintf(buf, sizeof(buf), "null");
                out += buf;
                break;
            }
            case STRING: escape(s_, out); break;
            case ARRAY:
                out.push_back('[');
                for (size_t i = 0; i < a_.size(); i++) {
                    if (i) out.push_back(',');
                    a_[i].dumpTo(out);
                }
                out.push_back(']');
                break;
            case OBJECT:
                out.push_back('{');
                for (size_t i = 0; i < o_.size(); i++) {
                    if (i) out.push_back(',');
                    escape(o_[i].first, out);
                    out.push_back(':');
                    o_[i].second.dumpTo(out);
                }
                out.push_back('}');
                break;
        }
    }
    static void skipWs(const std::string &s, size_t &i) {
        while (i < s.size() && (s[i] == ' ' || s[i] == '\n' || s[i] == '\r' || s[i] == '\t')) i++;
    }
    static void appendUtf8(std::string &out, unsigned cp) {
        if (cp < 0x80) {
            out.push_back((char)cp);
        } else if (cp < 0x800) {
            out.push_back((char)(0xC0 | (cp >> 6)));
            out.push_back((char)(0x80 | (cp & 0x3F)));
        } else if (cp < 0x10000) {
            out.push_back((char)(0xE0 | (cp >> 12)));
            out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
            out.push_back((char)(0x80 | (cp & 0x3F)));
        } else {
            out.push_back((char)(0xF0 | (cp >> 18)));
            out.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
            out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
            out.push_back((char)(0x80 | (cp & 0x3F)));
        }
    }
    static unsigned hex4(const std::string &s, size_t &i) {
        if (i + 4 > s.size()) throw std::runtime_error("json: bad \\u escape");
        unsigned v = 0;
        for (int k = 0; k < 4; k++) {
            const char c = s[i++];
            v <<= 4;
            if (c >= '0' && c <= '9') v |= (unsigned)(c - '0');
            else if (c >= 'a' && c <= 'f') v |= (unsigned)(c - 'a' + 10);
            else if (c >= 'A' && c <= 'F') v |= (unsigned)(c - 'A' + 10);
            else throw std::runtime_error("json: bad hex digit");
        }
        return v;
    }
    static std::string parseString(const std::string &s, size_t &i) {
        if (s[i] != '"') throw std::runtime_error("json: expected string");
        i++;
        std::string out;
        while (true) {
            if (i >= s.size()) throw std::runtime_error("json: unterminated string");
            const char c = s[i++];
            if (c == '"') break;
            if (c != '\\') {
                out.push_back(c);
                continue;
            }
            if (i >= s.size()) throw std::runtime_error("json: bad escape");
            const char e = s[i++];
            switch (e) {
                case '"': out.push_back('"'); break;
                case '\\': out.push_back('\\'); break;
                case '/': out.push_back('/'); break;
                case 'b': out.push_back('\b'); break;
                case 'f': out.push_back('\f'); break;
                case 'n': out.push_back('\n'); break;
                case 'r': out.push_back('\r'); break;
                case 't': out.push_back('\t'); break;
                case 'u': {
                    unsigned cp = hex4(s, i);
                    if (cp >= 0xD800 && cp <= 0xDBFF && i + 6 <= s.size() && s[i] == '\\' && s[i + 1] == 'u') {
                        i += 2;
                        const unsigned lo = hex4(s, i);
                        cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
                    }
                    appendUtf8(out, cp);
                    break;
                }
                default: throw std::runtime_error("json: bad escape");
            }
        }
        return out;
    }
    static Value parseValue(const std::string &s, size_t &i) {
        skipWs(s, i);
        if (i >= s.size()) throw std::runtime_error("json: unexpected end");
        const char c = s[i];
        if (c == '{') {
            i++;
            Value v = object();
            skipWs(s, i);
            if (i < s.size() && s[i] == '}') {
                i++;
                return v;
            }
            while (true) {
                skipWs(s, i);
                std::string k = parseString(s, i);
                skipWs(s, i);
                if (i >= s.size() || s[i] != ':') throw std::runtime_error("json: expected ':'");
                i++;
                v.o_.emplace_back(std::move(k), parseValue(s, i));
                skipWs(s, i);
                if (i < s.size() && s[i] == ',') {
                    i++;
                    continue;
                }
                if (i < s.size() && s[i] == '}') {
                    i++;
                    return v;
                }
                throw std::runtime_error("json: expected ',' or '}'");
            }
        }
        if (c == '[') {
            i++;
            Value v = array();
            skipWs(s, i);
            if (i < s.size() && s[i] == ']') {
                i++;
                return v;
            }
            while (true) {
                v.a_.push_back(parseValue(s, i));
                skipWs(s, i);
                if (i < s.size() && s[i] == ',') {
                    i++;
                    continue;
                }
                if (i < s.size() && s[i] == ']') {
                    i++;
                    return v;
                }
                throw std::runtime_error("json: expected ',' or ']'");
            }
        }
        if (c == '"') return Value(parseString(s, i));
        if (s.compare(i, 4, "true") == 0) {
            i += 4;
            return Value(true);
        }
        if (s.compare(i, 5, "false") == 0) {
            i += 5;
            return Value(false);
        }
        if (s.compare(i, 4, "null") == 0) {
            i += 4;
            return Value();
        }
        size_t end = i;
        while (end < s.size() && (std::isdigit((unsigned char)s[end]) || s[end] == '-' || s[end] == '+' || s[end] == '.' ||
                                  s[end] == 'e' || s[end] == 'E'))
            end++;
        if (end == i) throw std::runtime_error("json: unexpected character");
        const double v = std::stod(s.substr(i, end - i));
        i = end;
        return Value(v);
    }

    Type t_;
    bool b_ = false;
    double n_ = 0;
    std::string s_;
    std::vector<Value> a_;
    std::vector<std::pair<std::string, Value>> o_;
};

}  // namespace json
}  // namespace dl
