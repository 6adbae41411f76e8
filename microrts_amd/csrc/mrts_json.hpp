// mrts_json.hpp — a small JSON reader (RFC 8259 values; numbers kept as double + int64) for the
// reference's JSON inputs: unit-type tables (UnitTypeTable.fromJSON, rts/units/UnitTypeTable.java:
// 414-433) and game states (GameState.fromJSON, rts/GameState.java:897-915).  Header-only.
#pragma once
#include <cstdint>
#include <cstdlib>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace mjson {

struct Value {
    enum Kind { NUL, BOOL, NUM, STR, ARR, OBJ } kind = NUL;
    bool b = false;
    double num = 0;
    int64_t i = 0;
    bool isInt = false;
    std::string s;
    std::vector<Value> arr;
    std::vector<std::pair<std::string, Value>> obj;  // member order kept

    const Value* get(const std::string& k) const {
        for (auto& m : obj)
            if (m.first == k) return &m.second;
        return nullptr;
    }
    // minimal-json's JsonObject.getInt / getBoolean / getString(name, default): the default when the
    // member is absent; a present member of the wrong type throws (UnsupportedOperationException)
    int getInt(const std::string& k, int def) const {
        const Value* v = get(k);
        if (!v) return def;
        if (v->kind != NUM || !v->isInt || v->i < INT32_MIN || v->i > INT32_MAX) throw std::runtime_error("not an int: " + k);
        return (int)v->i;
    }
    int64_t getLong(const std::string& k, int64_t def) const {
        const Value* v = get(k);
        if (!v) return def;
        if (v->kind != NUM || !v->isInt) throw std::runtime_error("not a long: " + k);
        return v->i;
    }
    bool getBool(const std::string& k, bool def) const {
        const Value* v = get(k);
        if (!v) return def;
        if (v->kind != BOOL) throw std::runtime_error("not a boolean: " + k);
        return v->b;
    }
    std::string getString(const std::string& k, const std::string& def) const {
        const Value* v = get(k);
        if (!v) return def;
        if (v->kind != STR) throw std::runtime_error("not a string: " + k);
        return v->s;
    }
    const Value& at(const std::string& k) const {
        const Value* v = get(k);
        if (!v) throw std::runtime_error("missing member: " + k);
        return *v;
    }
};

class Parser {
public:
    explicit Parser(const std::string& t) : t_(t) {}
    Value parse() {
        Value v = value(0);
        ws();
        if (p_ != t_.size()) fail("trailing characters");
        return v;
    }

private:
    const std::string& t_;
    size_t p_ = 0;
    [[noreturn]] void fail(const char* m) const { throw std::runtime_error(std::string("JSON: ") + m + " at offset " + std::to_string(p_)); }
    void ws() {
        while (p_ < t_.size() && (t_[p_] == ' ' || t_[p_] == '\t' || t_[p_] == '\n' || t_[p_] == '\r')) p_++;
    }
    bool lit(const char* w) {
        size_t n = 0;
        while (w[n]) n++;
        if (t_.compare(p_, n, w) == 0) {
            p_ += n;
            return true;
        }
        return false;
    }
    Value value(int depth) {
        if (depth > 64) fail("nesting too deep");
        ws();
        if (p_ >= t_.size()) fail("unexpected end");
        Value v;
        const char c = t_[p_];
        if (c == '{') {
            v.kind = Value::OBJ;
            p_++;
            ws();
            if (p_ < t_.size() && t_[p_] == '}') {
                p_++;
                return v;
            }
            for (;;) {
                ws();
                if (p_ >= t_.size() || t_[p_] != '"') fail("expected a member name");
                std::string k = str();
                ws();
                if (p_ >= t_.size() || t_[p_] != ':') fail("expected ':'");
                p_++;
                v.obj.emplace_back(std::move(k), value(depth + 1));
                ws();
                if (p_ < t_.size() && t_[p_] == ',') {
                    p_++;
                    continue;
                }
                if (p_ < t_.size() && t_[p_] == '}') {
                    p_++;
                    return v;
                }
                fail("expected ',' or '}'");
            }
        }
        if (c == '[') {
            v.kind = Value::ARR;
            p_++;
            ws();
            if (p_ < t_.size() && t_[p_] == ']') {
                p_++;
                return v;
            }
            for (;;) {
                v.arr.push_back(value(depth + 1));
                ws();
                if (p_ < t_.size() && t_[p_] == ',') {
                    p_++;
                    continue;
                }
                if (p_ < t_.size() && t_[p_] == ']') {
                    p_++;
                    return v;
                }
                fail("expected ',' or ']'");
            }
        }
        if (c == '"') {
            v.kind = Value::STR;
            v.s = str();
            return v;
        }
        if (lit("true")) {
            v.kind = Value::BOOL;
            v.b = true;
            return v;
        }
        if (lit("false")) {
            v.kind = Value::BOOL;
            return v;
        }
        if (lit("null")) return v;
        return number();
    }
    std::string str() {
        p_++;  // opening quote
        std::string out;
        while (p_ < t_.size() && t_[p_] != '"') {
            char c = t_[p_++];
            if (c == '\\') {
                if (p_ >= t_.size()) fail("bad escape");
                const char e = t_[p_++];
                switch (e) {
                    case '"': out += '"'; break;
                    case '\\': out += '\\'; break;
                    case '/': out += '/'; break;
                    case 'b': out += '\b'; break;
                    case 'f': out += '\f'; break;
                    case 'n': out += '\n'; break;
                    case 'r': out += '\r'; break;
                    case 't': out += '\t'; break;
                    case 'u': {
                        if (p_ + 4 > t_.size()) fail("bad \\u escape");
                        const unsigned cp = (unsigned)std::strtoul(t_.substr(p_, 4).c_str(), nullptr, 16);
                        p_ += 4;
                        if (cp < 0x80) {
                            out += (char)cp;
                        } else if (cp < 0x800) {
                            out += (char)(0xC0 | (cp >> 6));
                            out += (char)(0x80 | (cp & 0x3F));
                        } else {
                            out += (char)(0xE0 | (cp >> 12));
                            out += (char)(0x80 | ((cp >> 6) & 0x3F));
                            out += (char)(0x80 | (cp & 0x3F));
                        }
                        break;
                    }
                    default: fail("bad escape");
                }
            } else {
                out += c;
            }
        }
        if (p_ >= t_.size()) fail("unterminated string");
        p_++;
        return out;
    }
    Value number() {
        const size_t b = p_;
        if (p_ < t_.size() && t_[p_] == '-') p_++;
        bool frac = false;
        while (p_ < t_.size()) {
            const char c = t_[p_];
            if (c >= '0' && c <= '9') {
                p_++;
            } else if (c == '.' || c == 'e' || c == 'E' || c == '+' || (c == '-' && p_ > b)) {
                frac = true;
                p_++;
            } else {
                break;
            }
        }
        if (p_ == b || (p_ == b + 1 && t_[b] == '-')) fail("unexpected character");
        Value v;
        v.kind = Value::NUM;
        const std::string tok = t_.substr(b, p_ - b);
        v.num = std::strtod(tok.c_str(), nullptr);
        if (!frac) {
            v.isInt = true;
            v.i = std::strtoll(tok.c_str(), nullptr, 10);
        }
        return v;
    }
};

inline Value parse(const std::string& text) { return Parser(text).parse(); }

}  // namespace mjson
