// json.cpp -- see json.hpp for the contract (jsoncpp 1.6.5 recovery semantics).
#include "json.hpp"

#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <stdexcept>

namespace fpmhost {

Json Json::make_bool(bool b) { Json j; j.type_ = Bool; j.b_ = b; return j; }
Json Json::make_int(int64_t v) { Json j; j.type_ = Int; j.i_ = v; return j; }
Json Json::make_real(double v) { Json j; j.type_ = Real; j.d_ = v; return j; }
Json Json::make_string(std::string s) { Json j; j.type_ = String; j.s_ = std::move(s); return j; }
Json Json::make_array() { Json j; j.type_ = Array; return j; }
Json Json::make_object() { Json j; j.type_ = Object; return j; }

size_t Json::size() const {
    if (type_ == Array) return arr_.size();
    if (type_ == Object) return obj_.size();
    return 0;
}

int Json::as_int() const {
    switch (type_) {
        case Null: return 0;
        case Bool: return b_ ? 1 : 0;
        case Int:
            if (i_ < INT32_MIN || i_ > INT32_MAX) throw std::runtime_error("LargestInt out of Int range");
            return (int)i_;
        case Real:
            if (!(d_ >= (double)INT32_MIN && d_ <= (double)INT32_MAX))
                throw std::runtime_error("double out of Int range");
            return (int)d_;  // truncation, like jsoncpp Int(value_.real_)
        default: throw std::runtime_error("Value is not convertible to Int.");
    }
}

double Json::as_double() const {
    switch (type_) {
        case Null: return 0.0;
        case Bool: return b_ ? 1.0 : 0.0;
        case Int: return (double)i_;
        case Real: return d_;
        default: throw std::runtime_error("Value is not convertible to double.");
    }
}

bool Json::as_bool() const {
    switch (type_) {
        case Null: return false;
        case Bool: return b_;
        case Int: return i_ != 0;
        case Real: return d_ != 0.0;
        default: throw std::runtime_error("Value is not convertible to bool.");
    }
}

std::string Json::as_string() const {
    char buf[64];
    switch (type_) {
        case Null: return "";
        case String: return s_;
        case Bool: return b_ ? "true" : "false";
        case Int: snprintf(buf, sizeof buf, "%lld", (long long)i_); return buf;
        case Real: snprintf(buf, sizeof buf, "%.17g", d_); return buf;
        default: throw std::runtime_error("Type is not convertible to string");
    }
}

bool Json::has(const std::string &key) const {
    if (type_ != Object) return false;
    for (auto &m : obj_)
        if (m.first == key) return true;
    return false;
}

const Json &Json::get(const std::string &key, const Json &dflt) const {
    if (type_ == Null) return dflt;
    if (type_ != Object) throw std::runtime_error("Json::get requires objectValue or nullValue");
    for (auto &m : obj_)
        if (m.first == key) return m.second;
    return dflt;
}

void Json::set(const std::string &key, Json v) {
    if (type_ == Null) type_ = Object;
    if (type_ != Object) throw std::runtime_error("Json::set requires objectValue or nullValue");
    for (auto &m : obj_)
        if (m.first == key) {
            m.second = std::move(v);
            return;
        }
    obj_.emplace_back(key, std::move(v));
}

const Json &Json::at(size_t i) const {
    static const Json null_value;
    if (type_ != Array || i >= arr_.size()) return null_value;
    return arr_[i];
}

namespace {

struct Parser {
    const std::string &s;
    size_t p = 0;
    bool failed = false;
    std::string err;
    size_t err_at = 0;

    explicit Parser(const std::string &text) : s(text) {}

    void ws() {
        while (p < s.size() && (s[p] == ' ' || s[p] == '\t' || s[p] == '\r' || s[p] == '\n')) ++p;
    }
    bool fail(const char *msg) {
        if (!failed) {
            failed = true;
            err = msg;
            err_at = p;
        }
        return false;
    }
    // jsoncpp: comments are allowed by default (Features::all)
    void skip_ws_comments() {
        for (;;) {
            ws();
            if (p + 1 < s.size() && s[p] == '/' && s[p + 1] == '/') {
                while (p < s.size() && s[p] != '\n') ++p;
            } else if (p + 1 < s.size() && s[p] == '/' && s[p + 1] == '*') {
                size_t e = s.find("*/", p + 2);
                p = (e == std::string::npos) ? s.size() : e + 2;
            } else {
                return;
            }
        }
    }

    bool value(Json &out) {
        skip_ws_comments();
        if (p >= s.size()) return fail("Syntax error: value, object or array expected.");
        char c = s[p];
        if (c == '{') return object(out);
        if (c == '[') return array(out);
        if (c == '"') {
            std::string str;
            if (!string(str)) return false;
            out = Json::make_string(std::move(str));
            return true;
        }
        if (c == '-' || (c >= '0' && c <= '9')) return number(out);
        if (s.compare(p, 4, "true") == 0) { p += 4; out = Json::make_bool(true); return true; }
        if (s.compare(p, 5, "false") == 0) { p += 5; out = Json::make_bool(false); return true; }
        if (s.compare(p, 4, "null") == 0) { p += 4; out = Json(); return true; }
        return fail("Syntax error: value, object or array expected.");
    }

    bool number(Json &out) {
        // jsoncpp readNumber: greedy over [0-9+-.eE]
        size_t b = p;
        bool is_real = false;
        while (p < s.size() && (isdigit((unsigned char)s[p]) || s[p] == '-' || s[p] == '+' || s[p] == '.' ||
                                s[p] == 'e' || s[p] == 'E')) {
            if (s[p] == '.' || s[p] == 'e' || s[p] == 'E') is_real = true;
            ++p;
        }
        std::string tok = s.substr(b, p - b);
        char *end = nullptr;
        if (!is_real) {
            errno = 0;
            long long v = strtoll(tok.c_str(), &end, 10);
            if (*end == 0 && errno == 0) {
                out = Json::make_int(v);
                return true;
            }
        }
        double d = strtod(tok.c_str(), &end);
        if (*end != 0) return fail("not a number");
        out = Json::make_real(d);
        return true;
    }

    bool string(std::string &out) {
        ++p;  // opening quote
        while (p < s.size()) {
            char c = s[p++];
            if (c == '"') return true;
            if (c == '\\') {
                if (p >= s.size()) break;
                char e = s[p++];
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
                        if (p + 4 > s.size()) return fail("bad unicode escape");
                        unsigned cp = (unsigned)strtoul(s.substr(p, 4).c_str(), nullptr, 16);
                        p += 4;
                        if (cp < 0x80) out += (char)cp;
                        else if (cp < 0x800) { out += (char)(0xC0 | (cp >> 6)); out += (char)(0x80 | (cp & 0x3F)); }
                        else { out += (char)(0xE0 | (cp >> 12)); out += (char)(0x80 | ((cp >> 6) & 0x3F)); out += (char)(0x80 | (cp & 0x3F)); }
                        break;
                    }
                    default: return fail("bad escape sequence");
                }
            } else {
                out += c;
            }
        }
        return fail("Missing '\"' at end of string");
    }

    bool object(Json &out) {
        out = Json::make_object();
        ++p;
        skip_ws_comments();
        if (p < s.size() && s[p] == '}') { ++p; return true; }
        for (;;) {
            skip_ws_comments();
            if (p >= s.size() || s[p] != '"') return fail("Missing '}' or object member name");
            std::string name;
            if (!string(name)) return false;
            skip_ws_comments();
            if (p >= s.size() || s[p] != ':') return fail("Missing ':' after object member name");
            ++p;
            // jsoncpp creates the member before parsing its value (currentValue()[name])
            Json *slot = nullptr;
            for (auto &m : out.members())
                if (m.first == name) slot = &m.second;
            if (!slot) {
                out.members().emplace_back(name, Json());
                slot = &out.members().back().second;
            }
            *slot = Json();
            if (!value(*slot)) return false;
            skip_ws_comments();
            if (p < s.size() && s[p] == ',') { ++p; continue; }
            if (p < s.size() && s[p] == '}') { ++p; return true; }
            return fail("Missing ',' or '}' in object declaration");
        }
    }

    bool array(Json &out) {
        out = Json::make_array();
        ++p;
        ws();
        if (p < s.size() && s[p] == ']') { ++p; return true; }
        for (;;) {
            // jsoncpp appends the element before reading it: a trailing comma
            // therefore leaves a null element behind (dataset_dogStomach.json:320-321)
            out.items().emplace_back();
            if (!value(out.items().back())) return false;
            skip_ws_comments();
            if (p < s.size() && s[p] == ',') { ++p; continue; }
            if (p < s.size() && s[p] == ']') { ++p; return true; }
            return fail("Missing ',' or ']' in array declaration");
        }
    }
};

}  // namespace

JsonParseResult parse_json(const std::string &text) {
    JsonParseResult r;
    Parser ps(text);
    bool ok = ps.value(r.root);
    r.ok = ok && !ps.failed;
    r.error = ps.err;
    r.error_offset = ps.err_at;
    return r;
}

bool read_file(const std::string &path, std::string *out) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    std::ostringstream ss;
    ss << f.rdbuf();
    *out = ss.str();
    return true;
}

}  // namespace fpmhost
