// toml.hpp — minimal TOML reader for the reference's scene files (the subset the `toml 0.8`
// crate accepts and src/main.rs:36 feeds to the loaders): [tables], [[arrays of tables]],
// dotted/quoted keys, basic & literal strings, integers (with _ , 0x/0o/0b), floats (incl. exponent,
// inf, nan), booleans, arrays and inline tables, # comments.  Dates/multi-line strings are rejected.
#pragma once
#include <cmath>
#include <cstdint>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace toml {

struct Value;
using Table = std::map<std::string, Value>;   // toml::Table is a BTreeMap (sorted keys) by default
using Array = std::vector<Value>;

struct Value {
    enum Kind { None, Str, Int, Float, Bool, Arr, Tab } kind = None;
    std::string s;
    int64_t i = 0;
    double f = 0;
    bool b = false;
    std::shared_ptr<Array> a;
    std::shared_ptr<Table> t;

    static Value table() { Value v; v.kind = Tab; v.t = std::make_shared<Table>(); return v; }
    static Value array() { Value v; v.kind = Arr; v.a = std::make_shared<Array>(); return v; }
    const Table* as_table() const { return kind == Tab ? t.get() : nullptr; }
    const Array* as_array() const { return kind == Arr ? a.get() : nullptr; }
    const std::string* as_str() const { return kind == Str ? &s : nullptr; }
    bool is_float() const { return kind == Float; }
    bool is_int() const { return kind == Int; }
    bool is_bool() const { return kind == Bool; }
};

struct ParseError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

class Parser {
  public:
    explicit Parser(const std::string& text) : src_(text) {}

    Value parse() {
        Value root = Value::table();
        Table* cur = root.t.get();
        while (true) {
            skip_ws_comments_newlines();
            if (eof()) break;
            if (peek() == '[') {
                bool array_of_tables = peek(1) == '[';
                pos_ += array_of_tables ? 2 : 1;
                std::vector<std::string> path = parse_key_path(']');
                expect(']');
                if (array_of_tables) expect(']');
                cur = array_of_tables ? open_array_table(root, path) : open_table(root, path);
                finish_line();
                continue;
            }
            parse_keyval(*cur);
            finish_line();
        }
        return root;
    }

  private:
    const std::string& src_;
    size_t pos_ = 0;
    int line_ = 1;

    bool eof() const { return pos_ >= src_.size(); }
    char peek(size_t o = 0) const { return pos_ + o < src_.size() ? src_[pos_ + o] : '\0'; }
    [[noreturn]] void fail(const std::string& m) const {
        throw ParseError("TOML parse error at line " + std::to_string(line_) + ": " + m);
    }
    void expect(char c) {
        skip_ws();
        if (peek() != c) fail(std::string("expected '") + c + "'");
        ++pos_;
    }
    void skip_ws() {
        while (!eof() && (peek() == ' ' || peek() == '\t')) ++pos_;
    }
    void skip_comment() {
        if (peek() == '#')
            while (!eof() && peek() != '\n') ++pos_;
    }
    void skip_ws_comments_newlines() {
        while (!eof()) {
            skip_ws();
            skip_comment();
            if (peek() == '\r' && peek(1) == '\n') { pos_ += 2; ++line_; continue; }
            if (peek() == '\n') { ++pos_; ++line_; continue; }
            break;
        }
    }
    void finish_line() {
        skip_ws();
        skip_comment();
        if (eof()) return;
        if (peek() == '\r') ++pos_;
        if (peek() != '\n') fail("expected end of line");
        ++pos_;
        ++line_;
    }

    static bool bare_char(char c) {
        return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9') || c == '_' || c == '-';
    }
    std::string parse_simple_key() {
        skip_ws();
        if (peek() == '"') return parse_basic_string();
        if (peek() == '\'') return parse_literal_string();
        size_t b = pos_;
        while (!eof() && bare_char(peek())) ++pos_;
        if (b == pos_) fail("expected a key");
        return src_.substr(b, pos_ - b);
    }
    std::vector<std::string> parse_key_path(char term) {
        std::vector<std::string> path{parse_simple_key()};
        skip_ws();
        while (peek() == '.') {
            ++pos_;
            path.push_back(parse_simple_key());
            skip_ws();
        }
        if (peek() != term) fail(std::string("expected '") + term + "' after key");
        return path;
    }

    Table* descend(Table* t, const std::string& k) {
        auto it = t->find(k);
        if (it == t->end()) it = t->emplace(k, Value::table()).first;
        Value& v = it->second;
        if (v.kind == Value::Tab) return v.t.get();
        if (v.kind == Value::Arr && !v.a->empty() && v.a->back().kind == Value::Tab) return v.a->back().t.get();
        fail("key '" + k + "' is not a table");
    }
    Table* open_table(Value& root, const std::vector<std::string>& path) {
        Table* t = root.t.get();
        for (const auto& k : path) t = descend(t, k);
        return t;
    }
    Table* open_array_table(Value& root, const std::vector<std::string>& path) {
        Table* t = root.t.get();
        for (size_t i = 0; i + 1 < path.size(); ++i) t = descend(t, path[i]);
        auto it = t->find(path.back());
        if (it == t->end()) it = t->emplace(path.back(), Value::array()).first;
        if (it->second.kind != Value::Arr) fail("key '" + path.back() + "' is not an array of tables");
        it->second.a->push_back(Value::table());
        return it->second.a->back().t.get();
    }

    void parse_keyval(Table& t) {
        std::vector<std::string> path = parse_key_path('=');
        ++pos_;  // '='
        skip_ws();
        Value v = parse_value();
        Table* dst = &t;
        for (size_t i = 0; i + 1 < path.size(); ++i) dst = descend(dst, path[i]);
        if (dst->count(path.back())) fail("duplicate key '" + path.back() + "'");
        dst->emplace(path.back(), std::move(v));
    }

    std::string parse_basic_string() {
        ++pos_;  // "
        if (peek() == '"' && peek(1) == '"') fail("multi-line strings are not supported");
        std::string out;
        while (true) {
            if (eof() || peek() == '\n') fail("unterminated string");
            char c = src_[pos_++];
            if (c == '"') break;
            if (c != '\\') { out += c; continue; }
            char e = src_[pos_++];
            switch (e) {
                case 'b': out += '\b'; break;
                case 't': out += '\t'; break;
                case 'n': out += '\n'; break;
                case 'f': out += '\f'; break;
                case 'r': out += '\r'; break;
                case '"': out += '"'; break;
                case '\\': out += '\\'; break;
                case 'u': case 'U': {
                    int n = e == 'u' ? 4 : 8;
                    uint32_t cp = (uint32_t)std::stoul(src_.substr(pos_, n), nullptr, 16);
                    pos_ += n;
                    if (cp < 0x80) out += (char)cp;
                    else if (cp < 0x800) { out += (char)(0xC0 | (cp >> 6)); out += (char)(0x80 | (cp & 63)); }
                    else if (cp < 0x10000) {
                        out += (char)(0xE0 | (cp >> 12)); out += (char)(0x80 | ((cp >> 6) & 63)); out += (char)(0x80 | (cp & 63));
                    } else {
                        out += (char)(0xF0 | (cp >> 18)); out += (char)(0x80 | ((cp >> 12) & 63));
                        out += (char)(0x80 | ((cp >> 6) & 63)); out += (char)(0x80 | (cp & 63));
                    }
                    break;
                }
                default: fail("invalid escape");
            }
        }
        return out;
    }
    std::string parse_literal_string() {
        ++pos_;
        size_t b = pos_;
        while (!eof() && peek() != '\'' && peek() != '\n') ++pos_;
        if (peek() != '\'') fail("unterminated literal string");
        std::string out = src_.substr(b, pos_ - b);
        ++pos_;
        return out;
    }

    Value parse_value() {
        skip_ws();
        Value v;
        char c = peek();
        if (c == '"') { v.kind = Value::Str; v.s = parse_basic_string(); return v; }
        if (c == '\'') { v.kind = Value::Str; v.s = parse_literal_string(); return v; }
        if (c == '[') return parse_array();
        if (c == '{') return parse_inline_table();
        if (src_.compare(pos_, 4, "true") == 0 && !bare_char(peek(4))) { pos_ += 4; v.kind = Value::Bool; v.b = true; return v; }
        if (src_.compare(pos_, 5, "false") == 0 && !bare_char(peek(5))) { pos_ += 5; v.kind = Value::Bool; v.b = false; return v; }
        return parse_number();
    }
    Value parse_number() {
        size_t b = pos_;
        while (!eof() && (bare_char(peek()) || peek() == '+' || peek() == '.' || peek() == ':')) ++pos_;
        std::string tok = src_.substr(b, pos_ - b);
        if (tok.empty()) fail("expected a value");
        std::string t;
        for (char ch : tok)
            if (ch != '_') t += ch;
        Value v;
        std::string body = (t[0] == '+' || t[0] == '-') ? t.substr(1) : t;
        const bool neg = t[0] == '-';
        if (body == "inf" || body == "nan") {
            v.kind = Value::Float;
            v.f = body == "inf" ? INFINITY : NAN;
            if (neg) v.f = -v.f;
            return v;
        }
        if (t.find(':') != std::string::npos || (t.find('-', 1) != std::string::npos &&
                                                 t.find_first_of("eE") == std::string::npos))
            fail("dates/times are not supported");
        try {
            if (body.size() > 2 && body[0] == '0' && (body[1] == 'x' || body[1] == 'o' || body[1] == 'b')) {
                int base = body[1] == 'x' ? 16 : body[1] == 'o' ? 8 : 2;
                v.kind = Value::Int;
                v.i = (int64_t)std::stoull(body.substr(2), nullptr, base);
                return v;
            }
            if (t.find_first_of(".eE") != std::string::npos) {
                size_t used = 0;
                v.kind = Value::Float;
                v.f = std::stod(t, &used);
                if (used != t.size()) fail("bad float '" + tok + "'");
                return v;
            }
            size_t used = 0;
            v.kind = Value::Int;
            v.i = std::stoll(t, &used, 10);
            if (used != t.size()) fail("bad integer '" + tok + "'");
            return v;
        } catch (const std::logic_error&) {
            fail("bad number '" + tok + "'");
        }
    }
    Value parse_array() {
        ++pos_;  // [
        Value v = Value::array();
        while (true) {
            skip_ws_comments_newlines();
            if (peek() == ']') { ++pos_; break; }
            v.a->push_back(parse_value());
            skip_ws_comments_newlines();
            if (peek() == ',') { ++pos_; continue; }
            if (peek() == ']') { ++pos_; break; }
            fail("expected ',' or ']' in array");
        }
        return v;
    }
    Value parse_inline_table() {
        ++pos_;  // {
        Value v = Value::table();
        skip_ws();
        if (peek() == '}') { ++pos_; return v; }
        while (true) {
            parse_keyval(*v.t);
            skip_ws();
            if (peek() == ',') { ++pos_; continue; }
            if (peek() == '}') { ++pos_; break; }
            fail("expected ',' or '}' in inline table");
        }
        return v;
    }
};

inline Value parse(const std::string& text) { return Parser(text).parse(); }

}  // namespace toml
