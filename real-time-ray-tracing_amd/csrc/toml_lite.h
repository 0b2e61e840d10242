// toml_lite.h — the small TOML subset the reference's config uses (configLoader.cpp:5-27):
// [table] headers, key = value with integers, floats, booleans, "strings" and
// ["string", ...] arrays, '#' comments.  Unknown keys are kept and ignored.
#pragma once
#include <stdio.h>
#include <stdlib.h>

#include <map>
#include <string>
#include <vector>

namespace rttoml {

struct Value {
    std::string raw;                  // scalar text (strings unquoted)
    std::vector<std::string> array;   // for [..] values
    bool isArray = false;
    bool isString = false;
};

using Table = std::map<std::string, Value>;
using Doc = std::map<std::string, Table>;

inline std::string trim(const std::string& s) {
    size_t a = s.find_first_not_of(" \t\r\n"), b = s.find_last_not_of(" \t\r\n");
    return a == std::string::npos ? std::string() : s.substr(a, b - a + 1);
}

inline std::string strip_comment(const std::string& s) {
    bool inStr = false;
    for (size_t i = 0; i < s.size(); ++i) {
        if (s[i] == '"') inStr = !inStr;
        if (s[i] == '#' && !inStr) return s.substr(0, i);
    }
    return s;
}

inline bool parse_string_list(const std::string& body, std::vector<std::string>& out) {
    out.clear();
    size_t i = 0;
    while (i < body.size()) {
        size_t q = body.find('"', i);
        if (q == std::string::npos) break;
        size_t e = body.find('"', q + 1);
        if (e == std::string::npos) return false;
        out.push_back(body.substr(q + 1, e - q - 1));
        i = e + 1;
    }
    return true;
}

inline bool parse(const std::string& text, Doc& doc, std::string& err) {
    std::string table;
    size_t pos = 0;
    int lineNo = 0;
    while (pos <= text.size()) {
        size_t nl = text.find('\n', pos);
        std::string line = text.substr(pos, nl == std::string::npos ? std::string::npos : nl - pos);
        pos = (nl == std::string::npos) ? text.size() + 1 : nl + 1;
        ++lineNo;
        line = trim(strip_comment(line));
        if (line.empty()) continue;
        if (line[0] == '[') {
            size_t e = line.find(']');
            if (e == std::string::npos) { err = "bad table header at line " + std::to_string(lineNo); return false; }
            table = trim(line.substr(1, e - 1));
            doc[table];
            continue;
        }
        size_t eq = line.find('=');
        if (eq == std::string::npos) { err = "expected key = value at line " + std::to_string(lineNo); return false; }
        std::string key = trim(line.substr(0, eq)), val = trim(line.substr(eq + 1));
        Value v;
        if (!val.empty() && val[0] == '[') {
            v.isArray = true;
            if (!parse_string_list(val, v.array)) { err = "bad array at line " + std::to_string(lineNo); return false; }
        } else if (!val.empty() && val[0] == '"') {
            size_t e = val.find('"', 1);
            if (e == std::string::npos) { err = "unterminated string at line " + std::to_string(lineNo); return false; }
            v.raw = val.substr(1, e - 1);
            v.isString = true;
        } else {
            v.raw = val;
        }
        doc[table][key] = v;
    }
    return true;
}

inline const Value* find(const Doc& d, const std::string& t, const std::string& k) {
    auto it = d.find(t);
    if (it == d.end()) return nullptr;
    auto jt = it->second.find(k);
    return jt == it->second.end() ? nullptr : &jt->second;
}
inline int find_or_int(const Doc& d, const std::string& t, const std::string& k, int def) {
    const Value* v = find(d, t, k);
    return (v && !v->isArray && !v->isString && !v->raw.empty()) ? (int)strtol(v->raw.c_str(), nullptr, 10) : def;
}
inline float find_or_float(const Doc& d, const std::string& t, const std::string& k, float def) {
    const Value* v = find(d, t, k);
    return (v && !v->isArray && !v->isString && !v->raw.empty()) ? strtof(v->raw.c_str(), nullptr) : def;
}
inline bool find_or_bool(const Doc& d, const std::string& t, const std::string& k, bool def) {
    const Value* v = find(d, t, k);
    if (!v || v->isArray) return def;
    if (v->raw == "true") return true;
    if (v->raw == "false") return false;
    return def;
}
inline std::string find_or_string(const Doc& d, const std::string& t, const std::string& k, const std::string& def) {
    const Value* v = find(d, t, k);
    return (v && v->isString) ? v->raw : def;
}
inline std::vector<std::string> find_or_strings(const Doc& d, const std::string& t, const std::string& k) {
    const Value* v = find(d, t, k);
    return (v && v->isArray) ? v->array : std::vector<std::string>();
}

}  // namespace rttoml
