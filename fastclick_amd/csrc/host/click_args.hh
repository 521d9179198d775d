// click_args.hh -- Click-style keyword arguments ("KEY value" strings), the
// subset of Args (include/click/args.hh) GPUIPCheckClassify's configure uses.
// Plain C++: shared by the FastClick element and the test harness.
#pragma once
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <string>
#include <vector>

namespace fcx {

// ---- Click-style keyword argument helpers (Args subset) ---------------------
// Splits "KEY value" words; a bare value with no keyword is positional.
struct ConfArg {
    std::string key, value;
};

inline std::string trim(const std::string &s) {
    size_t a = s.find_first_not_of(" \t\n\r"), b = s.find_last_not_of(" \t\n\r");
    return a == std::string::npos ? std::string() : s.substr(a, b - a + 1);
}

inline std::vector<std::string> split_conf(const std::string &s) {
    std::vector<std::string> out;
    std::string cur;
    int depth = 0;
    for (char c : s) {
        if (c == '(') depth++;
        if (c == ')') depth--;
        if (c == ',' && depth == 0) {
            out.push_back(trim(cur));
            cur.clear();
        } else {
            cur += c;
        }
    }
    if (!trim(cur).empty()) out.push_back(trim(cur));
    return out;
}

inline ConfArg parse_arg(const std::string &a) {
    ConfArg r;
    size_t sp = a.find_first_of(" \t");
    std::string k = a.substr(0, sp);
    bool upper = !k.empty();
    for (char c : k)
        if (!((c >= 'A' && c <= 'Z') || c == '_' || (c >= '0' && c <= '9'))) upper = false;
    if (upper && !(k[0] >= '0' && k[0] <= '9')) {
        r.key = k;
        r.value = sp == std::string::npos ? std::string() : trim(a.substr(sp));
    } else {
        r.value = a;
    }
    return r;
}

inline bool parse_bool(const std::string &v, bool &out) {
    if (v == "true" || v == "1" || v == "yes") { out = true; return true; }
    if (v == "false" || v == "0" || v == "no") { out = false; return true; }
    return false;
}

inline bool parse_int(const std::string &v, long &out) {
    if (v.empty()) return false;
    char *end = nullptr;
    out = strtol(v.c_str(), &end, 0);
    return end && *end == 0;
}

// "a.b.c.d" -> raw network-order word (IPAddress::addr())
inline bool parse_ip4(const std::string &v, uint32_t &out) {
    unsigned a, b, c, d;
    char tail;
    if (sscanf(v.c_str(), "%u.%u.%u.%u%c", &a, &b, &c, &d, &tail) != 4 || a > 255 || b > 255 || c > 255 || d > 255)
        return false;
    uint8_t bytes[4] = {(uint8_t)a, (uint8_t)b, (uint8_t)c, (uint8_t)d};
    memcpy(&out, bytes, 4);
    return true;
}

// IPPrefixArg(true) (lib/ipaddress.cc:196-255): "a[.b[.c[.d]]]/len",
// "a.b.c.d/m.m.m.m" or a bare address (mask 255.255.255.255); the mask may not
// cover more bytes than the address gives. Raw network-order words.
inline bool parse_ip4_prefix(const std::string &v, uint32_t &addr, uint32_t &mask) {
    const size_t slash = v.rfind('/');
    if (slash == std::string::npos) {
        if (!parse_ip4(v, addr)) return false;
        mask = 0xFFFFFFFFu;
        return true;
    }
    const std::string a = v.substr(0, slash), m = v.substr(slash + 1);
    uint8_t b[4] = {0, 0, 0, 0};
    int nbytes = 0;
    size_t pos = 0;
    while (nbytes < 4) {
        size_t e = pos;
        unsigned val = 0;
        while (e < a.size() && a[e] >= '0' && a[e] <= '9' && e - pos < 3) val = val * 10 + (unsigned)(a[e++] - '0');
        if (e == pos || val > 255) return false;
        b[nbytes++] = (uint8_t)val;
        if (e == a.size()) { pos = e; break; }
        if (a[e] != '.') return false;
        pos = e + 1;
    }
    if (pos != a.size()) return false;
    uint32_t mk;
    char *end = nullptr;
    const long l = strtol(m.c_str(), &end, 10);
    if (!m.empty() && end && *end == 0 && l >= 0 && l <= 32) {
        const uint32_t host = l == 0 ? 0u : 0xFFFFFFFFu << (32 - l);   // host-order prefix
        const uint8_t mb[4] = {(uint8_t)(host >> 24), (uint8_t)(host >> 16), (uint8_t)(host >> 8), (uint8_t)host};
        memcpy(&mk, mb, 4);
    } else if (!parse_ip4(m, mk)) {
        return false;
    }
    if (nbytes < 4) {   // the mask may not reach past the bytes given
        uint8_t mb[4];
        memcpy(mb, &mk, 4);
        for (int j = nbytes; j < 4; ++j)
            if (mb[j]) return false;
    }
    memcpy(&addr, b, 4);
    mask = mk;
    return true;
}

}  // namespace fcx
