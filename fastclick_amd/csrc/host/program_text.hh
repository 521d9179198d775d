// program_text.hh -- parse a decision program as the reference prints it.
//
// IPFilter / IPClassifier / Classifier expose their compiled program through
// the `program` read handler (Classification::Wordwise::Program::unparse,
// elements/standard/classification.cc:978-991, and CompressedProgram::unparse,
// :1104-1140), one step per line:
//
//    0 264/00110000%00ff0000  yes->step 1  no->step 5
//    3 512/00000000%fc000000  yes->[3]  no->step 4  short->yes
//   safe length 516
//   alignment offset 0
// or, for a program that sends everything to one output, "all->[N]".
// Value and mask are the four packet bytes in order; a jump is "step N", an
// output "[N]", or "[X]" (drop). Lines may be separated by newlines or '|'.
#pragma once
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <string>
#include <vector>

#include "../../../include/fastclick_gpu.h"

namespace fcx {

struct ParsedProgram {
    std::vector<fcgpu_step> steps;
    int32_t output_everything = -1;
    int32_t safe_length = -1;
    int32_t align_offset = 0;
};

inline bool parse_jump(const char *&p, int32_t &j) {
    while (*p == ' ') ++p;
    if (!strncmp(p, "step ", 5)) {
        p += 5;
        char *e;
        long v = strtol(p, &e, 10);
        if (e == p || v <= 0) return false;
        j = (int32_t)v;
        p = e;
        return true;
    }
    if (*p != '[') return false;
    ++p;
    if (*p == 'X' || *p == '-' || *p == '+') {   // j_never / j_failure / j_success
        j = -2147483647;
        ++p;
    } else {
        char *e;
        long v = strtol(p, &e, 10);
        if (e == p || v < 0) return false;
        j = (int32_t)-v;
        p = e;
    }
    if (*p != ']') return false;
    ++p;
    return true;
}

inline bool hex_word(const char *p, uint32_t &w) {
    uint8_t b[4];
    for (int k = 0; k < 4; ++k) {
        char t[3] = {p[2 * k], p[2 * k + 1], 0};
        char *e;
        unsigned long v = strtoul(t, &e, 16);
        if (*e || e != t + 2) return false;
        b[k] = (uint8_t)v;
    }
    memcpy(&w, b, 4);     // packet byte order, read little-endian like the reference
    return true;
}

// Returns an empty string on success, else an error message.
inline std::string parse_program(const std::string &text, ParsedProgram &out) {
    out = ParsedProgram();
    std::string norm = text;
    for (char &c : norm)
        if (c == '|') c = '\n';
    size_t pos = 0;
    int lineno = 0;
    while (pos <= norm.size()) {
        size_t nl = norm.find('\n', pos);
        std::string line = norm.substr(pos, nl == std::string::npos ? std::string::npos : nl - pos);
        pos = nl == std::string::npos ? norm.size() + 1 : nl + 1;
        ++lineno;
        const char *p = line.c_str();
        while (*p == ' ' || *p == '\t') ++p;
        if (!*p) continue;
        if (!strncmp(p, "safe length", 11)) { out.safe_length = atoi(p + 11); continue; }
        if (!strncmp(p, "alignment offset", 16)) { out.align_offset = atoi(p + 16); continue; }
        if (!strncmp(p, "all->", 5)) {
            const char *q = p + 5;
            int32_t j = 0;
            if (!parse_jump(q, j) || j > 0) return "bad all-> line " + std::to_string(lineno);
            out.output_everything = j <= -2147483647 ? 0x7fff : -j;
            continue;
        }
        char *e;
        long idx = strtol(p, &e, 10);
        if (e == p || idx != (long)out.steps.size()) return "bad step index on line " + std::to_string(lineno);
        p = e;
        while (*p == ' ') ++p;
        long off = strtol(p, &e, 10);
        if (e == p || *e != '/') return "bad offset on line " + std::to_string(lineno);
        p = e + 1;
        fcgpu_step st;
        memset(&st, 0, sizeof st);
        st.offset = (int32_t)off;
        if (strlen(p) < 17 || p[8] != '%' || !hex_word(p, st.value) || !hex_word(p + 9, st.mask))
            return "bad value%mask on line " + std::to_string(lineno);
        p += 17;
        while (*p == ' ') ++p;
        if (strncmp(p, "yes->", 5)) return "missing yes-> on line " + std::to_string(lineno);
        p += 5;
        if (!parse_jump(p, st.yes)) return "bad yes jump on line " + std::to_string(lineno);
        while (*p == ' ') ++p;
        if (strncmp(p, "no->", 4)) return "missing no-> on line " + std::to_string(lineno);
        p += 4;
        if (!parse_jump(p, st.no)) return "bad no jump on line " + std::to_string(lineno);
        while (*p == ' ') ++p;
        if (!strncmp(p, "short->yes", 10)) st.flags |= FCGPU_STEP_SHORT_YES;
        st.value &= st.mask;
        out.steps.push_back(st);
    }
    for (const auto &st : out.steps)
        if (st.yes >= (int32_t)out.steps.size() || st.no >= (int32_t)out.steps.size())
            return "jump past the last step";
    if (out.steps.empty() && out.output_everything < 0) return "empty program";
    return std::string();
}

}  // namespace fcx
