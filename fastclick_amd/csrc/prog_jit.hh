// prog_jit.hh -- decision programs compiled to code (host side, hiprtc).
//
// fcgpu_set_program installs a program in the device step format (table steps
// from build_tables included); k_rx walks it step by step (run_program_on in
// fcgpu_device.hh): a dependent LDS load of every step, a loop back. With
// fcgpu_program_jit the same program is also emitted as straight-line HIP --
// one labelled block per step, the step's offset, mask and value as
// immediates, a table step's jump table as a branch-free chain of compares
// over its runs -- and compiled with hiprtc into the k_rx instantiations the
// context launches, so the kernel runs the program as code. The generated
// function follows run_program_on step for step (availability of the word,
// the partial-word rule, the short branch, the table fallback), so outputs
// are identical; the tests compare both against the oracle.
//
// Programs with a cycle stay interpreted (the interpreter bounds its walk; a
// compiled cycle would not terminate).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>
#include <stdint.h>
#include <algorithm>
#include <map>
#include <string>
#include <vector>

namespace fcgpu {

// k_rx instantiation a compiled module provides: check mode, checksum,
// partition, L4 check, flow table (FAST follows from the check mode).
inline int jit_key(int cm, bool ck, int part, bool l4, bool flow) {
    return cm | (ck ? 4 : 0) | (part << 3) | (l4 ? 32 : 0) | (flow ? 64 : 0);
}

struct JitModule {
    hipModule_t mod = nullptr;
    std::map<int, hipFunction_t> fn;
    void unload() {
        if (mod) (void)hipModuleUnload(mod);
        mod = nullptr;
        fn.clear();
    }
};

// The program as one device function, or "" (why says why) when it has a cycle.
inline std::string jit_program_source(const std::vector<uint4> &dev, uint32_t nsteps, uint32_t tab_q, uint32_t kind,
                                      std::string &why) {
    const bool ipf = kind == FCGPU_PROG_IPFILTER;
    auto table = [&](uint32_t k) { return ((dev[k].x >> 16) & kStepTable) != 0; };
    auto tab = [&](uint32_t i) {
        const uint4 &q = dev[tab_q + i / 8];
        const uint32_t w = (i & 7) < 2 ? q.x : (i & 7) < 4 ? q.y : (i & 7) < 6 ? q.z : q.w;
        return (int32_t)(int16_t)((i & 1) ? w >> 16 : w & 0xffff);
    };
    // successors (positive jumps) of every step, for the cycle check
    std::vector<std::vector<uint32_t>> succ(nsteps);
    for (uint32_t k = 0; k < nsteps; ++k) {
        const uint4 &st = dev[k];
        auto add = [&](int32_t t) {
            if (t > 0) succ[k].push_back((uint32_t)t);
        };
        if (table(k)) {
            add((int32_t)st.w);
            const uint32_t n = 1u << (st.z >> 8);
            for (uint32_t i = 0; i < n; ++i) add(tab(st.y + i));
        } else {
            add((int16_t)(st.w & 0xffff));
            add((int16_t)(st.w >> 16));
        }
    }
    for (auto &v : succ)
        for (uint32_t t : v)
            if (t >= nsteps) {
                why = "program jumps past its steps";
                return "";
            }
    {   // iterative DFS from step 0: a back edge is a cycle
        std::vector<uint8_t> state(nsteps, 0);   // 0 new, 1 on stack, 2 done
        std::vector<std::pair<uint32_t, size_t>> st{{0u, 0u}};
        state[0] = 1;
        while (!st.empty()) {
            auto &[k, i] = st.back();
            if (i < succ[k].size()) {
                const uint32_t t = succ[k][i++];
                if (state[t] == 1) {
                    why = "program has a cycle: it stays interpreted";
                    return "";
                }
                if (state[t] == 0) {
                    state[t] = 1;
                    st.push_back({t, 0u});
                }
            } else {
                state[k] = 2;
                st.pop_back();
            }
        }
    }
    auto jump = [](int32_t t) {
        return t <= 0 ? "return " + std::to_string((uint32_t)(-t)) + "u;" : "goto S" + std::to_string(t) + ";";
    };
    auto bexpr = [&](int off) {
        if (!ipf) return std::to_string(off);
        if (off >= 512) return "(int)an.th + " + std::to_string(off - 512);
        if (off >= 256) return "(int)an.nh + " + std::to_string(off - 256);
        return std::to_string(off - 2);
    };
    std::string s;
    s.reserve(nsteps * 256 + 1024);
    s += "__device__ __forceinline__ uint32_t jit_program(const FrameView &f, const fcgpu_anno &an) {\n";
    if (ipf)
        s += "  const int nl = (int)an.length - (int)an.nh, nhl = (int)an.th - (int)an.nh;\n"
             "  const int plen = nl > nhl ? nl + 512 - nhl : nl + 256;\n";
    else
        s += "  const int plen = (int)an.length;\n";
    for (uint32_t k = 0; k < nsteps; ++k) {
        const uint4 &st = dev[k];
        const int off = (int16_t)(st.x & 0xffff);
        const uint32_t m = st.z;
        const std::string K = std::to_string(k), O = std::to_string(off + 4), B = bexpr(off);
        s += "S" + K + ": {\n";
        if (table(k)) {
            const uint32_t lo = m & 31, w = m >> 8, n = 1u << w;
            s += "  if (plen < " + O + ") goto S" + std::to_string(st.w) + ";\n";
            s += "  const uint32_t idx = (__builtin_bswap32(prog_word(f, " + B + ")) >> " + std::to_string(lo) +
                 ") & " + std::to_string(n - 1) + "u;\n";
            // runs of equal entries -> compares
            std::vector<std::pair<uint32_t, int32_t>> runs;
            for (uint32_t i = 0; i < n; ++i) {
                const int32_t v = tab(st.y + i);
                if (runs.empty() || runs.back().second != v) runs.push_back({i, v});
            }
            s += "  int j = " + std::to_string(runs[0].second) + ";\n";
            for (size_t r = 1; r < runs.size(); ++r)
                s += "  j = idx >= " + std::to_string(runs[r].first) + "u ? " + std::to_string(runs[r].second) +
                     " : j;\n";
            s += "  if (j <= 0) return (uint32_t)(-j);\n  switch (j) {\n";
            std::vector<int32_t> seen;
            for (auto &r : runs)
                if (r.second > 0 && std::find(seen.begin(), seen.end(), r.second) == seen.end()) {
                    seen.push_back(r.second);
                    s += "  case " + std::to_string(r.second) + ": goto S" + std::to_string(r.second) + ";\n";
                }
            s += "  default: return " + std::to_string(kProgUnmatched) + "u;\n  }\n";
        } else {
            const int32_t yes = (int16_t)(st.w & 0xffff), no = (int16_t)(st.w >> 16);
            const bool shorty = (st.x >> 16) & FCGPU_STEP_SHORT_YES;
            const std::string cmp = "((prog_word(f, " + B + ") & " + std::to_string(m) + "u) == " +
                                    std::to_string(st.y) + "u)";
            s += "  if (plen >= " + O + ") { if " + cmp + " " + jump(yes) + " " + jump(no) + " }\n";
            if ((m >> 24) == 0) {
                // the partial-word rule of run_program_on, with the mask's bytes known
                const bool m16 = (m >> 16) & 0xff, m8 = (m >> 8) & 0xff;
                std::string unavail;
                if (m16) unavail += "a <= 2";
                if (m8) unavail += std::string(unavail.empty() ? "" : " || ") + "a == 1";
                s += "  if (plen > " + std::to_string(off) + ") {\n";
                if (!unavail.empty()) s += "    const int a = plen - " + std::to_string(off) + ";\n";
                s += "    if (!(" + (unavail.empty() ? std::string("false") : unavail) + ")) { if " + cmp + " " +
                     jump(yes) + " " + jump(no) + " }\n  }\n";
            }
            s += "  " + jump(shorty ? yes : no) + "\n";
        }
        s += "}\n";
    }
    s += "}\n";
    return s;
}

// The program function and the k_rx instantiations `keys` as one hiprtc
// program; `dev_hh` / `abi_h` are the texts of fcgpu_device.hh and
// fastclick_gpu.h (embedded in the library at build time).
inline bool jit_compile(const std::string &program, const std::vector<int> &keys, const char *dev_hh,
                        const char *abi_h, JitModule &out, std::string &err) {
    std::string src =
        "namespace hi = __hip_internal;\n"
        "typedef hi::uint8_t uint8_t; typedef hi::uint16_t uint16_t; typedef hi::uint32_t uint32_t;\n"
        "typedef hi::uint64_t uint64_t; typedef hi::int8_t int8_t; typedef hi::int16_t int16_t;\n"
        "typedef hi::int32_t int32_t; typedef hi::int64_t int64_t;\n"
        "#define INT32_MIN (-2147483647 - 1)\n"
        "#define FCGPU_JIT_PROGRAM 1\n"
        "#include \"fcgpu_device.hh\"\n"
        "namespace fcgpu {\n" +
        program + "}\n";
    std::vector<std::string> names;
    for (int key : keys) {
        const int cm = key & 3, part = (key >> 3) & 3;
        const bool ck = key & 4, l4 = key & 32, flow = key & 64;
        const bool fast = cm == FCGPU_CHECK_IP4 || cm == FCGPU_CHECK_AUTO;
        std::string n = "fcgpu::k_rx<" + std::to_string(cm) + ", " + (ck ? "true" : "false") + ", " +
                        std::to_string(part) + ", true, " + (l4 ? "true" : "false") + ", " + (flow ? "true" : "false") +
                        ", " + (fast ? "true" : "false") + ">";
        src += "template __global__ void " + n + "(fcgpu::RxLaunch);\n";
        names.push_back(n);
    }
    const char *hdrs[] = {dev_hh, abi_h};
    const char *inc[] = {"fcgpu_device.hh", "../../include/fastclick_gpu.h"};
    hiprtcProgram prog;
    if (hiprtcCreateProgram(&prog, src.c_str(), "fcgpu_jit.hip", 2, hdrs, inc) != HIPRTC_SUCCESS) {
        err = "hiprtcCreateProgram failed";
        return false;
    }
    for (auto &n : names) hiprtcAddNameExpression(prog, n.c_str());
    const char *opts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17", "-Wno-unused-label"};
    const hiprtcResult r = hiprtcCompileProgram(prog, 4, opts);
    if (r != HIPRTC_SUCCESS) {
        size_t ls = 0;
        hiprtcGetProgramLogSize(prog, &ls);
        std::string log(ls, '\0');
        if (ls) hiprtcGetProgramLog(prog, &log[0]);
        err = "hiprtc: " + std::string(hiprtcGetErrorString(r)) + ": " + log.substr(0, 2000);
        hiprtcDestroyProgram(&prog);
        return false;
    }
    size_t cs = 0;
    hiprtcGetCodeSize(prog, &cs);
    std::vector<char> code(cs);
    hiprtcGetCode(prog, code.data());
    std::vector<std::string> lowered;
    for (auto &n : names) {
        const char *l = nullptr;
        hiprtcGetLoweredName(prog, n.c_str(), &l);
        lowered.push_back(l ? l : "");
    }
    hiprtcDestroyProgram(&prog);
    JitModule m;
    if (hipModuleLoadData(&m.mod, code.data()) != hipSuccess) {
        err = "hipModuleLoadData failed";
        return false;
    }
    for (size_t i = 0; i < keys.size(); ++i) {
        hipFunction_t f = nullptr;
        if (lowered[i].empty() || hipModuleGetFunction(&f, m.mod, lowered[i].c_str()) != hipSuccess) {
            err = "compiled program: no kernel " + names[i];
            m.unload();
            return false;
        }
        m.fn[keys[i]] = f;
    }
    out.unload();
    out = m;
    return true;
}

}  // namespace fcgpu
