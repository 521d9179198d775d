// fcgpu_program.hip -- decision programs (FCGPU_CLS_PROGRAM: IPFilter /
// IPClassifier / Classifier): upload with jump tables
// (build_tables), compiled programs (fcgpu_program_jit, hiprtc through
// prog_jit.hh), and the LoadBalancer hash tables (FCGPU_CLS_LB_TABLE).
#include "fcgpu_internal.hh"
#include "jit_sources.inc"   // kJitDeviceHh, kJitAbiH (fastclick_amd/build.py)

using namespace fcgpu;
using namespace fcgpu_rt;

namespace fcgpu_rt {

// Jump tables for runs of steps that test one word (SURVEY 8(a) A11 programs:
// a rule's fields, and above all a port range the reference's compiler splits
// into a chain of mask tests on the transport word). Lanes of a wave walking
// such a chain for different port values leave it at different steps; a
// table gives every lane the chain's outcome in one step. For each entry step
// e (step 0, and every step reached by a jump from a step at another offset)
// the run R(e) = steps reachable from e through steps at e's offset. If the
// bits R's masks test span at most kTabBits bits of the big-endian word, e
// becomes a table step: tab[(bswap(word) >> lo) & (2^w - 1)] = where a walk
// from e with that word leaves R (an output <= 0 or a step outside R), and
// its original step is appended as the fallback for words that are not
// entirely inside the packet (the length-checked rules decide those). The
// steps keep their indices; dev grows by the fallback copies and the tables.
// Returns the step count (copies included); tab_q = uint4 index of the tables.
static uint32_t build_tables(std::vector<uint4> &dev, uint32_t nsteps, uint32_t &tab_q) {
    constexpr uint32_t kTabBits = 8, kTabBudget = 2048;     // entries per table, in total
    auto off_of = [&](uint32_t k) { return (int16_t)(dev[k].x & 0xffff); };
    auto yes_of = [&](const uint4 &st) { return (int32_t)(int16_t)(st.w & 0xffff); };
    auto no_of = [&](const uint4 &st) { return (int32_t)(int16_t)(st.w >> 16); };
    std::vector<char> entry(nsteps, 0);
    entry[0] = 1;
    for (uint32_t k = 0; k < nsteps; ++k)
        for (int32_t t : {yes_of(dev[k]), no_of(dev[k])})
            if (t > 0 && off_of((uint32_t)t) != off_of(k)) entry[t] = 1;
    std::vector<uint4> copies;
    std::vector<uint16_t> tabs;
    std::vector<int> inr(nsteps, -1);
    for (uint32_t e = 0; e < nsteps; ++e) {
        if (!entry[e]) continue;
        // the run from e
        std::vector<uint32_t> run{e}, todo{e};
        inr[e] = (int)e;
        uint32_t mbe = 0;
        while (!todo.empty()) {
            const uint32_t k = todo.back();
            todo.pop_back();
            mbe |= __builtin_bswap32(dev[k].z);
            for (int32_t t : {yes_of(dev[k]), no_of(dev[k])})
                if (t > 0 && inr[t] != (int)e && off_of((uint32_t)t) == off_of(e)) {
                    inr[t] = (int)e;
                    run.push_back((uint32_t)t);
                    todo.push_back((uint32_t)t);
                }
        }
        if (run.size() < 2 || mbe == 0) continue;
        const uint32_t lo = __builtin_ctz(mbe), w = 32 - __builtin_clz(mbe) - lo;
        if (w > kTabBits || tabs.size() + (1u << w) > kTabBudget) continue;
        const uint32_t base = (uint32_t)tabs.size();
        for (uint32_t idx = 0; idx < (1u << w); ++idx) {
            const uint32_t word = __builtin_bswap32(idx << lo);   // the packet word as the device loads it
            int32_t pos = (int32_t)e, j = -kProgUnmatched;
            for (size_t hops = 0; hops <= run.size(); ++hops) {
                const uint4 &st = dev[pos];
                j = (word & st.z) == st.y ? yes_of(st) : no_of(st);
                if (j <= 0 || inr[j] != (int)e) break;
                pos = j;
                j = -kProgUnmatched;                                // a cycle inside the run
            }
            tabs.push_back((uint16_t)(int16_t)j);
        }
        copies.push_back(dev[e]);
        const uint32_t copy_at = nsteps + (uint32_t)copies.size() - 1;
        dev[e].x = (dev[e].x & 0xffffu) | (kStepTable << 16);
        dev[e].y = base;
        dev[e].z = lo | (w << 8);
        dev[e].w = copy_at;
    }
    dev.resize(nsteps);
    dev.insert(dev.end(), copies.begin(), copies.end());
    tab_q = (uint32_t)dev.size();
    tabs.resize((tabs.size() + 7) & ~(size_t)7, 0);
    for (size_t k = 0; k < tabs.size(); k += 8) {
        uint4 q;
        q.x = tabs[k] | (uint32_t)tabs[k + 1] << 16;
        q.y = tabs[k + 2] | (uint32_t)tabs[k + 3] << 16;
        q.z = tabs[k + 4] | (uint32_t)tabs[k + 5] << 16;
        q.w = tabs[k + 6] | (uint32_t)tabs[k + 7] << 16;
        dev.push_back(q);
    }
    return nsteps + (uint32_t)copies.size();
}

// ---- compiled programs (fcgpu_program_jit, prog_jit.hh) ---------------------
// The k_rx instantiations the context's configuration launches (as the
// launch_rx_part dispatch normalises them), for every partition shape.
static std::vector<int> jit_keys_for(const fcgpu_ctx *c) {
    int cm = (int)c->cfg.check_mode;
    bool ck = c->cfg.checksum != 0;
    if (cm == FCGPU_MARK_IP4 || cm == FCGPU_MARK_IP6) ck = false;
    const bool ip4 = cm == FCGPU_CHECK_IP4 || cm == FCGPU_MARK_IP4;
    const bool l4 = ip4 && c->cfg.l4_mode != FCGPU_L4_NONE, flow = ip4 && c->fl.slots != nullptr;
    std::vector<int> keys;
    for (int part : {kPartTile, kPartNone, kPartGlobal}) keys.push_back(jit_key(cm, ck, part, l4, flow));
    return keys;
}

// (Re)build the module for the installed program and `keys`.
static int jit_build(fcgpu_ctx *c, const std::vector<int> &keys) {
    std::string err;
    HIPCHK(c, hipSetDevice(c->device));
    // launches of the module being replaced may still run
    HIPCHK(c, hipDeviceSynchronize());
    if (!jit_compile(c->jit_src, keys, kJitDeviceHh, kJitAbiH, c->jit, err)) {
        c->jit_src.clear();
        c->jit_keys.clear();
        return fail(c, FCGPU_ERUNTIME, "fcgpu_program_jit: " + err);
    }
    c->jit_keys = keys;
    return FCGPU_OK;
}

// The installed program as code: generated and compiled for the current
// configuration; a program with a cycle stays interpreted (error returned).
static int jit_install(fcgpu_ctx *c) {
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipDeviceSynchronize());      // no launch of the old module still running
    c->jit.unload();
    c->jit_src.clear();
    c->jit_keys.clear();
    if (!c->jit_on || c->prog_all >= 0 || c->prog_dev.empty()) return FCGPU_OK;
    std::string why;
    c->jit_src = jit_program_source(c->prog_dev, c->prog_n, c->prog_tab, c->prog_kind, why);
    if (c->jit_src.empty()) return fail(c, FCGPU_EINVAL, "fcgpu_program_jit: " + why);
    return jit_build(c, jit_keys_for(c));
}

// The compiled kernel for an instantiation; one the module lacks (the
// configuration changed since) is added by recompiling. nullptr: interpret.
hipFunction_t jit_function(fcgpu_ctx *c, int key) {
    auto it = c->jit.fn.find(key);
    if (it != c->jit.fn.end()) return it->second;
    // a rebuild replaces the module, whose functions this context's queued
    // shared-queue submissions hold until they launch: interpret instead
    // (identical results) while one is queued
    if (agg_queued(c)) return nullptr;
    std::vector<int> keys = c->jit_keys;
    keys.push_back(key);
    if (jit_build(c, keys) != FCGPU_OK) return nullptr;
    it = c->jit.fn.find(key);
    return it == c->jit.fn.end() ? nullptr : it->second;
}

}  // namespace fcgpu_rt

extern "C" {

int fcgpu_set_program(fcgpu_ctx *c, uint32_t kind, const fcgpu_step *steps, uint32_t nsteps,
                      int32_t output_everything) {
    if (!c) return FCGPU_EINVAL;
    if (kind > FCGPU_PROG_CLASSIFIER) return fail(c, FCGPU_EINVAL, "bad program kind");
    if (nsteps > FCGPU_MAX_STEPS || (nsteps && !steps)) return fail(c, FCGPU_EINVAL, "bad program size");
    if (nsteps == 0 && output_everything < 0) return fail(c, FCGPU_EINVAL, "empty program without output");
    if (agg_queued(c)) return fail(c, FCGPU_EINVAL, "fcgpu_set_program: a queued span submission is not waited for");
    std::vector<uint4> dev(nsteps ? nsteps : 1);
    auto jump = [](int32_t j) -> int32_t {       // [X] (drop) and out-of-range -> unmatched
        if (j <= -32767 || j > 32767) return -kProgUnmatched;
        return j;
    };
    for (uint32_t k = 0; k < nsteps; ++k) {
        const fcgpu_step &st = steps[k];
        if (st.offset < -32768 || st.offset > 32767) return fail(c, FCGPU_EINVAL, "step offset out of range");
        const int32_t y = jump(st.yes), n = jump(st.no);
        if (y > (int32_t)nsteps - 1 || n > (int32_t)nsteps - 1) return fail(c, FCGPU_EINVAL, "jump past the program");
        dev[k].x = (uint32_t)(uint16_t)st.offset | ((st.flags & FCGPU_STEP_SHORT_YES) << 16);
        dev[k].y = st.value & st.mask;
        dev[k].z = st.mask;
        dev[k].w = (uint32_t)(uint16_t)y | ((uint32_t)(uint16_t)n << 16);
    }
    uint32_t tab_q = 0;
    const uint32_t total_n = nsteps ? build_tables(dev, nsteps, tab_q) : 0;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipDeviceSynchronize());
    // the new program is uploaded before the old one is freed: a failure
    // leaves the context's program (and the device config naming it) intact
    uint4 *np = nullptr;
    if (int rc = alloc_or_fail(c, "fcgpu_set_program", {dev_buf(np, sizeof(uint4) * dev.size())})) return rc;
    if (hipError_t e = hipMemcpy(np, dev.data(), sizeof(uint4) * dev.size(), hipMemcpyHostToDevice)) {
        (void)hipFree(np);
        return fail(c, FCGPU_ERUNTIME, std::string("fcgpu_set_program upload: ") + hipGetErrorString(e));
    }
    hipFree(c->d_prog);
    c->d_prog = np;
    c->prog_host.assign(steps, steps + nsteps);
    c->prog_n = total_n;
    c->prog_q = (uint32_t)dev.size();
    c->prog_tab = tab_q;
    c->dcfg.prog_q = c->prog_q;
    c->dcfg.prog_tab = c->prog_tab;
    c->prog_kind = kind;
    c->prog_all = nsteps == 0 ? output_everything : -1;
    c->dcfg.prog = c->d_prog;
    c->dcfg.prog_n = c->prog_n;
    c->dcfg.prog_kind = c->prog_kind;
    c->dcfg.prog_all = c->prog_all;
    c->prog_dev = dev;
    // contents, not the device copy: contexts with one program share launches
    uint64_t key = 1469598103934665603ull;
    auto mix = [&key](uint32_t v) {
        for (int b = 0; b < 4; ++b) key = (key ^ ((v >> (8 * b)) & 0xff)) * 1099511628211ull;
    };
    for (const uint4 &q : dev) {
        mix(q.x);
        mix(q.y);
        mix(q.z);
        mix(q.w);
    }
    for (uint32_t v : {c->prog_n, c->prog_q, c->prog_tab, c->prog_kind, (uint32_t)c->prog_all}) mix(v);
    c->prog_key = key | 1;
    if (c->jit_on && jit_install(c) != FCGPU_OK) c->err.clear();   // a cycle: interpreted
    return FCGPU_OK;
}

// Server i at cantor(i, j) % size (include/click/algorithm.hh:136-138,
// unsigned) for j < ((size - 1) / nsel) + 1, later placements winning; an
// empty bucket takes the last server placed before it (server 0 before the
// first).
int fcgpu_lb_hash_ring(uint32_t nsel, uint32_t size, uint8_t *out) {
    if (nsel < 1 || nsel > FCGPU_MAX_PORTS || size < 1 || size > FCGPU_LB_TABLE_MAX || !out) return FCGPU_EINVAL;
    std::vector<uint32_t> ring(size, 0xffffffffu);
    const uint32_t fac = (size - 1) / nsel + 1;
    for (uint32_t j = 0; j < fac; ++j)
        for (uint32_t i = 0; i < nsel; ++i) ring[(((i + j) * (i + j + 1)) / 2 + j) % size] = i;
    uint32_t cur = 0;
    for (uint32_t i = 0; i < size; ++i) {
        if (ring[i] != 0xffffffffu) cur = ring[i];
        out[i] = (uint8_t)cur;
    }
    return FCGPU_OK;
}

int fcgpu_set_lb_table(fcgpu_ctx *c, const uint8_t *table, uint32_t nbuckets) {
    if (!c) return FCGPU_EINVAL;
    if (!table || nbuckets == 0 || nbuckets > FCGPU_LB_TABLE_MAX) return fail(c, FCGPU_EINVAL, "bad LB table size");
    if (agg_queued(c)) return fail(c, FCGPU_EINVAL, "fcgpu_set_lb_table: a queued span submission is not waited for");
    // ((h >> 16) ^ (h & 0xffff)) < 65536: entries past 65535 are never read
    const uint32_t n = std::min(nbuckets, 65536u);
    uint32_t mx = 0;
    for (uint32_t k = 0; k < n; ++k) mx = std::max(mx, (uint32_t)table[k]);
    if (c->configured && mx >= c->cfg.nports) return fail(c, FCGPU_EINVAL, "LB table output >= nports");
    // k_rx copies whole uint4s of it into LDS: zero-padded to 16 B
    std::vector<uint8_t> dev((n + 15u) & ~15u, 0);
    memcpy(dev.data(), table, n);
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipDeviceSynchronize());
    // uploaded before the old table is freed: a failure leaves it intact
    uint8_t *nt = nullptr;
    if (int rc = alloc_or_fail(c, "fcgpu_set_lb_table", {dev_buf(nt, dev.size())})) return rc;
    if (hipError_t e = hipMemcpy(nt, dev.data(), dev.size(), hipMemcpyHostToDevice)) {
        (void)hipFree(nt);
        return fail(c, FCGPU_ERUNTIME, std::string("fcgpu_set_lb_table upload: ") + hipGetErrorString(e));
    }
    hipFree(c->d_lbtab);
    c->d_lbtab = nt;
    c->lbtab_n = n;
    c->lbtab_max = mx;
    uint64_t key = 1469598103934665603ull;
    for (uint32_t k = 0; k < n; ++k) key = (key ^ table[k]) * 1099511628211ull;
    c->lbtab_key = (key ^ n) | 1;
    DevCfg &d = c->dcfg;
    d.lb_tab = c->cfg.classify == FCGPU_CLS_LB_TABLE ? c->d_lbtab : nullptr;
    d.lb_tab_n = n;
    d.lb_tab_magic = n > 1 ? (uint32_t)((((uint64_t)1 << 32) + n - 1) / n) : 0u;
    return FCGPU_OK;
}

int fcgpu_program_jit(fcgpu_ctx *c, int enable) {
    if (!c) return FCGPU_EINVAL;
    if (agg_queued(c)) return fail(c, FCGPU_EINVAL, "fcgpu_program_jit: a queued span submission is not waited for");
    c->jit_on = enable != 0;
    return jit_install(c);
}

int fcgpu_program_jit_active(fcgpu_ctx *c) { return c && !c->jit_src.empty() ? 1 : 0; }

}  // extern "C"
