// host_fuzz.cc -- host-code sanitizer run (TEST INFRASTRUCTURE, CPU only).
//
// SURVEY §5 ("race detection / sanitizers"): the reference builds no
// sanitizer target; this repo runs its host-side parsers and the oracle under
// AddressSanitizer + UndefinedBehaviorSanitizer (tests/test_host_sanitizers.py
// compiles this file with -fsanitize=address,undefined and the product
// sources it exercises). Seeded random and mutated inputs, a time budget:
//   1. the FromDump-compatible pcap reader (pcap_reader.cc): valid files in
//      every header variant (both byte orders, us/ns/modified magic, minor
//      versions 2-4, caplen > len), read through fcpcap_read with random
//      buffer sizes and through fcpcap_map + fcpcap_index, record counts
//      checked; then byte-flipped and truncated copies, which must fail
//      cleanly or read fewer records, never fault;
//   2. the decision-program text parser (program_text.hh) on the reference
//      programs (argv[1]: one program per line, '|' between program lines)
//      and mutations of them;
//   3. the element's keyword parser (RxCore::configure, click_args.hh) on
//      random keyword lists;
//   4. the oracle (fc_oracle.c) on random frames and descriptors for every
//      check mode, classifier, L4 mode and rewrite, and its flow tables.
// Prints "host_fuzz ok <iterations>" and exits 0, or aborts on a finding.
#include <assert.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <chrono>
#include <fstream>
#include <random>
#include <string>
#include <vector>

#include "../include/fcpcap.h"
#include "../oracle/fc_oracle.h"
#include "../fastclick_amd/csrc/host/gpu_element.hh"

using Rng = std::mt19937_64;

#define CHECK(c)                                                                      \
    do {                                                                              \
        if (!(c)) {                                                                   \
            fprintf(stderr, "host_fuzz: check failed at %s:%d: %s\n", __FILE__, __LINE__, #c); \
            abort();                                                                  \
        }                                                                             \
    } while (0)

static uint32_t bswap(uint32_t x) { return __builtin_bswap32(x); }

// ---- 1. pcap reader ---------------------------------------------------------
struct PcapSpec {
    uint32_t magic;     // 0xa1b2c3d4 us, 0xa1b23c4d ns, 0xa1b2cd34 modified (8 extra record bytes)
    bool swapped;
    uint16_t minor;
};

static std::vector<uint8_t> make_pcap(Rng &rng, const PcapSpec &sp, uint32_t nrec, uint32_t &expect) {
    std::vector<uint8_t> f;
    auto put32 = [&](uint32_t v) {
        if (sp.swapped) v = bswap(v);
        uint8_t b[4];
        memcpy(b, &v, 4);
        f.insert(f.end(), b, b + 4);
    };
    auto put16 = [&](uint16_t v) {
        if (sp.swapped) v = (uint16_t)((v >> 8) | (v << 8));
        uint8_t b[2];
        memcpy(b, &v, 2);
        f.insert(f.end(), b, b + 2);
    };
    put32(sp.magic);
    put16(2);
    put16(sp.minor);
    put32(0);
    put32(0);
    put32(65535);
    put32(1);
    const bool extra = sp.magic == 0xa1b2cd34u;
    expect = nrec;
    for (uint32_t i = 0; i < nrec; ++i) {
        uint32_t len = 14 + (uint32_t)(rng() % 1500);
        uint32_t cap = (uint32_t)(rng() % 4 == 0 ? len + rng() % 64 : rng() % (len + 1));   // sometimes caplen > len
        if (cap > 2000) cap = 2000;
        // a 2.3 file with caplen > len is read with the two swapped (FromDump's
        // rule for files written by old libpcaps): not a valid file of this shape
        if (sp.minor == 3 && cap > len) cap = len;
        // header fields as FromDump reads them: before 2.3 the two are swapped
        const bool old = sp.minor < 3;
        put32((uint32_t)(rng() % 100000));
        put32((uint32_t)(rng() % 1000000));
        put32(old ? len : cap);
        put32(old ? cap : len);
        if (extra) { put32(0); put32(0); }
        for (uint32_t k = 0; k < cap; ++k) f.push_back((uint8_t)rng());
    }
    return f;
}

static std::string write_tmp(const std::vector<uint8_t> &bytes) {
    char path[] = "/tmp/fc_host_fuzz_XXXXXX";
    const int fd = mkstemp(path);
    CHECK(fd >= 0);
    size_t done = 0;
    while (done < bytes.size()) {
        const ssize_t k = write(fd, bytes.data() + done, bytes.size() - done);
        CHECK(k > 0);
        done += (size_t)k;
    }
    close(fd);
    return path;
}

// Reads the whole file; returns the record count, or -1 if the reader
// reported an error (a valid outcome for a corrupted file).
static long read_all(const std::string &path, Rng &rng, bool small_bufs, bool mapped) {
    fcpcap *r = nullptr;
    char err[256];
    if (fcpcap_open(path.c_str(), &r, err, sizeof err) != 0) return -1;
    fcpcap_set_threads(r, 1 + (unsigned)(rng() % 3));
    long total = 0;
    const uint32_t max = 1 + (uint32_t)(rng() % 300);
    std::vector<uint32_t> desc(2 * max), wire(max);
    std::vector<uint64_t> ts(max);
    if (mapped) {
        const uint8_t *base = nullptr;
        size_t bytes = 0;
        if (fcpcap_map(r, &base, &bytes) != 0) { fcpcap_close(r); return -1; }
        for (int it = 0; it < 1000000; ++it) {
            size_t off = 0, cb = 0;
            const int n = fcpcap_index(r, max, 64 + rng() % (1 << 20), &off, &cb, desc.data(), wire.data(), ts.data());
            if (n < 0) { total = -1; break; }
            if (n == 0) break;
            CHECK(off + cb <= bytes);
            for (int i = 0; i < n; ++i) {
                CHECK((size_t)desc[2 * i] + desc[2 * i + 1] <= cb);
                volatile uint8_t x = 0;
                if (desc[2 * i + 1]) x = base[off + desc[2 * i] + desc[2 * i + 1] - 1];   // in the mapping
                (void)x;
            }
            total += n;
        }
    } else {
        const size_t cap = small_bufs ? 16 + rng() % 4096 : 70000 + rng() % (1 << 20);
        std::vector<uint8_t> buf(cap);
        for (int it = 0; it < 1000000; ++it) {
            size_t used = 0;
            const int n = fcpcap_read(r, buf.data(), cap, desc.data(), wire.data(), ts.data(), max, &used);
            if (n < 0) { total = -1; break; }
            if (n == 0) break;
            CHECK(used <= cap);
            for (int i = 0; i < n; ++i) CHECK((size_t)desc[2 * i] + desc[2 * i + 1] <= used);
            total += n;
        }
    }
    fcpcap_close(r);
    return total;
}

static void fuzz_pcap(Rng &rng) {
    static const uint32_t magics[] = {0xa1b2c3d4u, 0xa1b23c4du, 0xa1b2cd34u};
    PcapSpec sp{magics[rng() % 3], (rng() & 1) != 0, (uint16_t)(2 + rng() % 3)};
    uint32_t expect = 0;
    auto f = make_pcap(rng, sp, (uint32_t)(rng() % 400), expect);
    const std::string p = write_tmp(f);
    CHECK(read_all(p, rng, false, false) == (long)expect);
    CHECK(read_all(p, rng, false, true) == (long)expect);
    read_all(p, rng, true, false);   // tiny buffers: a record may not fit (an error), never a fault
    unlink(p.c_str());
    // corrupted copies
    for (int m = 0; m < 4; ++m) {
        auto g = f;
        const int kind = (int)(rng() % 3);
        if (kind == 0 && !g.empty()) {
            for (int k = 0; k < 1 + (int)(rng() % 8); ++k) g[rng() % g.size()] ^= (uint8_t)(1u << (rng() % 8));
        } else if (kind == 1 && !g.empty()) {
            g.resize(rng() % g.size());
        } else {
            for (int k = 0; k < 4 && g.size() > 24; ++k) g[24 + rng() % (g.size() - 24)] = 0xff;   // huge caplen bytes
        }
        const std::string q = write_tmp(g);
        const long a = read_all(q, rng, false, false);
        const long b = read_all(q, rng, false, true);
        CHECK(a <= (long)expect + 100000 && b <= (long)expect + 100000);
        unlink(q.c_str());
    }
}

// The mapped index of one file, one call at a time: every call's outcome.
static std::vector<std::vector<uint64_t>> index_calls(const std::string &path, unsigned threads, uint32_t max,
                                                      size_t max_bytes) {
    std::vector<std::vector<uint64_t>> calls;
    fcpcap *r = nullptr;
    char err[256];
    if (fcpcap_open(path.c_str(), &r, err, sizeof err) != 0) return calls;
    fcpcap_set_threads(r, threads);
    const uint8_t *base = nullptr;
    size_t bytes = 0;
    CHECK(fcpcap_map(r, &base, &bytes) == 0);
    std::vector<uint32_t> desc(2ull * max), wire(max);
    std::vector<uint64_t> ts(max);
    for (int it = 0; it < 100000; ++it) {
        size_t off = 0, cb = 0;
        const int n = fcpcap_index(r, max, max_bytes, &off, &cb, desc.data(), wire.data(), ts.data());
        std::vector<uint64_t> c{(uint64_t)(int64_t)n, off, cb};
        for (int i = 0; i < n; ++i) {
            CHECK((size_t)desc[2 * i] + desc[2 * i + 1] <= cb && off + cb <= bytes);
            c.insert(c.end(), {desc[2 * i], desc[2 * i + 1], wire[i], ts[i]});
        }
        calls.push_back(c);
        if (n <= 0) break;
    }
    fcpcap_close(r);
    return calls;
}

// The parallel mapped index (fcpcap_set_threads > 1, chunks of >= 8 MiB) is
// the one-thread walk, call for call -- on a ~20 MB file and on copies with
// flipped bits and forced huge caplens. Once per run (under ThreadSanitizer
// this is the check that its threads share nothing but the read-only map).
static void check_parallel_index(Rng &rng) {
    for (int v = 0; v < 3; ++v) {
        PcapSpec sp{v == 1 ? 0xa1b23c4du : 0xa1b2c3d4u, v == 2, 4};
        uint32_t expect = 0;
        auto f = make_pcap(rng, sp, 26000, expect);
        if (v) {
            for (int k = 0; k < 40; ++k) f[24 + rng() % (f.size() - 24)] ^= (uint8_t)(1u << (rng() % 8));
            if (v == 2) f[f.size() / 2] = 0xff;
        }
        const std::string p = write_tmp(f);
        for (size_t mb : {(size_t)9 << 20, (size_t)16 << 20}) {
            const auto ref = index_calls(p, 1, 1u << 20, mb);
            for (unsigned t : {2u, 4u, 7u}) CHECK(index_calls(p, t, 1u << 20, mb) == ref);
        }
        unlink(p.c_str());
    }
}

// ---- 2. decision-program text -------------------------------------------------
static void fuzz_program(Rng &rng, const std::vector<std::string> &progs) {
    if (progs.empty()) return;
    const std::string &p = progs[rng() % progs.size()];
    fcx::ParsedProgram out;
    std::string text = p;
    for (char &c : text)
        if (c == '|') c = '\n';
    CHECK(fcx::parse_program(text, out).empty());
    CHECK(!out.steps.empty() || out.output_everything >= 0);
    static const char alphabet[] = "0123456789abcdef []/%-+>X|\nstepyesnoshort";
    for (int m = 0; m < 8; ++m) {
        std::string t = text;
        const int kind = (int)(rng() % 4);
        if (t.empty()) break;
        const size_t at = rng() % t.size();
        if (kind == 0) t.erase(at, 1 + rng() % 4);
        else if (kind == 1) t.insert(at, 1, alphabet[rng() % (sizeof alphabet - 1)]);
        else if (kind == 2) t[at] = alphabet[rng() % (sizeof alphabet - 1)];
        else t.resize(at);
        fcx::ParsedProgram o2;
        const std::string e = fcx::parse_program(t, o2);
        if (e.empty())   // accepted: every jump stays inside the program
            for (const auto &st : o2.steps) CHECK(st.yes < (int32_t)o2.steps.size() && st.no < (int32_t)o2.steps.size());
    }
}

// ---- 3. element keywords --------------------------------------------------------
static void fuzz_keywords(Rng &rng) {
    static const char *keys[] = {"OFFSET", "CHECKSUM", "BADSRC", "GOODDST", "VERBOSE", "DETAILS", "NATIVE_VLAN",
                                 "VLAN_ETHERTYPE", "MODE", "BADADDRS", "PROCESS_EH", "N", "LB_MODE", "HASHSWITCH",
                                 "PROGRAM", "PROGRAM_KIND", "PROGRAM_JIT", "L4", "L4_CHECKSUM", "COLOR",
                                 "FLOW_CAPACITY", "FLOWID_ANNO", "FLOW_RUNS", "FLOW_MANAGER", "FLOW_TIMEOUT",
                                 "FLOW_RECYCLE_INTERVAL", "DEC_TTL", "TTL_MULTICAST", "SET_CHECKSUM", "HASH",
                                 "STRIP", "DEVICE", "BATCH", "TIMER", "PARTITION", "INTERFACES", "CST_BUCKETS", "BOGUS"};
    static const char *vals[] = {"", "0", "1", "14", "-1", "65536", "4294967296", "true", "false", "yes", "0x10",
                                 "1.2.3.4", "1.2.3.4 5.6.7.8", "256.1.1.1", "hash", "hash_ip", "hash_crc", "hash_agg",
                                 "chash", "cst_hash_agg", "rr", "16777217",
                                 "AUTO", "MARK", "MARK6", "CHECK", "UDP", "TCP", "IMP", "HMP", "TILE", "GLOBAL",
                                 "\"14 4\"", "14 4", "IPFILTER", "CLASSIFIER", "0.001", "65.536", "1e9", "x",
                                 "\"0 12/00000000%00000000 yes->[0] no->[1]\"", "99999999999999999999",
                                 "18.26.4.9/24 1.0.0.1/255.0.0.0", "18.26/24", "18.26.4/24", "1.2.3.4/", "/8",
                                 "1.2.3.4/33", "1.2.3.4/255.0", "1.2.3.4 5.6.7.8 9.9.9.9 1.1.1.1 2.2.2.2 3.3.3.3 "
                                 "4.4.4.4 5.5.5.5 6.6.6.6 7.7.7.7 8.8.8.8 9.9.9.8 1.1.1.2 1.1.1.3 1.1.1.4"};
    std::vector<std::string> conf;
    const int n = (int)(rng() % 8);
    for (int i = 0; i < n; ++i)
        conf.push_back(std::string(keys[rng() % (sizeof keys / sizeof *keys)]) + " " +
                       vals[rng() % (sizeof vals / sizeof *vals)]);
    if (rng() % 4 == 0) {   // raw noise through the Args splitter
        std::string s;
        for (int i = 0; i < (int)(rng() % 40); ++i) s += (char)(32 + rng() % 95);
        for (const auto &a : fcx::split_conf(s)) conf.push_back(a);
    }
    fcx::RxCore<fcx::ModelPolicy> core;
    std::string err;
    core.configure(conf, err);   // accepted or rejected with a message; never a fault
    long v;
    uint32_t ip;
    for (const auto &c : conf) {
        fcx::parse_int(c, v);
        fcx::parse_ip4(c, ip);
        fcx::parse_arg(c);
    }
}

// ---- 4. oracle ---------------------------------------------------------------------
static void fuzz_oracle(Rng &rng, const std::vector<std::string> &progs) {
    const uint32_t n = 1 + (uint32_t)(rng() % 700);
    std::vector<uint32_t> desc(2 * n);
    size_t pos = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t len = (uint32_t)(rng() % 4 ? 20 + rng() % 120 : rng() % 1600);
        desc[2 * i] = (uint32_t)pos;
        desc[2 * i + 1] = len;
        pos += len + (rng() % 3);
    }
    std::vector<uint8_t> arena(pos + 256);
    for (auto &b : arena) b = (uint8_t)rng();
    // make many frames plausible: Ethernet(+VLAN) + IPv4/IPv6 headers with sane fields
    for (uint32_t i = 0; i < n; ++i) {
        uint8_t *f = arena.data() + desc[2 * i];
        const uint32_t len = desc[2 * i + 1];
        if (len < 60 || rng() % 4 == 0) continue;
        uint32_t o = 14;
        if (rng() % 3 == 0) { f[12] = 0x81; f[13] = 0x00; o = 18; f[16] = 0x08; f[17] = 0x00; }
        else { f[12] = 0x08; f[13] = 0x00; }
        if (rng() % 4 == 0 && len >= o + 48) {
            f[o] = 0x60;
            const uint32_t pl = len - o - 40;
            f[o + 4] = (uint8_t)(pl >> 8);
            f[o + 5] = (uint8_t)pl;
            f[o + 6] = (uint8_t)(rng() % 2 ? 17 : 6);
        } else {
            f[o] = (uint8_t)(0x40 | (5 + rng() % 3));
            const uint32_t il = len - o - (uint32_t)(rng() % 3);
            f[o + 2] = (uint8_t)(il >> 8);
            f[o + 3] = (uint8_t)il;
            f[o + 6] = (uint8_t)(rng() % 3 ? 0 : rng());
            f[o + 9] = (uint8_t)(rng() % 2 ? 17 : 6);
        }
    }
    fcgpu_cfg cfg;
    fcgpu_default_cfg(&cfg);
    cfg.check_mode = (uint32_t)(rng() % 4);
    cfg.offset = cfg.check_mode == FCGPU_CHECK_AUTO ? 0 : (uint32_t)(rng() % 4 ? 14 : rng() % 40);
    cfg.checksum = (uint32_t)(rng() & 1);
    cfg.hash_mode = (uint32_t)(rng() % 3);
    cfg.nports = 1 + (uint32_t)(rng() % 64);
    cfg.classify = (uint32_t)(rng() % 6);
    cfg.hs_offset = (uint32_t)(rng() % 80);
    cfg.hs_length = 1 + (uint32_t)(rng() % 16);
    if (cfg.check_mode == FCGPU_CHECK_IP4 || cfg.check_mode == FCGPU_MARK_IP4) {
        cfg.l4_mode = (uint32_t)(rng() % 3);
        cfg.l4_checksum = (uint32_t)(rng() & 1);
        cfg.rewrite = (uint32_t)(rng() % 4);
    }
    fcx::ParsedProgram prog;
    if (cfg.classify == FCGPU_CLS_PROGRAM) {
        if (progs.empty()) {
            cfg.classify = FCGPU_CLS_LB_HASH;
        } else {
            std::string text = progs[rng() % progs.size()];
            for (char &c : text)
                if (c == '|') c = '\n';
            CHECK(fcx::parse_program(text, prog).empty());
            fco_set_program((uint32_t)(rng() & 1), prog.steps.data(), (uint32_t)prog.steps.size(),
                            prog.output_everything);
        }
    }
    std::vector<uint16_t> verdict(n), tile_count((size_t)(n + 255) / 256 * (cfg.nports + 1));
    std::vector<uint32_t> hash(n), perm(n), start(cfg.nports + 2), perm_tile(n), ip_rw(n), fid(n);
    std::vector<fcgpu_anno> anno(n);
    std::vector<uint64_t> ctr(FCGPU_NCOUNTERS, 0);
    fco_process_batch2(&cfg, arena.data(), desc.data(), n, verdict.data(), hash.data(), anno.data(), perm.data(),
                       start.data(), perm_tile.data(), tile_count.data(), ctr.data(), ip_rw.data());
    // the partition is a permutation
    std::vector<uint8_t> seen(n, 0);
    for (uint32_t i = 0; i < n; ++i) {
        CHECK(perm[i] < n && !seen[perm[i]]);
        seen[perm[i]] = 1;
    }
    if (cfg.check_mode == FCGPU_CHECK_IP4 || cfg.check_mode == FCGPU_MARK_IP4) {
        fco_flowtab *t = fco_flow_new(1 + (uint32_t)(rng() % 600));
        fco_flow_batch(t, arena.data(), desc.data(), n, verdict.data(), anno.data(), fid.data());
        fco_flow_batch(t, arena.data(), desc.data(), n, verdict.data(), anno.data(), fid.data());
        fco_flow_free(t);
        fco_imp *m = fco_imp_new(1 + (uint32_t)(rng() % 600), (uint32_t)(rng() % 3), 100 + (uint32_t)(rng() % 900));
        uint32_t now = 1000;
        for (int k = 0; k < 4; ++k) {
            fco_imp_batch(m, arena.data(), desc.data(), n, verdict.data(), anno.data(), now, fid.data());
            now += (uint32_t)(rng() % 2000);
            fco_imp_maintain(m, now);
        }
        uint32_t c, fr, pe;
        fco_imp_stats(m, &c, &fr, &pe);
        fco_imp_free(m);
    }
}

int main(int argc, char **argv) {
    std::vector<std::string> progs;
    if (argc > 1) {
        std::ifstream in(argv[1]);
        std::string line;
        while (std::getline(in, line))
            if (!line.empty()) progs.push_back(line);
    }
    const double budget = argc > 2 ? atof(argv[2]) : 5.0;
    Rng rng(argc > 3 ? strtoull(argv[3], nullptr, 10) : 12345);
    const auto t0 = std::chrono::steady_clock::now();
    check_parallel_index(rng);
    long it = 0;
    for (;; ++it) {
        fuzz_pcap(rng);
        for (int k = 0; k < 8; ++k) fuzz_program(rng, progs);
        for (int k = 0; k < 8; ++k) fuzz_keywords(rng);
        fuzz_oracle(rng, progs);
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > budget) break;
    }
    printf("host_fuzz ok %ld\n", it + 1);
    return 0;
}
