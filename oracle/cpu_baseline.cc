// cpu_baseline.cc -- TEST INFRASTRUCTURE ONLY: the reported CPU baseline.
//
// Scalar restatement of the reference CPU pipeline the GPU element replaces,
// run the way FastClick runs it:
//   ReplayUnqueue-style source (preloaded trace, BURST 32 linked-list
//   PacketBatches) -> Strip(14) -> CheckIPHeader(CHECKSUM true)
//   -> AggregateHash -> FlowSwitch LB_MODE hash (16 outputs, CLASSIFY_EACH_PACKET)
//   -> Discard (packets recycled)
// Per-element atomic counters as CheckIPHeader's atomic_uint64_t _count
// (checkipheader.hh:160-162); one independent pipeline per thread, like
// `click -j N` with StaticThreadSched. Packet semantics from
// fastclick_amd/csrc/host/click_model.hh; per-packet functions from the C
// oracle (fc_oracle.c). Only bench.py's cpu_baseline leg and tests run this.
//
//   fc_cpu_baseline --seconds S --threads T [--flows K] [--program FILE]
//                   [--l4 udp] [--flow-capacity C] [--imix] [--trace N]
//       -> one JSON line. With --program, the classify stage is an IPClassifier
//       running the given program (reference `program` handler text) instead
//       of FlowSwitch: IPFilter::match (elements/ip/ipfilter.hh:393-481) per
//       packet, then CLASSIFY_EACH_PACKET. --l4 udp adds CheckUDPHeader
//       (elements/tcpudp/checkudpheader.cc: length and pseudo-header checksum
//       over the whole datagram) behind CheckIPHeader. --flow-capacity adds
//       FlowIPManagerHMP (elements/research/flowipmanagerhmp.cc:96-126:
//       IPFlow5ID find_create, IDs by an atomic fetch-and-add, each run of one
//       flow pushed downstream as its own PacketBatch) behind the checks.
//       --imix: C3's frames (64/570/1500 B on the wire, 7:4:1) with each packet
//       on a uniformly drawn flow of --flows; --trace N: trace packets (4096).
//   fc_cpu_baseline --verify                              -> exit 0 if the
//       pipeline matches fco_process_batch on a batch with injected errors
#include <atomic>
#include <chrono>
#include <thread>
#include <vector>
#include <string>
#include <string.h>
#include <stdio.h>
#include <stdlib.h>

#include "fc_oracle.h"
#include "../fastclick_amd/csrc/host/click_model.hh"
#include "../fastclick_amd/csrc/host/program_text.hh"

using namespace fcx;

namespace {

inline uint32_t le32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
inline uint16_t raw16(const uint8_t *p) { uint16_t v; memcpy(&v, p, 2); return v; }

struct Pipeline {
    // CheckIPHeader state
    std::atomic<uint64_t> count{0}, drops{0};
    std::atomic<uint64_t> reason_drops[6];
    uint64_t port_count[17] = {0};
    std::vector<uint32_t> *record_port = nullptr;   // verify mode: per-packet port
    std::vector<uint32_t> *record_hash = nullptr;
    int stages = 3;    // 0: Strip only (harness floor), 1: Strip+CheckIPHeader, 2: +AggregateHash, 3: +FlowSwitch classify
    bool program = false;   // stage 3 = IPClassifier program (fco_set_program) instead of FlowSwitch
    bool udp = false;       // CheckUDPHeader behind CheckIPHeader
    std::atomic<uint64_t> udp_count{0}, udp_drops{0};
    // FlowIPManagerHMP: open addressing over IPFlow5ID keys, IDs in order of
    // first appearance (the reference's HashTableMP find_create + _current)
    struct FlowKey { uint32_t s, d, ports, proto; };
    std::vector<FlowKey> fkeys;
    std::vector<uint32_t> fids;       // id + 1, 0 = empty
    uint32_t fmask = 0;
    std::atomic<uint32_t> fcurrent{0};
    uint32_t fcap = 0;
    void flow_init(uint32_t cap) {
        fcap = cap;
        uint32_t sz = 1;
        while (sz < 2 * cap) sz <<= 1;
        fkeys.assign(sz, FlowKey{0, 0, 0, 0});
        fids.assign(sz, 0);
        fmask = sz - 1;
    }
    Pipeline() { for (auto &r : reason_drops) r = 0; }

    // Strip::simple_action_batch (elements/standard/strip.cc:38-50)
    void strip(PacketBatch *b) {
        for (Packet *p = b->first(); p; p = p->next()) p->pull(14);
    }

    // CheckIPHeader::valid (elements/ip/checkipheader.cc:163-226), CHECKSUM true
    int valid(Packet *p) {
        unsigned plen = p->length();
        if ((int)plen < 20) return 0;
        const uint8_t *ip = p->data();
        if ((ip[0] >> 4) != 4) return 1;
        unsigned hlen = (unsigned)(ip[0] & 15) << 2;
        if (hlen < 20) return 2;
        unsigned len = ((unsigned)ip[2] << 8) | ip[3];
        if (len > plen || len < hlen) return 3;
        if (fco_in_cksum(ip, (int)hlen) != 0) return 4;
        p->set_network_header(0, (int)hlen);
        if (plen > len) p->take(plen - len);
        p->set_anno_u32(DST_IP_ANNO_OFFSET, le32(ip + 16));
        count++;
        return 6;
    }

    // EXECUTE_FOR_EACH_PACKET_DROPPABLE (include/click/packetbatch.hh:111-142)
    PacketBatch *check(PacketBatch *b) {
        Packet *last = nullptr, *p = b->first();
        PacketBatch *head = b;
        unsigned cnt = b->count();
        while (p) {
            Packet *nx = p->next();
            int r = valid(p);
            if (r != 6) {
                drops++;
                reason_drops[r]++;
                if (record_port) (*record_port)[p->id] = 16;
                p->kill();
                if (last) last->set_next(nx);
                else head = nx ? PacketBatch::start_head(nx) : nullptr;
                cnt--;
            } else {
                last = p;
            }
            p = nx;
        }
        if (head) {
            head->set_count(cnt);
            head->set_tail(last);
            last->set_next(nullptr);
        }
        return head;
    }

    // CheckUDPHeader::simple_action (elements/tcpudp/checkudpheader.cc), CHECKSUM true,
    // in EXECUTE_FOR_EACH_PACKET_DROPPABLE
    PacketBatch *check_udp(PacketBatch *b) {
        Packet *last = nullptr, *p = b->first();
        PacketBatch *head = b;
        unsigned cnt = b->count();
        while (p) {
            Packet *nx = p->next();
            const uint8_t *ip = p->network_header();
            const uint8_t *uh = p->transport_header();
            bool ok = ip[9] == 17;
            if (ok) {
                const unsigned hl = (unsigned)(ip[0] & 15) << 2;
                const unsigned len = ((unsigned)uh[4] << 8) | uh[5];
                ok = len >= 8 && p->length() >= len + hl + (unsigned)(ip - p->data());
                if (ok && raw16(uh + 6) != 0)
                    ok = fco_in_cksum_pseudohdr(fco_in_cksum(uh, (int)len), ip, (int)len) == 0;
            }
            if (!ok) {
                udp_drops++;
                if (record_port) (*record_port)[p->id] = 16;
                p->kill();
                if (last) last->set_next(nx);
                else head = nx ? PacketBatch::start_head(nx) : nullptr;
                cnt--;
            } else {
                udp_count++;
                last = p;
            }
            p = nx;
        }
        if (head) {
            head->set_count(cnt);
            head->set_tail(last);
            last->set_next(nullptr);
        }
        return head;
    }

    // FlowIPManagerHMP::push_batch / process: the flow ID of each packet
    // (IPFlow5ID(p), a new one at first sight), consecutive packets of one
    // flow gathered by a BatchBuilder and pushed on as one batch.
    void flow_stage(PacketBatch *b) {
        Packet *p = b->first();
        Packet *rhead = nullptr, *rtail = nullptr;
        unsigned rcnt = 0;
        uint32_t rid = 0xffffffffu;
        auto finish = [&]() {
            if (!rhead) return;
            rtail->set_next(nullptr);
            downstream(PacketBatch::make_from_list(rhead, rtail, rcnt));
            rhead = rtail = nullptr;
            rcnt = 0;
        };
        while (p) {
            Packet *nx = p->next();
            const uint8_t *nh = p->network_header(), *th = p->transport_header();
            FlowKey k{le32(nh + 12), le32(nh + 16), le32(th), nh[9]};
            uint32_t h = fco_ipflowid_hash(k.s, (uint16_t)k.ports, k.d, (uint16_t)(k.ports >> 16)) ^ k.proto;
            uint32_t i = (h * 0x9E3779B1u) & fmask, id = 0xffffffffu;
            while (true) {
                if (!fids[i]) {
                    if (fcurrent.load(std::memory_order_relaxed) < fcap) {
                        id = fcurrent.fetch_add(1);
                        fkeys[i] = k;
                        fids[i] = id + 1;
                    }
                    break;
                }
                const FlowKey &q = fkeys[i];
                if (q.s == k.s && q.d == k.d && q.ports == k.ports && q.proto == k.proto) {
                    id = fids[i] - 1;
                    break;
                }
                i = (i + 1) & fmask;
            }
            if (id == 0xffffffffu) {      // table full: the new flow is dropped
                p->kill();
                p = nx;
                continue;
            }
            p->set_anno_u32(28, id);
            if (id != rid) {
                finish();
                rid = id;
                rhead = p;
            } else {
                rtail->set_next(p);
            }
            rtail = p;
            rcnt++;
            p = nx;
        }
        finish();
    }

    void downstream(PacketBatch *b) {
        if (stages >= 2) aggregate(b);
        if (stages >= 3) classify(b);
        else b->kill();
    }

    // AggregateHash::simple_action (elements/analysis/aggregatehash.cc:49-55)
    void aggregate(PacketBatch *b) {
        for (Packet *p = b->first(); p; p = p->next()) {
            const uint8_t *nh = p->network_header(), *th = p->transport_header();
            uint32_t h = 0;
            if (((((unsigned)nh[6] << 8) | nh[7]) & 0x1fff) == 0)
                h = fco_ipflowid_hash(le32(nh + 12), raw16(th), le32(nh + 16), raw16(th + 2));
            p->set_anno_u32(AGGREGATE_ANNO_OFFSET, h);
        }
    }

    // FlowSwitch LB_MODE hash_agg port + CLASSIFY_EACH_PACKET into 17 lists
    void classify(PacketBatch *b) {
        PacketBatch *out[17] = {nullptr};
        Packet *p = b->first();
        while (p) {
            Packet *nx = p->next();
            int o;
            if (program) {
                // IPClassifier: offsets relative to the network/transport headers
                fcgpu_anno a;
                memset(&a, 0, sizeof a);
                a.nh = 14;
                a.th = (uint8_t)(14 + (p->transport_header() - p->network_header()));
                a.length = (uint16_t)(p->length() + 14);
                uint32_t out = fco_run_program(p->data() - 14, &a);
                o = out < 16 ? (int)out : 16;
            } else {
                o = fco_lb_hash_port(p->anno_u32(AGGREGATE_ANNO_OFFSET), 16);
            }
            if (record_port) {
                (*record_port)[p->id] = (uint32_t)o;
                (*record_hash)[p->id] = p->anno_u32(AGGREGATE_ANNO_OFFSET);
            }
            if (!out[o]) {
                out[o] = PacketBatch::start_head(p);
                out[o]->set_count(1);
                out[o]->set_tail(p);
            } else {
                out[o]->append_packet(p);
            }
            p = nx;
        }
        for (int i = 0; i < 17; ++i)
            if (out[i]) {
                out[i]->tail()->set_next(nullptr);
                port_count[i] += out[i]->count();
                out[i]->kill();          // Discard::push_batch -> fast_kill
            }
    }

    void push_batch(PacketBatch *b) {
        strip(b);
        if (stages == 0) { b->kill(); return; }
        b = check(b);
        if (!b) return;
        if (udp && !(b = check_udp(b))) return;
        if (fcap) flow_stage(b);
        else downstream(b);
    }
};

// preloaded trace -> BURST-packet batches from a packet pool (ReplayUnqueue)
struct Replay {
    const uint8_t *arena;
    const uint32_t *desc;
    uint32_t n, pos = 0;
    PacketPool pool;
    Replay(const uint8_t *a, const uint32_t *d, uint32_t n_, uint32_t maxlen)
        : arena(a), desc(d), n(n_), pool(4096, 128 + maxlen + 64, 128) {}
    PacketBatch *next(uint32_t burst) {
        Packet *head = nullptr, *prev = nullptr;
        uint32_t m = 0;
        for (; m < burst; ++m) {
            uint32_t i = pos;
            pos = pos + 1 == n ? 0 : pos + 1;
            Packet *p = pool.make(arena + desc[2 * i], desc[2 * i + 1]);
            if (!p) break;
            p->id = i;
            if (prev) prev->set_next(p);
            else head = p;
            prev = p;
        }
        return m ? PacketBatch::make_from_list(head, prev, m) : nullptr;
    }
};

// C2-shaped trace: 60-B UDP/IPv4 frames, `flows` distinct 5-tuples (1 = C2;
// packet i on flow i % flows); imix: C3's 60/566/1496-B frames (64/570/1500 B
// on the wire, 7:4:1), each packet on a uniformly drawn flow. UDP checksums
// are valid (CheckUDPHeader verifies them).
void make_trace(uint32_t n, uint32_t flows, std::vector<uint8_t> &arena, std::vector<uint32_t> &desc,
                bool imix = false) {
    static const uint32_t kLen[3] = {60, 566, 1496};
    uint64_t r = 0x2545F4914F6CDD1Dull;
    auto rnd = [&r]() { r ^= r << 13; r ^= r >> 7; r ^= r << 17; return r; };
    std::vector<uint32_t> len(n, 60);
    if (imix)
        for (uint32_t i = 0; i < n; ++i) {
            const uint32_t w = (uint32_t)(rnd() % 12);
            len[i] = kLen[w < 7 ? 0 : w < 11 ? 1 : 2];
        }
    size_t total = 256;
    for (uint32_t i = 0; i < n; ++i) total += (len[i] + 63) & ~63u;
    arena.assign(total, 0);
    desc.resize(2 * n);
    uint64_t x = 0x9E3779B97F4A7C15ull;
    size_t off = 0;
    for (uint32_t i = 0; i < n; ++i) {
        uint8_t *f = arena.data() + off;
        uint32_t flow = flows > 1 ? (imix ? (uint32_t)(rnd() % flows) : (uint32_t)(i % flows)) : 0;
        uint64_t h = (flow + 1) * x;
        uint8_t eth[14] = {2, 0, 0, 0, 0, 2, 2, 0, 0, 0, 0, 1, 8, 0};
        memcpy(f, eth, 14);
        uint8_t *ip = f + 14;
        const uint32_t iplen = len[i] - 14, ulen = iplen - 20;
        ip[0] = 0x45; ip[2] = (uint8_t)(iplen >> 8); ip[3] = (uint8_t)iplen; ip[8] = 64; ip[9] = 17;
        uint8_t src[4] = {10, 0, 0, 1}, dst[4] = {10, 0, 0, 2};
        if (flows > 1) { memcpy(src, &h, 4); memcpy(dst, (uint8_t *)&h + 4, 4); }
        memcpy(ip + 12, src, 4);
        memcpy(ip + 16, dst, 4);
        uint16_t c = fco_in_cksum(ip, 20);
        memcpy(ip + 10, &c, 2);
        uint16_t sp = flows > 1 ? (uint16_t)(h >> 13) : 1234, dp = flows > 1 ? (uint16_t)(h >> 29) : 5678;
        ip[20] = sp >> 8; ip[21] = sp & 0xff; ip[22] = dp >> 8; ip[23] = dp & 0xff;
        ip[24] = (uint8_t)(ulen >> 8); ip[25] = (uint8_t)ulen;
        uint16_t uc = fco_in_cksum_pseudohdr(fco_in_cksum(ip + 20, (int)ulen), ip, (int)ulen);
        if (uc == 0) uc = 0xffff;
        memcpy(ip + 26, &uc, 2);
        desc[2 * i] = (uint32_t)off;
        desc[2 * i + 1] = len[i];
        off += (len[i] + 63) & ~63u;
    }
}

int verify() {
    // a trace with every error kind and IP options, checked against the oracle
    const uint32_t n = 20000;
    std::vector<uint8_t> arena;
    std::vector<uint32_t> desc;
    make_trace(n, 4096, arena, desc);
    uint64_t s = 12345;
    auto rnd = [&]() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; };
    for (uint32_t i = 0; i < n; ++i) {
        uint8_t *ip = arena.data() + desc[2 * i] + 14;
        switch (rnd() % 40) {
        case 0: desc[2 * i + 1] = 14 + rnd() % 20; break;
        case 1: ip[0] = 0x55; break;
        case 2: ip[0] = 0x43; break;
        case 3: ip[3] = 200; break;
        case 4: ip[10] ^= 1; break;
        case 5: ip[6] = 0x01; break;   // non-first fragment (hash 0 by definition)
        default: break;
        }
    }
    fcgpu_cfg cfg;
    memset(&cfg, 0, sizeof cfg);
    cfg.size = sizeof cfg;
    cfg.check_mode = FCGPU_CHECK_IP4;
    cfg.offset = 14;
    cfg.checksum = 1;
    cfg.hash_mode = FCGPU_HASH_FLOWID;
    cfg.classify = FCGPU_CLS_LB_HASH;
    cfg.nports = 16;
    std::vector<uint16_t> verdict(n);
    std::vector<uint32_t> hash(n);
    fco_process_batch(&cfg, arena.data(), desc.data(), n, verdict.data(), hash.data(), nullptr, nullptr,
                      nullptr, nullptr);
    Pipeline pl;
    std::vector<uint32_t> port(n, 999), h(n, 0);
    pl.record_port = &port;
    pl.record_hash = &h;
    Replay src(arena.data(), desc.data(), n, 64);
    for (uint32_t done = 0; done < n;) {
        uint32_t m = n - done < 32 ? n - done : 32;
        PacketBatch *b = src.next(m);
        pl.push_batch(b);
        done += m;
    }
    uint32_t bad = 0;
    for (uint32_t i = 0; i < n; ++i) {
        uint32_t ep = verdict[i] >> 8;
        if (port[i] != ep || ((verdict[i] & 0xff) == FCGPU_R_OK && h[i] != hash[i])) bad++;
    }
    // + CheckUDPHeader, on the same trace with some UDP errors
    for (uint32_t i = 0; i < n; i += 97) {
        uint8_t *ip = arena.data() + desc[2 * i] + 14;
        if ((i / 97) % 3 == 0) ip[27] ^= 1;                 // UDP checksum
        else if ((i / 97) % 3 == 1) ip[25] = 200;           // UDP length past the packet
        else ip[28] ^= 0x55;                                // payload byte
    }
    cfg.l4_mode = FCGPU_L4_UDP;
    cfg.l4_checksum = 1;
    fco_process_batch(&cfg, arena.data(), desc.data(), n, verdict.data(), hash.data(), nullptr, nullptr,
                      nullptr, nullptr);
    Pipeline pu;
    pu.udp = true;
    std::vector<uint32_t> port2(n, 999), h2(n, 0);
    pu.record_port = &port2;
    pu.record_hash = &h2;
    Replay src2(arena.data(), desc.data(), n, 64);
    for (uint32_t done = 0; done < n;) {
        uint32_t m = n - done < 32 ? n - done : 32;
        pu.push_batch(src2.next(m));
        done += m;
    }
    uint32_t l4drops = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t r = verdict[i] & 0xff, ep = verdict[i] >> 8;
        l4drops += r >= FCGPU_R_L4_PROTO && r <= FCGPU_R_L4_CKSUM;
        if (port2[i] != ep) bad++;
    }
    if (l4drops < 100) bad++;
    printf("{\"verify\": %s, \"mismatches\": %u, \"valid\": %llu}\n", bad ? "false" : "true", bad,
           (unsigned long long)pl.count.load());
    return bad ? 1 : 0;
}

}  // namespace

int main(int argc, char **argv) {
    double seconds = 10;
    int threads = 1;
    uint32_t flows = 1;
    int stages = 3;
    std::string progfile;
    bool udp = false, imix = false;
    uint32_t flow_cap = 0, trace_n = 4096;
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        if (a == "--verify") return verify();
        if (a == "--seconds" && i + 1 < argc) seconds = atof(argv[++i]);
        else if (a == "--threads" && i + 1 < argc) threads = atoi(argv[++i]);
        else if (a == "--flows" && i + 1 < argc) flows = (uint32_t)atoi(argv[++i]);
        else if (a == "--stages" && i + 1 < argc) stages = atoi(argv[++i]);
        else if (a == "--program" && i + 1 < argc) progfile = argv[++i];
        else if (a == "--l4" && i + 1 < argc) udp = std::string(argv[++i]) == "udp";
        else if (a == "--flow-capacity" && i + 1 < argc) flow_cap = (uint32_t)atoi(argv[++i]);
        else if (a == "--imix") imix = true;
        else if (a == "--trace" && i + 1 < argc) trace_n = (uint32_t)atoi(argv[++i]);
    }
    if (!progfile.empty()) {
        FILE *f = fopen(progfile.c_str(), "rb");
        if (!f) { fprintf(stderr, "cannot open %s\n", progfile.c_str()); return 2; }
        std::string text;
        char buf[4096];
        size_t k;
        while ((k = fread(buf, 1, sizeof buf, f)) > 0) text.append(buf, k);
        fclose(f);
        ParsedProgram pr;
        std::string e = parse_program(text, pr);
        if (!e.empty()) { fprintf(stderr, "program: %s\n", e.c_str()); return 2; }
        fco_set_program(FCGPU_PROG_IPFILTER, pr.steps.data(), (uint32_t)pr.steps.size(), pr.output_everything);
    }
    const uint32_t n = trace_n;
    std::vector<uint8_t> arena;
    std::vector<uint32_t> desc;
    make_trace(n, flows, arena, desc, imix);

    auto run = [&](int nth, double secs) {
        std::vector<std::thread> th;
        std::vector<uint64_t> pk(nth, 0);
        std::atomic<bool> stop{false};
        for (int t = 0; t < nth; ++t)
            th.emplace_back([&, t]() {
                Pipeline pl;
                pl.stages = stages;
                pl.program = !progfile.empty();
                pl.udp = udp;
                if (flow_cap) pl.flow_init(flow_cap);
                Replay src(arena.data(), desc.data(), n, imix ? 1536 : 64);
                uint64_t c = 0;
                while (!stop.load(std::memory_order_relaxed)) {
                    for (int k = 0; k < 64; ++k) {
                        PacketBatch *b = src.next(32);
                        pl.push_batch(b);
                        c += 32;
                    }
                }
                if (stages > 0 && pl.count.load() + pl.drops.load() != c) fprintf(stderr, "count mismatch\n");
                if (udp && pl.udp_count.load() + pl.udp_drops.load() != pl.count.load())
                    fprintf(stderr, "udp count mismatch\n");
                pk[t] = c;
            });
        auto t0 = std::chrono::steady_clock::now();
        std::this_thread::sleep_for(std::chrono::duration<double>(secs));
        stop = true;
        for (auto &x : th) x.join();
        double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        uint64_t tot = 0;
        for (auto v : pk) tot += v;
        return tot / dt / 1e6;
    };
    double one = run(1, seconds / 2);
    double all = threads > 1 ? run(threads, seconds / 2) : one;
    std::string chain = "Strip(14)";
    if (stages >= 1) chain += " -> CheckIPHeader(CHECKSUM true)";
    if (udp) chain += " -> CheckUDPHeader";
    if (flow_cap) chain += " -> FlowIPManagerHMP(CAPACITY " + std::to_string(flow_cap) + ")";
    if (stages >= 2) chain += " -> AggregateHash";
    if (stages >= 3) chain += progfile.empty() ? " -> FlowSwitch hash x16" : " -> IPClassifier program x16";
    chain += " -> Discard";
    printf("{\"mpps\": %.3f, \"mpps_1core\": %.3f, \"threads\": %d, \"stages\": %d, \"sample\": \"%s\"}\n", all,
           one, threads, stages,
           (std::string(imix ? "IMIX 64/570/1500-B (7:4:1)" : "60-B") + " UDP/IPv4 trace (" + std::to_string(n) +
            " pkts, " + std::to_string(flows) +
            " flow(s)) replayed in 32-packet linked-list batches: " + chain + "; " +
            std::to_string(seconds / 2) + " s at 1 thread + " + std::to_string(seconds / 2) + " s at " +
            std::to_string(threads) + " threads")
               .c_str());
    return 0;
}
