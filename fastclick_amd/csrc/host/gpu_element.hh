// gpu_element.hh -- GPUIPCheckClassify: the drop-in BatchElement.
//
// Replaces the CPU chain
//     [Strip(14) | StripEtherVLANHeader] -> CheckIPHeader / CheckIP6Header
//         -> AggregateHash -> FlowSwitch(LB_MODE hash) | HashSwitch   (=> N outputs)
// with one element whose push_batch gathers the batch, runs it through the
// MI355X kernels (C ABI, include/fastclick_gpu.h) and pushes one PacketBatch per
// output, packets in input order within each output (CLASSIFY_EACH_PACKET,
// include/click/packetbatch.hh:259-307). Invalid packets leave on output N
// when it exists, else are killed (CheckIPHeader::drop, checkipheader.cc:143-161).
//
// Keyword arguments mirror the replaced elements:
//   OFFSET, CHECKSUM (default FALSE: checkipheader.cc:110), BADSRC, GOODDST,
//   VERBOSE, DETAILS                         -- CheckIPHeader
//   NATIVE_VLAN (default 0)                  -- StripEtherVLANHeader
//   VLAN_ETHERTYPE (default 0x8100)          -- VLANDecap(ETHERTYPE) + Strip(14) (MODE AUTO)
//   MODE MARK6                               -- MarkIP6Header(OFFSET)
//   BADADDRS, PROCESS_EH                     -- CheckIP6Header (IPv6, MODE AUTO)
//   N / LB_MODE hash|hash_agg|hash_ip        -- FlowSwitch / LoadBalancer
//   HASHSWITCH "OFFSET LENGTH"               -- HashSwitch
//   PROGRAM "<program text>", PROGRAM_KIND IPFILTER|CLASSIFIER
//                                            -- IPFilter / IPClassifier / Classifier:
//     the compiled program as the reference's `program` handler prints it
//     (lines separated by newlines or '|', program_text.hh); N is the
//     classifier's output count. Packets no rule matches are killed, as
//     CLASSIFY_EACH_PACKET kills a packet whose port is out of range.
//   L4 UDP|TCP, L4_CHECKSUM (default true)   -- CheckUDPHeader / CheckTCPHeader
//     behind the IPv4 check (MODE CHECK or MARK); their drops join output N
//   COLOR (PAINT annotation on every packet)  -- IPInputCombo (with OFFSET 14,
//     CHECKSUM true, STRIP true and no invalid output: ipinputcombo.cc:65-141)
//   FLOW_CAPACITY n, FLOWID_ANNO o (default 28)
//                                            -- FlowIPManagerHMP (CAPACITY) behind the
//     checks: each checked IPv4 packet gets its flow's ID (IPFlow5ID, IDs in
//     order of first appearance, elements/research/flowipmanagerhmp.cc:96-126)
//     in the 4-byte annotation at FLOWID_ANNO; a new flow beyond the capacity
//     is killed (as the IMP managers do when their flow stack is empty). Output
//     batches are the classifier's, not split at flow changes.
//   DEC_TTL, TTL_MULTICAST (default true), SET_CHECKSUM
//                                            -- DecIPTTL / SetIPChecksum after the
//     classifier (IPv4): TTL-expired packets (DecIPTTL output 1) join output N,
//     headers SetIPChecksum rejects are killed; the rewritten ttl/checksum
//     bytes are written back into each packet.
//   MODE CHECK|MARK|AUTO, HASH NONE|FLOWID|FLOW5ID, STRIP, BATCH, DEVICE,
//   PARTITION TILE (default: each 256-packet tile classified as one batch, one
//   fused launch) | GLOBAL (the whole staged batch as one, three launches)
// Handlers: count, drops, drop_details (DETAILS true), port_counts,
// flow_count, flow_drops.
//
// Packets are parked until BATCH packets are staged (MinBatch pattern,
// elements/standard/minbatch.cc:57-76) or flush() is called. GPU/runtime
// errors are reported, never papered over: the staged packets are killed and
// the error is returned through the `error` handler.
#pragma once
#include <vector>
#include <string>
#include <sstream>
#include <inttypes.h>
#include <arpa/inet.h>
#include <string.h>

#include "click_model.hh"
#include "program_text.hh"
#include "../../../include/fastclick_gpu.h"

namespace fcx {

class GPUIPCheckClassify : public Element {
  public:
    GPUIPCheckClassify() { fcgpu_default_cfg(&_cfg); }
    ~GPUIPCheckClassify() override { if (_ctx) fcgpu_close(_ctx); }

    const char *class_name() const override { return "GPUIPCheckClassify"; }

    int configure(const std::vector<std::string> &conf, std::string &errh) override {
        fcgpu_default_cfg(&_cfg);
        _cfg.checksum = 0;
        bool strip_set = false;
        for (const auto &raw : conf) {
            ConfArg a = parse_arg(raw);
            const std::string &k = a.key, &v = a.value;
            long n;
            bool b;
            if (k == "OFFSET") {
                if (!parse_int(v, n) || n < 0 || n > 255) return err(errh, "OFFSET expects an integer in [0,255]");
                _cfg.offset = (int32_t)n;
            } else if (k == "CHECKSUM") {
                if (!parse_bool(v, b)) return err(errh, "CHECKSUM expects true/false");
                _cfg.checksum = b;
            } else if (k == "VERBOSE") {
                if (!parse_bool(v, _verbose)) return err(errh, "VERBOSE expects true/false");
            } else if (k == "DETAILS") {
                if (!parse_bool(v, _details)) return err(errh, "DETAILS expects true/false");
            } else if (k == "BADSRC" || k == "GOODDST") {
                std::istringstream ss(v);
                std::string w;
                uint32_t *dst = k == "BADSRC" ? _cfg.badsrc : _cfg.gooddst;
                uint32_t &cnt = k == "BADSRC" ? _cfg.nbadsrc : _cfg.ngooddst;
                cnt = 0;
                while (ss >> w) {
                    uint32_t ip;
                    if (!parse_ip4(w, ip)) return err(errh, k + " expects IP addresses");
                    if (cnt >= FCGPU_MAX_ADDRS) return err(errh, k + ": too many addresses");
                    dst[cnt++] = ip;
                }
            } else if (k == "VLAN_ETHERTYPE") {
                // VLANDecap ETHERTYPE (vlandecap.cc:35-45): the tag protocol removed
                if (!parse_int(v, n) || n < 0 || n > 0xFFFF) return err(errh, "bad VLAN_ETHERTYPE");
                _cfg.vlan_ethertype = (uint32_t)n;
            } else if (k == "NATIVE_VLAN") {
                if (!parse_int(v, n) || n > 0xFFF) return err(errh, "bad NATIVE_VLAN");
                _cfg.native_vlan = n >= 0 ? (int32_t)n : -1;
            } else if (k == "N" || k == "NPORTS") {
                if (!parse_int(v, n) || n < 1 || n > FCGPU_MAX_PORTS) return err(errh, "N out of range");
                _cfg.nports = (uint32_t)n;
                if (_cfg.classify == FCGPU_CLS_NONE) _cfg.classify = FCGPU_CLS_LB_HASH;
            } else if (k == "LB_MODE") {
                if (v == "hash" || v == "hash_agg") _cfg.classify = FCGPU_CLS_LB_HASH;
                else if (v == "hash_ip") _cfg.classify = FCGPU_CLS_HASH_IP;
                else return err(errh, "unsupported LB_MODE " + v);
            } else if (k == "HASHSWITCH") {
                long o, l;
                std::istringstream ss(v);
                std::string a1, a2;
                ss >> a1 >> a2;
                if (!parse_int(a1, o) || !parse_int(a2, l) || l <= 0 || o < 0)
                    return err(errh, "HASHSWITCH expects OFFSET LENGTH (length must be > 0)");
                _cfg.classify = FCGPU_CLS_HASHSWITCH;
                _cfg.hs_offset = (int32_t)o;
                _cfg.hs_length = (int32_t)l;
            } else if (k == "L4") {
                if (v == "UDP") _cfg.l4_mode = FCGPU_L4_UDP;
                else if (v == "TCP") _cfg.l4_mode = FCGPU_L4_TCP;
                else if (v == "NONE") _cfg.l4_mode = FCGPU_L4_NONE;
                else return err(errh, "L4 expects UDP, TCP or NONE");
            } else if (k == "L4_CHECKSUM") {
                if (!parse_bool(v, b)) return err(errh, "L4_CHECKSUM expects true/false");
                _cfg.l4_checksum = b;
            } else if (k == "COLOR") {
                if (!parse_int(v, n) || n < 0 || n > 255) return err(errh, "COLOR expects an integer in [0,255]");
                _color = (int)n;
            } else if (k == "PROGRAM") {
                std::string text = v;
                if (text.size() >= 2 && text.front() == '"' && text.back() == '"') text = text.substr(1, text.size() - 2);
                std::string e = parse_program(text, _prog);
                if (!e.empty()) return err(errh, "PROGRAM: " + e);
                _cfg.classify = FCGPU_CLS_PROGRAM;
            } else if (k == "PROGRAM_KIND") {
                if (v == "IPFILTER") _prog_kind = FCGPU_PROG_IPFILTER;
                else if (v == "CLASSIFIER") _prog_kind = FCGPU_PROG_CLASSIFIER;
                else return err(errh, "PROGRAM_KIND expects IPFILTER or CLASSIFIER");
            } else if (k == "MODE") {
                if (v == "CHECK") _cfg.check_mode = FCGPU_CHECK_IP4;
                else if (v == "MARK") _cfg.check_mode = FCGPU_MARK_IP4;
                else if (v == "AUTO") _cfg.check_mode = FCGPU_CHECK_AUTO;
                else if (v == "MARK6") _cfg.check_mode = FCGPU_MARK_IP6;
                else return err(errh, "MODE expects CHECK, MARK, AUTO or MARK6");
            } else if (k == "HASH") {
                if (v == "NONE") _cfg.hash_mode = FCGPU_HASH_NONE;
                else if (v == "FLOWID") _cfg.hash_mode = FCGPU_HASH_FLOWID;
                else if (v == "FLOW5ID") _cfg.hash_mode = FCGPU_HASH_FLOW5ID;
                else return err(errh, "HASH expects NONE, FLOWID or FLOW5ID");
            } else if (k == "STRIP") {
                if (!parse_bool(v, _strip)) return err(errh, "STRIP expects true/false");
                strip_set = true;
            } else if (k == "BATCH") {
                if (!parse_int(v, n) || n < 0 || n > (1L << 26)) return err(errh, "bad BATCH");
                _batch = (uint32_t)n;
            } else if (k == "DEVICE") {
                if (!parse_int(v, n) || n < 0) return err(errh, "bad DEVICE");
                _device = (int)n;
            } else if (k == "PARTITION") {
                if (v == "TILE") _partition = FCGPU_PART_TILE;
                else if (v == "GLOBAL") _partition = FCGPU_PART_GLOBAL;
                else return err(errh, "PARTITION expects TILE or GLOBAL");
            } else if (k == "BADADDRS") {
                // CheckIP6Header::configure (checkip6header.cc:47-87): the list
                // adds to the default ff..ff, duplicates dropped
                std::istringstream ss(v);
                std::string w;
                while (ss >> w) {
                    uint8_t a[16];
                    if (inet_pton(AF_INET6, w.c_str(), a) != 1) return err(errh, "BADADDRS expects IPv6 addresses");
                    bool dup = false;
                    for (uint32_t j = 0; j < _cfg.nbad6; ++j) dup |= memcmp(_cfg.bad6[j], a, 16) == 0;
                    if (dup) continue;
                    if (_cfg.nbad6 >= FCGPU_MAX_ADDRS) return err(errh, "BADADDRS: too many addresses");
                    memcpy(_cfg.bad6[_cfg.nbad6++], a, 16);
                }
            } else if (k == "DEC_TTL" || k == "SET_CHECKSUM" || k == "TTL_MULTICAST") {
                if (!parse_bool(v, b)) return err(errh, k + " expects true/false");
                if (k == "TTL_MULTICAST") _cfg.ttl_multicast = b;
                else {
                    const uint32_t f = k == "DEC_TTL" ? FCGPU_RW_DECTTL : FCGPU_RW_SETCKSUM;
                    _cfg.rewrite = b ? (_cfg.rewrite | f) : (_cfg.rewrite & ~f);
                }
            } else if (k == "FLOW_CAPACITY") {
                if (!parse_int(v, n) || n < 0 || n > (long)FCGPU_MAX_FLOWS) return err(errh, "bad FLOW_CAPACITY");
                _flow_cap = (uint32_t)n;
            } else if (k == "FLOWID_ANNO") {
                if (!parse_int(v, n) || n < 0 || n > ANNO_SIZE - 4) return err(errh, "bad FLOWID_ANNO");
                _flow_anno = (int)n;
            } else if (k == "PROCESS_EH") {
                if (!parse_bool(v, b)) return err(errh, "PROCESS_EH expects true/false");
                _cfg.process_eh = b;
            } else if (k.empty()) {
                return err(errh, "too many arguments");        // Args::complete(): OFFSET is keyword-only
            } else {
                return err(errh, "unknown keyword " + k);
            }
        }
        if (!strip_set) _strip = (_cfg.check_mode == FCGPU_CHECK_AUTO);
        const bool ip4 = _cfg.check_mode == FCGPU_CHECK_IP4 || _cfg.check_mode == FCGPU_MARK_IP4;
        if (_cfg.l4_mode != FCGPU_L4_NONE && !ip4)
            return err(errh, "L4 needs MODE CHECK or MARK");
        if (_flow_cap && !ip4)
            return err(errh, "FLOW_CAPACITY needs MODE CHECK or MARK");
        if (_cfg.rewrite && !ip4)
            return err(errh, "DEC_TTL / SET_CHECKSUM need MODE CHECK or MARK");
        if (_cfg.classify == FCGPU_CLS_PROGRAM) {
            if (_prog.output_everything >= (int32_t)_cfg.nports && _prog.output_everything != 0x7fff)
                return err(errh, "PROGRAM sends everything to a missing output");
            for (const auto &st : _prog.steps)
                if ((st.yes <= 0 && -st.yes >= (int32_t)_cfg.nports && st.yes != -2147483647) ||
                    (st.no <= 0 && -st.no >= (int32_t)_cfg.nports && st.no != -2147483647))
                    return err(errh, "PROGRAM jumps to an output >= N");
        }
        return 0;
    }

    int initialize(std::string &errh) override {
        uint32_t cap = _batch ? _batch : 65536;
        _cap = cap + 8192;   // a burst may overshoot BATCH
        int rc = fcgpu_open(_device, _cap, &_ctx);
        if (rc != FCGPU_OK) return err(errh, std::string("fcgpu_open: ") + fcgpu_last_error(nullptr));
        rc = fcgpu_configure(_ctx, &_cfg);
        if (rc != FCGPU_OK) return err(errh, std::string("fcgpu_configure: ") + fcgpu_last_error(_ctx));
        if (_cfg.classify == FCGPU_CLS_PROGRAM) {
            rc = fcgpu_set_program(_ctx, _prog_kind, _prog.steps.data(), (uint32_t)_prog.steps.size(),
                                   _prog.output_everything);
            if (rc != FCGPU_OK) return err(errh, std::string("fcgpu_set_program: ") + fcgpu_last_error(_ctx));
        }
        if (_flow_cap) {
            rc = fcgpu_flow_enable(_ctx, _flow_cap);
            if (rc != FCGPU_OK) return err(errh, std::string("fcgpu_flow_enable: ") + fcgpu_last_error(_ctx));
            _flowid.resize(_cap);
        }
        if (_cfg.rewrite) _iprw.resize(_cap);
        _pkts.reserve(_cap);
        _frames.reserve(_cap);
        _lens.reserve(_cap);
        _verdict.resize(_cap);
        _hash.resize(_cap);
        _anno.resize(_cap);
        _perm.resize(_cap);
        _keep.resize(_cap);
        _tperm.resize(_cap + FCGPU_TILE);
        _start.resize(FCGPU_MAX_PORTS + 2);
        _tile_count.resize((size_t)(FCGPU_MAX_PORTS + 1) * ((_cap + FCGPU_TILE - 1) / FCGPU_TILE));
        return 0;
    }

    void push_batch(int, PacketBatch *batch) override {
        for (Packet *p = batch->first(); p; p = p->next()) {
            if (_pkts.size() == _cap) process_staged();
            _pkts.push_back(p);
        }
        if (_pkts.size() >= (_batch ? _batch : 1)) process_staged();
    }

    // A non-batch upstream: the packet is parked in the same staging ring, so a
    // stream of single pushes still reaches the device BATCH packets at a time
    // (without BATCH every push is its own one-packet launch).
    void push(int, Packet *p) override {
        if (_pkts.size() == _cap) process_staged();
        _pkts.push_back(p);
        if (_pkts.size() >= (_batch ? _batch : 1)) process_staged();
    }

    void flush() override {
        if (!_pkts.empty()) process_staged();
    }

    std::string read_handler(const std::string &h) override {
        uint64_t c[FCGPU_NCOUNTERS] = {0};
        if (_ctx) fcgpu_read_counters(_ctx, c, FCGPU_NCOUNTERS);
        std::ostringstream s;
        if (h == "count") s << c[FCGPU_CTR_COUNT];
        else if (h == "drops") s << c[FCGPU_CTR_DROPS];
        else if (h == "drop_details" && _details) {
            // checkipheader.cc:247-256 format
            static const char *texts[6] = {"tiny packet", "bad IPv4 version", "bad IPv4 header length",
                                           "bad IPv4 length", "bad IPv4 checksum", "bad source address"};
            char line[96];
            for (int i = 0; i < 6; ++i) {
                snprintf(line, sizeof line, "%15" PRIu64 " packets due to: %24s\n", c[FCGPU_CTR_REASON + i], texts[i]);
                s << line;
            }
        } else if (h == "port_counts") {
            for (uint32_t p = 0; p <= _cfg.nports; ++p) s << (p ? " " : "") << c[FCGPU_CTR_PORT + p];
        } else if (h == "flow_count") {
            uint32_t f = 0;
            if (_ctx) fcgpu_flow_count(_ctx, &f);
            s << f;
        } else if (h == "flow_drops") s << _flow_drops;
        else if (h == "error") s << _error;
        return s.str();
    }

  private:
    int err(std::string &errh, const std::string &m) {
        errh = std::string(class_name()) + ": " + m;
        return -1;
    }

    void process_staged() {
        const uint32_t n = (uint32_t)_pkts.size();
        _frames.resize(n);
        _lens.resize(n);
        for (uint32_t i = 0; i < n; ++i) {
            _frames[i] = _pkts[i]->data();
            _lens[i] = _pkts[i]->length();
        }
        fcgpu_out o{};
        o.flowid = _flow_cap ? _flowid.data() : nullptr;
        o.ip_rw = _cfg.rewrite ? _iprw.data() : nullptr;
        o.verdict = _verdict.data();
        o.hash = _hash.data();
        o.anno = _anno.data();
        o.perm = _partition == FCGPU_PART_GLOBAL ? _perm.data() : nullptr;
        o.tile_perm = _partition == FCGPU_PART_TILE ? _tperm.data() : nullptr;
        o.partition = _partition;
        o.port_start = _partition == FCGPU_PART_GLOBAL ? _start.data() : nullptr;
        o.tile_count = _partition == FCGPU_PART_TILE ? _tile_count.data() : nullptr;
        o.reserved = 0;
        int rc = fcgpu_process_host(_ctx, _frames.data(), _lens.data(), n, &o);
        if (rc != FCGPU_OK) {
            // no CPU fallback: report, drop the staged packets, keep running
            _error = fcgpu_last_error(_ctx);
            fprintf(stderr, "%s: GPU processing failed: %s\n", class_name(), _error.c_str());
            for (Packet *p : _pkts) p->kill();
            _pkts.clear();
            return;
        }
        const bool hashing = _cfg.hash_mode != FCGPU_HASH_NONE;
        const bool autom = _cfg.check_mode == FCGPU_CHECK_AUTO;
        for (uint32_t i = 0; i < n; ++i) {
            Packet *p = _pkts[i];
            const fcgpu_anno &a = _anno[i];
            const uint32_t reason = _verdict[i] & 0xff;
            if (_color >= 0) p->set_anno_u8(PAINT_ANNO_OFFSET, (uint8_t)_color);   // SET_PAINT_ANNO
            if (autom && reason != FCGPU_R_VLAN_REJECT)
                p->set_anno_u16(VLAN_TCI_ANNO_OFFSET, a.vlan_tci);    // StripEtherVLANHeader
            if (reason == FCGPU_R_OK || reason >= FCGPU_R_NO_MATCH) {
                if (_cfg.rewrite && _iprw[i])                          // DecIPTTL / SetIPChecksum
                    memcpy(p->data() + a.nh + 8, &_iprw[i], 4);
                p->set_network_header(a.nh, a.th);                     // set_ip_header / set_ip6_header
                if (a.length < p->length()) p->take(p->length() - a.length);
                if (a.ipver == 6) p->set_anno_u8(IP6_NXT_ANNO_OFFSET, a.ip6_nxt);
                else p->set_anno_u32(DST_IP_ANNO_OFFSET, a.dst_ip);
                if (hashing && reason <= FCGPU_R_NO_MATCH)   // AggregateHash (not after an L4 drop)
                    p->set_anno_u32(AGGREGATE_ANNO_OFFSET, _hash[i]);
                if (_flow_cap && _flowid[i] != FCGPU_FLOW_NONE && _flowid[i] != FCGPU_FLOW_FULL)
                    p->set_anno_u32(_flow_anno, _flowid[i]);
                if (_strip) p->pull(a.nh);
            } else {
                if (!_warned || _verbose) {
                    fprintf(stderr, "%s: IP header check failed: reason %u\n", class_name(), reason);
                    _warned = true;
                }
                // the replaced Strip / StripEtherVLANHeader ran before the checker
                if (_strip && reason != FCGPU_R_VLAN_REJECT) p->pull(autom ? a.nh : (uint32_t)_cfg.offset);
            }
        }
        const uint32_t nb = _cfg.nports + 1;
        if (_partition == FCGPU_PART_GLOBAL) {
            // one batch per output in port order, input order within a port
            // (chunked to MAX_BATCH_SIZE, include/click/packetbatch.hh:416)
            for (uint32_t port = 0; port < nb; ++port)
                emit_run(port, _start[port], _start[port + 1], [this](uint32_t j) { return _perm[j]; });
        } else {
            // every FCGPU_TILE-packet tile is one classified PacketBatch: its
            // runs leave in port order, tiles in input order
            const uint32_t ntiles = (n + FCGPU_TILE - 1) / FCGPU_TILE;
            for (uint32_t t = 0; t < ntiles; ++t) {
                const uint32_t base = t * FCGPU_TILE;
                uint32_t s = base;
                auto idx = [this, base](uint32_t j) { return base + _tperm[j]; };
                for (uint32_t port = 0; port < nb; ++port) {
                    const uint32_t c = _tile_count[(size_t)t * nb + port];
                    emit_run(port, s, s + c, idx);
                    s += c;
                }
            }
        }
        _pkts.clear();
    }

    // link packets idx(s) .. idx(e-1) into PacketBatches of <= MAX_BATCH_SIZE
    template <class Idx>
    void emit_run(uint32_t port, uint32_t s, uint32_t e, Idx idx) {
        const bool nomatch = port == _cfg.nports && _cfg.classify == FCGPU_CLS_PROGRAM;
        const bool setck = port == _cfg.nports && (_cfg.rewrite & FCGPU_RW_SETCKSUM);
        if (nomatch || setck || _flow_cap) {
            // the last slot mixes invalid packets (output N) and packets no
            // rule matched (killed); a full flow table kills new flows. Keep
            // input order for the rest.
            uint32_t w = s;
            for (uint32_t j = s; j < e; ++j) {
                const uint32_t i = idx(j);
                if ((nomatch && (_verdict[i] & 0xff) == FCGPU_R_NO_MATCH) ||
                    (setck && (_verdict[i] & 0xff) == FCGPU_R_SETCKSUM_BAD)) {
                    _pkts[i]->kill();
                } else if (_flow_cap && _flowid[i] == FCGPU_FLOW_FULL) {
                    ++_flow_drops;
                    _pkts[i]->kill();
                } else {
                    _keep[w++ - s] = i;
                }
            }
            emit_list(port, w - s);
            return;
        }
        while (s < e) {
            uint32_t m = e - s < kMaxBatch ? e - s : kMaxBatch;
            Packet *head = _pkts[idx(s)], *prev = head;
            for (uint32_t j = 1; j < m; ++j) {
                Packet *q = _pkts[idx(s + j)];
                prev->set_next(q);
                prev = q;
            }
            checked_output_push_batch((int)port, PacketBatch::make_from_list(head, prev, m));
            s += m;
        }
    }

    void emit_list(uint32_t port, uint32_t m) {
        for (uint32_t s = 0; s < m;) {
            uint32_t k = m - s < kMaxBatch ? m - s : kMaxBatch;
            Packet *head = _pkts[_keep[s]], *prev = head;
            for (uint32_t j = 1; j < k; ++j) {
                Packet *q = _pkts[_keep[s + j]];
                prev->set_next(q);
                prev = q;
            }
            checked_output_push_batch((int)port, PacketBatch::make_from_list(head, prev, k));
            s += k;
        }
    }

    static constexpr uint32_t kMaxBatch = 8192;
    ParsedProgram _prog;
    uint32_t _prog_kind = FCGPU_PROG_IPFILTER;
    int _color = -1;
    uint32_t _flow_cap = 0;
    int _flow_anno = 28;
    uint64_t _flow_drops = 0;
    std::vector<uint32_t> _flowid;
    std::vector<uint32_t> _iprw;
    std::vector<uint32_t> _keep;
    fcgpu_cfg _cfg;
    fcgpu_ctx *_ctx = nullptr;
    int _device = 0;
    uint32_t _batch = 0;      // 0: process every incoming batch immediately
    uint32_t _cap = 0;
    bool _verbose = false, _details = false, _strip = false, _warned = false;
    std::string _error;
    std::vector<Packet *> _pkts;
    std::vector<const uint8_t *> _frames;
    std::vector<uint32_t> _lens;
    std::vector<uint16_t> _verdict;
    std::vector<uint32_t> _hash;
    std::vector<fcgpu_anno> _anno;
    std::vector<uint32_t> _perm;
    std::vector<uint8_t> _tperm;
    std::vector<uint32_t> _start;
    std::vector<uint16_t> _tile_count;
    uint32_t _partition = FCGPU_PART_TILE;
};

}  // namespace fcx
