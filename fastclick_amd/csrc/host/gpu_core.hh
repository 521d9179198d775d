// gpu_core.hh -- the logic of the GPUIPCheckClassify element, written once for
// two packet models:
//   - FastClick's (fastclick_pkg/gpuipcheckclassify.{hh,cc}: Packet /
//     PacketBatch of include/click/packet.hh and packetbatch.hh), and
//   - the test harness's (click_model.hh, driven by tests through libfcclick).
// A policy class P maps the few Packet/PacketBatch operations the element
// needs onto each model (see ModelPolicy in gpu_element.hh and ClickPolicy in
// fastclick_pkg/gpuipcheckclassify.hh), so the code the tests exercise is the
// code the FastClick element runs.
//
// Replaces the CPU chain
//     [Strip(14) | StripEtherVLANHeader] -> CheckIPHeader / CheckIP6Header
//         -> AggregateHash -> FlowSwitch(LB_MODE hash) | HashSwitch | IPClassifier
// with one element: push_batch stages every packet's leading bytes (the reach
// of the configured chain, capture.hh) into pinned memory while the packet is
// still in the CPU cache, BATCH packets form one device batch that goes to
// the GPU asynchronously (fcgpu_span_submit: H2D copy, kernels, D2H of the
// results), and while it is there the next batch is staged in the other slot
// (double buffering). A slot's results are applied when the slot is needed
// again, on flush(), or when the TIMER fires: annotations are written into
// the packets and one PacketBatch per output run leaves in input order
// (CLASSIFY_EACH_PACKET, include/click/packetbatch.hh:259-307). Invalid
// packets leave on output N when it exists, else are killed
// (CheckIPHeader::drop, elements/ip/checkipheader.cc:143-161).
//
// Accumulation follows MinBatch (elements/standard/minbatch.cc:57-76): a
// batch leaves when BATCH packets are staged or TIMER microseconds after its
// first packet, whichever comes first (TIMER -1: only on BATCH or flush()).
// Every packet the element receives leaves exactly once: pushed on one
// output, or killed. A batch the GPU fails (a submission or its completion
// returns an error, SURVEY 8(b) "Errors") is re-submitted once through copies
// (FCGPU_SUBMIT_COPY: no zero-copy, no shared queue); if that fails too its
// packets leave unprocessed on ERROR_OUTPUT, or are killed (the default), and
// are counted (gpu_errors, drop_details) -- never dropped silently. There is
// no CPU fallback.
//
// Keyword arguments mirror the replaced elements:
//   OFFSET, CHECKSUM (default FALSE: checkipheader.cc:110), BADSRC, GOODDST,
//   INTERFACES, VERBOSE, DETAILS             -- CheckIPHeader
//   NATIVE_VLAN (default 0)                  -- StripEtherVLANHeader
//   VLAN_ETHERTYPE (default 0x8100)          -- VLANDecap(ETHERTYPE) + Strip(14) (MODE AUTO)
//   MODE MARK6                               -- MarkIP6Header(OFFSET)
//   BADADDRS, PROCESS_EH                     -- CheckIP6Header (IPv6, MODE AUTO)
//   N / LB_MODE hash|hash_agg|hash_ip|hash_crc|chash|cst_hash_agg, CST_BUCKETS
//                                            -- FlowSwitch / LoadBalancer (the hash
//     modes: decided per packet, as the reference's per-flow decision caches it)
//   HASHSWITCH "OFFSET LENGTH"               -- HashSwitch (hash_ip, chash and
//     HASHSWITCH count their bytes from the frame start, or with STRIP from the
//     stripped data, as behind Strip(OFFSET); MODE AUTO needs STRIP false for them)
//   PROGRAM "<program text>", PROGRAM_KIND IPFILTER|CLASSIFIER, PROGRAM_JIT (default
//     true: the program compiled to code at initialize, fcgpu_program_jit)
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
//     is killed (as the IMP managers do when their flow stack is empty).
//   FLOW_RUNS (default true): each output's packets leave in runs of one
//     flow, a PacketBatch per run, as the flow managers' BatchBuilder pushes
//     them (flowipmanagerhmp.cc:101-117); false: one batch per output run.
//   FLOW_MANAGER HMP|IMP, FLOW_TIMEOUT s, FLOW_RECYCLE_INTERVAL s (default 1)
//                                            -- IMP: FlowIPManager_CuckooPP /
//     FlowIPManagerIMP (CAPACITY, TIMEOUT, RECYCLE_INTERVAL): IDs from a free-ID
//     stack, flows idle for TIMEOUT s expire (include/click/flow/
//     virtualflowmanager.hh); the maintainer runs every RECYCLE_INTERVAL from
//     the first batch on the element's clock: each submission first runs the
//     runs that are due, and so does the element's Timer, which fires for
//     them with no traffic as the reference's maintain_timer does.
//   DEC_TTL, TTL_MULTICAST (default true), SET_CHECKSUM
//                                            -- DecIPTTL / SetIPChecksum after the
//     classifier (IPv4): TTL-expired packets (DecIPTTL output 1) join output N,
//     headers SetIPChecksum rejects are killed; the rewritten ttl/checksum
//     bytes are written back into each packet.
//   MODE CHECK|MARK|AUTO, HASH NONE|FLOWID|FLOW5ID, STRIP, DEVICE,
//   BATCH (packets per device batch; 0: each incoming PacketBatch is one;
//   default auto: 16384 while the batches are copied, 4096 while they are
//   zero-copy -- many threads' batches then share the PCIe-read path, and
//   smaller ones keep each thread's round trip short: profiles/archive/r03_s24.txt
//   -- and 8192 zero-copy with COMPACT records, half the bytes per packet:
//   profiles/r04_crossover/el_sweep2_compact.log),
//   TIMER (us, default 100; -1 none),
//   SLOTS (default 2): device batches a thread stages or has in flight
//   (double or triple buffering),
//   ZEROCOPY true|false|auto (default auto): true -- the device reads each
//   slot's staged block and writes its results in pinned host memory, where
//   they lie (fcgpu_span_mode FCGPU_SPAN_ZEROCOPY), instead of one H2D and one
//   D2H copy per batch; auto -- zero-copy while >= 4 element threads share
//   the GPU (their copies would queue on one copy engine), else copies,
//   PARTITION TILE (default: each 256-packet tile classified as one batch,
//   one fused launch) | GLOBAL (the whole device batch as one, three launches)
//   COMPACT true|false (default true): for IPv4 chains that read only the
//     header, the ports and fixed byte ranges, each packet stages just those
//     bytes in a 16-B record (capture.hh stage_plan): 32 B for a 60-B UDP
//     frame instead of a 64-B slot -- the bytes a batch moves over PCIe
//   ERROR_OUTPUT p (default -1: kill)          -- where the packets of a batch the
//     GPU failed twice leave, unprocessed and in input order
// Handlers: count, drops, drop_details (DETAILS true), port_counts,
// flow_count, flow_count_fids (IMP: the free-ID stack's entries, the
// reference's count_fids), flow_drops, gpu_errors (packets of batches the GPU failed twice),
// gpu_retries (batches re-submitted through copies), error (the last failure
// that cost packets).
#pragma once
#include <inttypes.h>
#include <arpa/inet.h>
#include <stdio.h>
#include <string.h>
#include <atomic>
#include <mutex>
#include <sstream>
#include <string>
#include <vector>

#include "click_args.hh"
#include "program_text.hh"
#include "../capture.hh"
#include "../../../include/fastclick_gpu.h"

namespace fcx {

template <class P>
class RxCore {
  public:
    using Packet = typename P::Packet;
    using Batch = typename P::Batch;
    static constexpr uint32_t kMaxSlots = FCGPU_SPAN_SLOTS;   // batches staged / in flight: SLOTS (2..3)
    static constexpr uint32_t kMaxBatch = 8192;    // MAX_BATCH_SIZE (packetbatch.hh:416)

    RxCore() { fcgpu_default_cfg(&_cfg); }
    ~RxCore() { release(); }
    RxCore(const RxCore &) = delete;
    RxCore &operator=(const RxCore &) = delete;

    std::string name = "GPUIPCheckClassify";       // for chatter: the element's name

    // ---- configuration (keyword arguments, "KEY value" strings) ------------
    int configure(const std::vector<std::string> &conf, std::string &errh) {
        fcgpu_default_cfg(&_cfg);
        _cfg.checksum = 0;
        bool strip_set = false;
        bool have_if = false, badsrc_set = false, gooddst_set = false;
        std::vector<uint32_t> if_bad, if_good;   // INTERFACES (raw network-order words)
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
            } else if (k == "INTERFACES") {
                // CheckIPHeader::InterfacesArg (checkipheader.cc:56-80): per
                // prefix, its broadcast address is a bad source and the address
                // a good destination; then 0.0.0.0 and 255.255.255.255
                std::istringstream ss(v);
                std::string w;
                if_bad.clear();
                if_good.clear();
                while (ss >> w) {
                    uint32_t ip, mask;
                    if (!parse_ip4_prefix(w, ip, mask)) return err(errh, "INTERFACES expects IP prefixes");
                    if_bad.push_back((ip & mask) | ~mask);
                    if_good.push_back(ip);
                }
                if_bad.push_back(0u);
                if_bad.push_back(0xFFFFFFFFu);
                if (if_bad.size() > FCGPU_MAX_ADDRS) return err(errh, "INTERFACES: too many addresses");
                have_if = true;
            } else if (k == "BADSRC" || k == "GOODDST") {
                std::istringstream ss(v);
                std::string w;
                uint32_t *dst = k == "BADSRC" ? _cfg.badsrc : _cfg.gooddst;
                uint32_t &cnt = k == "BADSRC" ? _cfg.nbadsrc : _cfg.ngooddst;
                (k == "BADSRC" ? badsrc_set : gooddst_set) = true;
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
                // LoadBalancer modetrans (include/click/loadbalancer.hh:23-58)
                _lb_direct = v == "hash";
                if (v == "hash" || v == "hash_agg") _cfg.classify = FCGPU_CLS_LB_HASH;
                else if (v == "hash_ip") _cfg.classify = FCGPU_CLS_HASH_IP;
                else if (v == "hash_crc") _cfg.classify = FCGPU_CLS_LB_CRC;
                else if (v == "cst_hash_agg") _cfg.classify = FCGPU_CLS_LB_TABLE;
                else if (v == "chash") {
                    // direct_chash = hash_4tuple (:138-152, :666-668): HashSwitch's
                    // byte sum over frame bytes [26, 38)
                    _cfg.classify = FCGPU_CLS_HASHSWITCH;
                    _cfg.hs_offset = 26;
                    _cfg.hs_length = 12;
                } else return err(errh, "unsupported LB_MODE " + v);
            } else if (k == "CST_BUCKETS") {
                // the constant_hash_agg ring's size (:264, :273-275)
                if (!parse_int(v, n) || n < 1 || n > (long)FCGPU_LB_TABLE_MAX) return err(errh, "bad CST_BUCKETS");
                _cst_buckets = (uint32_t)n;
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
            } else if (k == "PROGRAM_JIT") {
                if (!parse_bool(v, _prog_jit)) return err(errh, "PROGRAM_JIT expects true/false");
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
                if (v == "auto" || v == "AUTO") {
                    _batch = kBatchCopy;
                    _batch_auto = true;
                } else {
                    if (!parse_int(v, n) || n < 0 || n > (1L << 24)) return err(errh, "bad BATCH");
                    _batch = (uint32_t)n;              // 0: every incoming PacketBatch is one device batch
                    _batch_auto = false;
                }
            } else if (k == "TIMER") {
                if (!parse_int(v, n) || n < -1 || n > 10000000) return err(errh, "TIMER expects microseconds (-1: none)");
                _timer_us = n;
            } else if (k == "DEVICE") {
                if (!parse_int(v, n) || n < 0) return err(errh, "bad DEVICE");
                _device = (int)n;
            } else if (k == "SLOTS") {
                if (!parse_int(v, n) || n < 2 || n > (long)kMaxSlots) return err(errh, "SLOTS expects 2 or 3");
                _nslots = (uint32_t)n;
            } else if (k == "ZEROCOPY") {
                if (v == "auto" || v == "AUTO") _span_mode = FCGPU_SPAN_AUTO;
                else if (parse_bool(v, b)) _span_mode = b ? FCGPU_SPAN_ZEROCOPY : FCGPU_SPAN_COPY;
                else return err(errh, "ZEROCOPY expects true, false or auto");
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
            } else if (k == "FLOW_MANAGER") {
                if (v == "HMP") _flow_mgr = FCGPU_FLOW_MGR_HMP;
                else if (v == "IMP") _flow_mgr = FCGPU_FLOW_MGR_IMP;
                else return err(errh, "FLOW_MANAGER expects HMP or IMP");
            } else if (k == "FLOW_TIMEOUT") {
                if (!parse_int(v, n) || n < 0 || n > 86400) return err(errh, "bad FLOW_TIMEOUT");
                _flow_timeout = (uint32_t)n;
            } else if (k == "FLOW_RECYCLE_INTERVAL") {
                // seconds, as RECYCLE_INTERVAL (virtualflowmanager.hh:68-71)
                char *end = nullptr;
                const double d = strtod(v.c_str(), &end);
                if (v.empty() || *end || !(d >= 0.001 && d <= 65.535)) return err(errh, "bad FLOW_RECYCLE_INTERVAL");
                _flow_recycle_ms = (uint32_t)(d * 1000);
            } else if (k == "FLOW_RUNS") {
                if (!parse_bool(v, b)) return err(errh, "FLOW_RUNS expects true/false");
                _flow_runs = b;
            } else if (k == "FLOWID_ANNO") {
                if (!parse_int(v, n) || n < 0 || n > P::kAnnoSize - 4) return err(errh, "bad FLOWID_ANNO");
                _flow_anno = (int)n;
            } else if (k == "COMPACT") {
                if (!parse_bool(v, _compact)) return err(errh, "COMPACT expects true/false");
            } else if (k == "ERROR_OUTPUT") {
                if (!parse_int(v, n) || n < -1 || n > FCGPU_MAX_PORTS + 1) return err(errh, "bad ERROR_OUTPUT");
                _error_output = (int)n;
            } else if (k == "PROCESS_EH") {
                if (!parse_bool(v, b)) return err(errh, "PROCESS_EH expects true/false");
                _cfg.process_eh = b;
            } else if (k.empty()) {
                return err(errh, "too many arguments");        // Args::complete(): OFFSET is keyword-only
            } else {
                return err(errh, "unknown keyword " + k);
            }
        }
        // Args reads INTERFACES before BADSRC and GOODDST, which replace its
        // lists (IPAddressArg's Vector parse swaps, lib/ipaddress.cc:174-193)
        if (have_if && !badsrc_set) {
            _cfg.nbadsrc = (uint32_t)if_bad.size();
            for (size_t j = 0; j < if_bad.size(); ++j) _cfg.badsrc[j] = if_bad[j];
        }
        if (have_if && !gooddst_set) {
            _cfg.ngooddst = (uint32_t)if_good.size();
            for (size_t j = 0; j < if_good.size(); ++j) _cfg.gooddst[j] = if_good[j];
        }
        if (!strip_set) _strip = (_cfg.check_mode == FCGPU_CHECK_AUTO);
        // The byte-sum classifiers read from p->data() (hashswitch.cc:52-59,
        // loadbalancer.hh:138-152,227-243): with STRIP the chain is
        // Strip(OFFSET) -> CheckIPHeader -> ..., so their bytes count from the
        // IP header, OFFSET bytes into the frame the device indexes
        if ((_cfg.classify == FCGPU_CLS_HASH_IP || _cfg.classify == FCGPU_CLS_HASHSWITCH) && _strip) {
            if (_cfg.check_mode == FCGPU_CHECK_AUTO)
                return err(errh, "LB_MODE hash_ip / chash / HASHSWITCH behind StripEtherVLANHeader read bytes at a "
                                 "per-packet offset: use STRIP false (offsets from the frame start)");
            if (_cfg.classify == FCGPU_CLS_HASH_IP) {   // hash_ip = HashSwitch(26, 8)'s sum
                _cfg.classify = FCGPU_CLS_HASHSWITCH;
                _cfg.hs_offset = 26;
                _cfg.hs_length = 8;
            }
            _cfg.hs_offset += _cfg.offset;
        }
        _eff_batch = _batch;
        const bool ip4 = _cfg.check_mode == FCGPU_CHECK_IP4 || _cfg.check_mode == FCGPU_MARK_IP4;
        if (_cfg.l4_mode != FCGPU_L4_NONE && !ip4) return err(errh, "L4 needs MODE CHECK or MARK");
        if (_flow_cap && !ip4) return err(errh, "FLOW_CAPACITY needs MODE CHECK or MARK");
        if (_flow_timeout && _flow_mgr != FCGPU_FLOW_MGR_IMP) return err(errh, "FLOW_TIMEOUT needs FLOW_MANAGER IMP");
        if (_cfg.rewrite && !ip4) return err(errh, "DEC_TTL / SET_CHECKSUM need MODE CHECK or MARK");
        if (_cfg.classify == FCGPU_CLS_LB_CRC && !ip4) return err(errh, "LB_MODE hash_crc needs MODE CHECK or MARK");
        // direct_hash hashes IPFlowID (loadbalancer.hh:580-584), hash_agg the
        // AGGREGATE annotation HASH sets
        if (_lb_direct && _cfg.hash_mode == FCGPU_HASH_FLOW5ID)
            return err(errh, "LB_MODE hash hashes IPFlowID: with HASH FLOW5ID use LB_MODE hash_agg");
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

    int64_t timer_us() const { return _timer_us; }
    int error_output() const { return _error_output; }
    const fcgpu_cfg &device_cfg() const { return _cfg; }
    uint32_t nports() const { return _cfg.nports; }

    // ---- device context and staging slots ----------------------------------
    int initialize(std::string &errh) {
        // BATCH packets, or (BATCH 0) a whole incoming PacketBatch (16-bit count)
        _cap = _batch ? _batch : 65536;
        int rc = fcgpu_open(_device, _cap, &_ctx);
        if (rc != FCGPU_OK) return err(errh, std::string("fcgpu_open: ") + fcgpu_last_error(nullptr));
        rc = fcgpu_configure(_ctx, &_cfg);
        if (rc != FCGPU_OK) return err(errh, std::string("fcgpu_configure: ") + fcgpu_last_error(_ctx));
        rc = fcgpu_span_mode(_ctx, _span_mode);
        if (rc != FCGPU_OK) return err(errh, std::string("fcgpu_span_mode: ") + fcgpu_last_error(_ctx));
        uint32_t reach = 0;
        if (_cfg.classify == FCGPU_CLS_PROGRAM) {
            // the program as code (fcgpu_program_jit) unless PROGRAM_JIT false;
            // one with a cycle stays interpreted
            if (_prog_jit) fcgpu_program_jit(_ctx, 1);
            rc = fcgpu_set_program(_ctx, _prog_kind, _prog.steps.data(), (uint32_t)_prog.steps.size(),
                                   _prog.output_everything);
            if (rc != FCGPU_OK) return err(errh, std::string("fcgpu_set_program: ") + fcgpu_last_error(_ctx));
            const uint32_t l3 = (uint32_t)_cfg.offset + (_cfg.check_mode == FCGPU_CHECK_AUTO ? 18u : 0u);
            reach = fcgpu::program_reach(_prog_kind, _prog.steps.data(), (uint32_t)_prog.steps.size(), l3, l3 + 60);
        }
        if (_cfg.classify == FCGPU_CLS_LB_TABLE) {
            // the ring of LoadBalancer::set_mode (loadbalancer.hh:526-530):
            // CST_BUCKETS, or 100 per output
            std::vector<uint8_t> ring(_cst_buckets ? _cst_buckets : 100u * _cfg.nports);
            rc = fcgpu_lb_hash_ring(_cfg.nports, (uint32_t)ring.size(), ring.data());
            if (rc == FCGPU_OK) rc = fcgpu_set_lb_table(_ctx, ring.data(), (uint32_t)ring.size());
            if (rc != FCGPU_OK) return err(errh, std::string("fcgpu_set_lb_table: ") + fcgpu_last_error(_ctx));
        }
        if (_flow_cap) {
            fcgpu_flow_config fc{_flow_mgr, _flow_cap, _flow_timeout, _flow_recycle_ms};
            rc = fcgpu_flow_configure(_ctx, &fc);
            if (rc != FCGPU_OK) return err(errh, std::string("fcgpu_flow_configure: ") + fcgpu_last_error(_ctx));
        }
        _capture = fcgpu::capture_bytes(_cfg, reach);
        _plan = fcgpu::stage_plan(_cfg);
        _plan.compact = _plan.compact && _compact;
        // compact records go with 4-B descriptors (FCGPU_SUBMIT_DESC32): each
        // frame's start (record - start) falls on an 8-B boundary, and on a
        // 16-B one while the records so far add up to 16-B multiples (always,
        // for rest-of-frame records)
        _desc32 = _plan.compact;
        _lead = _plan.compact ? fcgpu::kStageLead + (_plan.start & 15u) : 0u;
        const size_t per = _capture == fcgpu::kCaptureWhole ? 1536 : _capture;
        // IPv4 chains: 8-B annotations (half the bytes written back per packet)
        const bool a8 = (_cfg.check_mode == FCGPU_CHECK_IP4 || _cfg.check_mode == FCGPU_MARK_IP4) &&
                        _cfg.offset >= 0 && _cfg.offset <= 255;
        _outputs = FCGPU_OUT_VERDICT | FCGPU_OUT_HASH | (a8 ? FCGPU_OUT_ANNO8 : FCGPU_OUT_ANNO) |
                   (_partition == FCGPU_PART_TILE ? FCGPU_OUT_TILE_PERM | FCGPU_OUT_TILE_COUNT
                                                  : FCGPU_OUT_PERM | FCGPU_OUT_PORT_START) |
                   (_flow_cap ? FCGPU_OUT_FLOWID : 0u) | (_cfg.rewrite ? FCGPU_OUT_IP_RW : 0u);
        fcgpu_block_layout L;
        if (fcgpu_block_layout_for(_ctx, _cap, _outputs, _partition, &L) != FCGPU_OK)
            return err(errh, "fcgpu_block_layout_for failed");
        for (uint32_t k = 0; k < _nslots; ++k)
            if (!_slot[k].alloc(_cap, (size_t)_cap * per + 65536 + _lead, L.bytes))
                return err(errh, "cannot allocate pinned staging (fcgpu_host_alloc)");
        // the device blocks of every slot now, at the staging blocks' size: a
        // submission through copies -- and a failed batch's re-submission
        // while other threads' batches run on the shared queue -- then never
        // allocates, frees or synchronises the device
        if (fcgpu_span_reserve(_ctx, _slot[0].in_cap, _outputs, _partition) != FCGPU_OK)
            return err(errh, std::string("fcgpu_span_reserve: ") + fcgpu_last_error(_ctx));
        return 0;
    }

    // Kill whatever is still staged or in flight (router cleanup).
    void release() {
        std::lock_guard<std::mutex> g(_mu);
        for (uint32_t k = 0; k < _nslots; ++k) {
            Slot &s = _slot[k];
            if (s.inflight && _ctx) fcgpu_span_wait(_ctx, k);
            s.inflight = false;
            for (uint32_t i = 0; i < s.n; ++i) P::kill(s.pkts[i]);
            s.n = 0;
            s.used = 0;
            s.free();
        }
        if (_ctx) fcgpu_close(_ctx);
        _ctx = nullptr;
    }

    // ---- data path -----------------------------------------------------------
    // A PacketBatch's packets, in order (the element owns them from here).
    template <class Emit>
    void push_list(Packet *p, Emit &&emit) {
        while (p) {
            if ((p = stage_run(p)) == nullptr) break;
            Packet *nx = P::next(p);
            stage(p, emit);
            p = nx;
        }
        if (!_batch && _slot[_cur].n) submit(emit);      // BATCH 0: one device batch per PacketBatch
    }
    template <class Emit>
    void push_one(Packet *p, Emit &&emit) {
        stage(p, emit);
        if (!_batch) submit(emit);
    }

    // Everything staged goes to the device and every batch in flight
    // completes, in order.
    template <class Emit>
    void flush(Emit &&emit) {
        if (_slot[_cur].n) submit(emit);
        for (uint32_t k = 0; k < _nslots; ++k) {
            const uint32_t j = (_cur + k) % _nslots;      // oldest first
            if (_slot[j].inflight) complete(j, emit);
        }
    }

    // The TIMER: batches in flight complete (they left before anything
    // staged), and a partial batch staged at least TIMER us ago goes to the
    // device and completes too. Returns true while packets remain staged:
    // the caller reschedules the timer for due_ns().
    // With IMP timeouts the Timer also runs the maintainer runs due by now,
    // with no packet needed -- the reference's maintain_timer fires every
    // RECYCLE_INTERVAL whether or not packets arrive
    // (virtualflowmanager.hh:118-124,134-144), so idle flows expire and the
    // handlers see it.
    template <class Emit>
    bool run_timer(uint64_t now_ns, Emit &&emit) {
        if (_flow_cap && _flow_timeout) {
            std::lock_guard<std::mutex> g(_mu);
            if (_ctx) flow_catch_up(now_ns / 1000000ull);
        }
        if (_timer_us < 0) return false;                  // TIMER -1: no timer
        Slot &s = _slot[_cur];
        if (s.n && now_ns >= due_ns()) {
            flush(emit);
            return false;
        }
        for (uint32_t k = 1; k < _nslots; ++k) {
            const uint32_t j = (_cur + k) % _nslots;      // oldest first
            if (_slot[j].inflight) complete(j, emit);
        }
        return s.n != 0;
    }
    // ns at which the staged partial batch is due (valid while staged() > 0)
    uint64_t due_ns() const { return _slot[_cur].t_first + (uint64_t)(_timer_us < 0 ? 0 : _timer_us) * 1000ull; }
    // IMP timeouts configured: the Timer also serves the maintainer
    bool flow_timeouts() const { return _flow_cap && _flow_timeout; }
    // The next maintainer run (IMP timeouts, once the first batch armed them):
    // true and its time in *ns, for the Timer that must also fire for it.
    bool maint_due_ns(uint64_t *ns) const {
        if (!(_flow_cap && _flow_timeout && _maint_armed)) return false;
        *ns = _next_maint_ms * 1000000ull;
        return true;
    }
    uint32_t staged() const { return _slot[_cur].n; }
    uint32_t held() const {
        uint32_t h = 0;
        for (const Slot &s : _slot) h += s.n;
        return h;
    }
    uint32_t max_held() const { return _nslots * (_cap ? _cap : (_batch ? _batch : 65536)); }
    bool idle() const {
        for (const Slot &s : _slot)
            if (s.n || s.inflight) return false;
        return true;
    }

    // ---- handlers ------------------------------------------------------------
    // What the host side counts besides the device counters (summed over
    // threads on read like them).
    struct HostStats {
        uint64_t flows = 0;        // flow IDs issued (flow table)
        uint64_t flow_fids = 0;    // IMP: entries on the free-ID stack, ID 0 included (count_fids)
        uint64_t flow_drops = 0;   // new flows killed, table full
        uint64_t gpu_errors = 0;   // packets of batches the GPU failed twice (killed or on ERROR_OUTPUT)
        uint64_t gpu_killed = 0;   // ... of which killed (no ERROR_OUTPUT)
        uint64_t gpu_retries = 0;  // batches re-submitted through copies after a failure
        HostStats &operator+=(const HostStats &o) {
            flows += o.flows;
            flow_fids += o.flow_fids;
            flow_drops += o.flow_drops;
            gpu_errors += o.gpu_errors;
            gpu_killed += o.gpu_killed;
            gpu_retries += o.gpu_retries;
            return *this;
        }
    };
    // This core's counters (fcgpu_read_counters), host-side counts and last
    // error. Safe from any thread (a handler reads every thread's core,
    // ELEMENT_MT_SAFE): the context and the error string are only touched
    // under _mu, which the owning data thread holds around its own context
    // calls (submit, completion wait, maintainer, failure).
    void counters(uint64_t (&c)[FCGPU_NCOUNTERS], HostStats &hs, std::string *error = nullptr) {
        memset(c, 0, sizeof c);
        uint32_t f = 0;
        fcgpu_flow_stat st{};
        {
            std::lock_guard<std::mutex> g(_mu);
            if (_ctx) fcgpu_read_counters(_ctx, c, FCGPU_NCOUNTERS);
            if (_ctx && _flow_cap) fcgpu_flow_count(_ctx, &f);
            if (_ctx && _flow_cap && _flow_mgr == FCGPU_FLOW_MGR_IMP) fcgpu_flow_stats(_ctx, &st);
            if (error) *error = _error;
        }
        hs.flows = f;
        // flows_stack_i (virtualflowmanager.hh:33,389-391): the stack holds
        // 0 .. cap-1 after initialization (:113-115), so it reads cap; ID 0 is
        // on it but never handed out
        hs.flow_fids = st.capacity ? (uint64_t)st.free_ids + 1 : 0;
        hs.flow_drops = _flow_drops.load(std::memory_order_relaxed);
        hs.gpu_errors = _gpu_errors.load(std::memory_order_relaxed);
        hs.gpu_killed = _gpu_killed.load(std::memory_order_relaxed);
        hs.gpu_retries = _gpu_retries.load(std::memory_order_relaxed);
    }
    bool details() const { return _details; }

    // Handler text from (summed) counters, in the replaced elements' formats.
    // Packets a GPU failure killed count as drops; drop_details gives them a
    // line of their own once there are any (the six CheckIPHeader lines
    // otherwise, exactly).
    static std::string format_handler(const std::string &h, const uint64_t (&c)[FCGPU_NCOUNTERS], uint32_t nports,
                                      bool details, const HostStats &hs, const std::string &error) {
        std::ostringstream s;
        if (h == "count") s << c[FCGPU_CTR_COUNT];
        else if (h == "drops") s << c[FCGPU_CTR_DROPS] + hs.gpu_killed;
        else if (h == "drop_details" && details) {
            char line[96];
            for (int i = 0; i < 6; ++i) {     // checkipheader.cc:247-256 format
                snprintf(line, sizeof line, "%15" PRIu64 " packets due to: %24s\n", c[FCGPU_CTR_REASON + i],
                         kReasonTexts[i]);
                s << line;
            }
            if (hs.gpu_errors) {
                snprintf(line, sizeof line, "%15" PRIu64 " packets due to: %24s\n", hs.gpu_errors, "GPU failure");
                s << line;
            }
        } else if (h == "port_counts") {
            for (uint32_t p = 0; p <= nports; ++p) s << (p ? " " : "") << c[FCGPU_CTR_PORT + p];
        } else if (h == "flow_count") s << hs.flows;
        else if (h == "flow_count_fids") s << hs.flow_fids;
        else if (h == "flow_drops") s << hs.flow_drops;
        else if (h == "gpu_errors") s << hs.gpu_errors;
        else if (h == "gpu_retries") s << hs.gpu_retries;
        else if (h == "error") s << error;
        return s.str();
    }
    std::string read_handler(const std::string &h) {
        uint64_t c[FCGPU_NCOUNTERS];
        HostStats hs;
        std::string error;
        counters(c, hs, &error);
        return format_handler(h, c, _cfg.nports, _details, hs, error);
    }
    std::string error() const {
        std::lock_guard<std::mutex> g(_mu);
        return _error;
    }

    // CheckIPHeader::reason_texts (elements/ip/checkipheader.cc:35-38)
    static constexpr const char *kReasonTexts[6] = {"tiny packet", "bad IPv4 version", "bad IPv4 header length",
                                                    "bad IPv4 length", "bad IPv4 checksum", "bad source address"};

  private:
    // One device batch: the staged bytes and descriptors (pinned, so the H2D
    // copy is DMA), the packets, and the pinned result arrays the D2H copies
    // land in.
    struct Slot {
        // pinned input block: [descriptors: cap x 8 B][frames]; pinned result
        // block laid out by fcgpu_block_layout_for -- one copy each way per batch
        uint8_t *in = nullptr, *res = nullptr;
        size_t in_cap = 0, frames_off = 0, used = 0;
        uint8_t *span = nullptr;          // in + frames_off
        uint32_t *desc = nullptr;         // in
        std::vector<Packet *> pkts;
        std::vector<uint32_t> keep;
        uint32_t n = 0;
        bool inflight = false;
        bool desc32 = false;       // descriptors as FCGPU_SUBMIT_DESC32 words (compact records)
        bool holes = false;        // a packet freed while its results were applied
        uint64_t t_first = 0;
        // the result arrays of the completed batch (inside res)
        uint16_t *verdict = nullptr, *tile_count = nullptr;
        uint32_t *hash = nullptr, *perm = nullptr, *start = nullptr, *flowid = nullptr, *iprw = nullptr;
        fcgpu_anno *anno = nullptr;
        const fcgpu_anno8 *anno8 = nullptr;    // FCGPU_OUT_ANNO8 (IPv4 chains) instead of anno
        uint8_t *tperm = nullptr;

        bool alloc(uint32_t cap, size_t frame_bytes, size_t res_bytes) {
            pkts.resize(cap);
            keep.resize(cap);
            frames_off = ((size_t)cap * 8 + 255) & ~(size_t)255;
            in_cap = frames_off + frame_bytes;
            in = static_cast<uint8_t *>(fcgpu_host_alloc(in_cap));
            res = static_cast<uint8_t *>(fcgpu_host_alloc(res_bytes ? res_bytes : 1));
            span = in ? in + frames_off : nullptr;
            desc = reinterpret_cast<uint32_t *>(in);
            return in && res;
        }
        void free() {
            fcgpu_host_free(in);
            fcgpu_host_free(res);
            in = res = span = nullptr;
            desc = nullptr;
        }
        // point the result arrays at their place in res for an n-packet batch
        void map(const fcgpu_block_layout &L, bool a8) {
            auto at = [this](size_t o) -> void * { return o == FCGPU_OUT_ABSENT ? nullptr : res + o; };
            verdict = (uint16_t *)at(L.verdict);
            hash = (uint32_t *)at(L.hash);
            anno = a8 ? nullptr : (fcgpu_anno *)at(L.anno);
            anno8 = a8 ? (const fcgpu_anno8 *)at(L.anno) : nullptr;
            perm = (uint32_t *)at(L.perm);
            start = (uint32_t *)at(L.port_start);
            tile_count = (uint16_t *)at(L.tile_count);
            tperm = (uint8_t *)at(L.tile_perm);
            flowid = (uint32_t *)at(L.flowid);
            iprw = (uint32_t *)at(L.ip_rw);
        }
    };

    int err(std::string &errh, const std::string &m) {
        errh = name + ": " + m;
        return -1;
    }

    // cp bytes, no byte read outside [src, src + cp): 16-B moves, the last
    // one overlapping its predecessor (a frame is 60 B in the headline case)
    static inline void copy_head(uint8_t *dst, const uint8_t *src, uint32_t cp) {
        if (cp >= 16) {
            uint32_t k = 0;
            for (; k + 16 <= cp; k += 16) memcpy(dst + k, src + k, 16);
            if (k < cp) memcpy(dst + cp - 16, src + cp - 16, 16);
        } else {
            memcpy(dst, src, cp);
        }
    }

    // The slot's DESC32 words so far back to (offset, length) pairs, in place
    // from the last (a frame longer than 65535 B, or records past 512 KiB).
    static void widen_desc(Slot &s) {
        for (uint32_t i = s.n; i-- > 0;) {
            const uint32_t w = s.desc[i];
            s.desc[2 * i + 1] = w >> 16;
            s.desc[2 * i] = (w & 0xffffu) << 3;
        }
        s.desc32 = false;
    }

    // Copy the packet's leading bytes into the current slot (64-B aligned
    // records), remember the packet; a full slot goes to the device.
    template <class Emit>
    inline void stage(Packet *p, Emit &emit) {
        Slot *s = &_slot[_cur];
        const uint32_t len = P::length(p);
        const uint8_t *src = P::data(p);
        uint32_t cp;
        size_t rec;
        if (_plan.compact) {
            // the frame bytes [start, end) the chain reads, in records packed kStageAlign (8) bytes apart
            uint32_t so;
            rec = fcgpu::stage_record_size(_plan, (uint32_t)_cfg.offset, src, len, so, cp);
            src += so;
        } else {
            cp = len < _capture ? len : _capture;
            rec = cp ? ((size_t)cp + 63) & ~(size_t)63 : 64;
        }
        if (s->n && s->frames_off + _lead + s->used + rec > s->in_cap) {   // whole frames overflowing the block
            submit(emit);
            s = &_slot[_cur];
        }
        if (s->n == 0) {
            if (!_ctx) {                                 // not initialized / released
                P::kill(p);
                return;
            }
            s->t_first = _timer_us >= 0 ? P::now_ns() : 0;
            s->desc32 = _desc32;
        }
        copy_head(s->span + _lead + s->used, src, cp);
        // compact: frame byte b of the packet is at record + b - start
        const uint32_t fo = (uint32_t)(_lead + s->used) - (_plan.compact ? _plan.start : 0u);
        // a length or an offset DESC32 cannot carry: (offset, length) pairs from here
        if (s->desc32 && (len > 0xffffu || _lead + s->used + rec > kDesc32Reach)) widen_desc(*s);
        if (s->desc32) {
            s->desc[s->n] = (fo >> 3) | (len << 16);
        } else {
            s->desc[2 * s->n] = fo;
            s->desc[2 * s->n + 1] = len;
        }
        s->pkts[s->n++] = p;
        s->used += rec;
        if (s->n == _cap || (_batch && s->n >= _eff_batch)) submit(emit);
    }

    // stage() over a run of a list, with the plan and the slot's state in
    // locals (stage() reloads them per packet: its descriptor stores may alias
    // them). Stages packets while the open slot takes them as they are --
    // room in the block, below the batch size, and with compact records
    // DESC32 words -- and returns the first packet it leaves to stage() (a
    // slot to open or submit, a descriptor DESC32 cannot carry), nullptr at
    // the list's end. Same records and descriptors as stage().
    Packet *stage_run(Packet *p) {
        if (!_plan.compact) return stage_capture_run(p);
        Slot &s = _slot[_cur];
        if (!s.n || !s.desc32) return p;
        const fcgpu::StagePlan plan = _plan;
        const uint32_t off = (uint32_t)_cfg.offset;
        const size_t lead = _lead, room = s.in_cap - s.frames_off - lead;
        // stage() submits once n reaches _cap, or _eff_batch under BATCH: the
        // packet that reaches it goes through stage()
        const uint32_t limit = _batch && _eff_batch < _cap ? _eff_batch : _cap;
        uint8_t *const span = s.span + lead;
        uint32_t *const desc = s.desc;
        Packet **const pkts = s.pkts.data();
        uint32_t n = s.n;
        size_t used = s.used;
        while (p && n + 1 < limit) {
            const uint32_t len = P::length(p);
            const uint8_t *src = P::data(p);
            uint32_t so, cp;
            const size_t rec = fcgpu::stage_record_size(plan, off, src, len, so, cp);
            if (used + rec > room || len > 0xffffu || lead + used + rec > kDesc32Reach) break;
            copy_head(span + used, src + so, cp);
            desc[n] = (uint32_t)((lead + used - plan.start) >> 3) | (len << 16);
            pkts[n++] = p;
            used += rec;
            p = P::next(p);
        }
        s.n = n;
        s.used = used;
        return p;
    }
    // The same for whole captures (the first min(len, capture) bytes of every
    // frame in 64-B aligned records, (offset, length) descriptors).
    Packet *stage_capture_run(Packet *p) {
        Slot &s = _slot[_cur];
        if (!s.n || s.desc32) return p;
        const uint32_t capture = _capture;
        const size_t lead = _lead, room = s.in_cap - s.frames_off - lead;
        const uint32_t limit = _batch && _eff_batch < _cap ? _eff_batch : _cap;
        uint8_t *const span = s.span + lead;
        uint32_t *const desc = s.desc;
        Packet **const pkts = s.pkts.data();
        uint32_t n = s.n;
        size_t used = s.used;
        while (p && n + 1 < limit) {
            const uint32_t len = P::length(p);
            const uint32_t cp = len < capture ? len : capture;
            const size_t rec = cp ? ((size_t)cp + 63) & ~(size_t)63 : 64;
            if (used + rec > room) break;
            copy_head(span + used, P::data(p), cp);
            desc[2 * n] = (uint32_t)(lead + used);
            desc[2 * n + 1] = len;
            pkts[n++] = p;
            used += rec;
            p = P::next(p);
        }
        s.n = n;
        s.used = used;
        return p;
    }

    // The current slot goes to the device (asynchronous); the next slot is
    // made free, completing the batch in it first if it is still in flight.
    template <class Emit>
    void submit(Emit &emit) {
        const uint32_t k = _cur;
        Slot &s = _slot[k];
        bool failed = false;
        {
            std::lock_guard<std::mutex> g(_mu);
            if (_flow_cap && _flow_timeout) flow_clock();
            int rc = fcgpu_span_submit_block(_ctx, k, s.in, s.frames_off + _lead + s.used, 0, s.frames_off, s.n, s.res,
                                             _outputs | (s.desc32 ? FCGPU_SUBMIT_DESC32 : 0u), _partition);
            // BATCH auto: the next batches' size for the path they now take
            _eff_batch = _batch_auto && fcgpu_span_zerocopy_active(_ctx)
                             ? (_plan.compact ? kBatchZeroCopyCompact : kBatchZeroCopy)
                             : _batch;
            if (rc != FCGPU_OK) rc = resubmit(k);
            if (rc == FCGPU_OK) s.inflight = true;
            else failed = true;
        }
        if (failed) fail_slot(s, emit);
        _cur = (_cur + 1) % _nslots;
        if (_slot[_cur].inflight) complete(_cur, emit);
    }

    // Slot k's batch failed (submission or completion): once more, through
    // copies (FCGPU_SUBMIT_COPY). The staged block is intact -- nothing the
    // failed attempt ran writes it. Called with _mu held; returns the
    // re-submission's code.
    int resubmit(uint32_t k) {
        Slot &s = _slot[k];
        _gpu_retries.fetch_add(1, std::memory_order_relaxed);
        P::chatter(name + ": GPU batch failed (" + std::string(fcgpu_last_error(_ctx)) + "), re-submitting it");
        _fail_msg = fcgpu_last_error(_ctx);
        return fcgpu_span_submit_block(_ctx, k, s.in, s.frames_off + _lead + s.used, 0, s.frames_off, s.n, s.res,
                                       _outputs | FCGPU_SUBMIT_COPY | (s.desc32 ? FCGPU_SUBMIT_DESC32 : 0u),
                                       _partition);
    }

    // IMP timeouts: the maintainer runs due by now (every RECYCLE_INTERVAL from
    // the first batch, virtualflowmanager.hh:118-124,134-144), then this
    // batch's time stamp (Timestamp::recent_steady() at push_batch, :227-230).
    // Queued on the context's stream ahead of the batch. Called with _mu held.
    void flow_clock() {
        const uint64_t now = P::now_ns() / 1000000ull;
        if (!_maint_armed) {
            _next_maint_ms = now + _flow_recycle_ms;
            _maint_armed = true;
        }
        flow_catch_up(now);
        fcgpu_flow_set_time(_ctx, (uint32_t)now);
    }
    // The maintainer runs due by now_ms (ms on the element's clock; the
    // device takes times mod 2^32). Called with _mu held.
    void flow_catch_up(uint64_t now_ms) {
        while (_maint_armed && now_ms >= _next_maint_ms) {
            if (fcgpu_flow_maintain(_ctx, (uint32_t)_next_maint_ms, nullptr) != FCGPU_OK)
                _error = fcgpu_last_error(_ctx);
            _next_maint_ms += _flow_recycle_ms;
        }
    }

    // The batch failed twice (no CPU fallback): its packets leave
    // unprocessed, in input order, on ERROR_OUTPUT, or are killed; either way
    // they are counted (gpu_errors; killed ones also in drops).
    template <class Emit>
    void fail_slot(Slot &s, Emit &emit) {
        const uint32_t n = s.n;
        std::string msg;
        {
            std::lock_guard<std::mutex> g(_mu);
            const char *m = _ctx ? fcgpu_last_error(_ctx) : nullptr;
            _error = m && *m ? m : (_fail_msg.empty() ? "GPU processing failed" : _fail_msg);
            msg = _error;
        }
        _gpu_errors.fetch_add(n, std::memory_order_relaxed);
        s.n = 0;
        s.used = 0;
        s.inflight = false;
        // an ERROR_OUTPUT the element does not have (the harness connects its
        // outputs after initialize) would kill them in checked_output_push_batch:
        // they are killed and counted here instead
        if (_error_output >= 0 && _error_output < emit.noutputs()) {
            P::chatter(name + ": GPU processing failed twice: " + msg + "; " + std::to_string(n) +
                       " packets to output " + std::to_string(_error_output));
            for (uint32_t a = 0; a < n;) {
                const uint32_t k = n - a < kMaxBatch ? n - a : kMaxBatch;
                Packet *head = s.pkts[a], *prev = head;
                for (uint32_t j = 1; j < k; ++j) {
                    P::set_next(prev, s.pkts[a + j]);
                    prev = s.pkts[a + j];
                }
                emit(_error_output, P::make_batch(head, prev, k));
                a += k;
            }
        } else {
            P::chatter(name + ": GPU processing failed twice: " + msg + "; " + std::to_string(n) + " packets killed");
            _gpu_killed.fetch_add(n, std::memory_order_relaxed);
            for (uint32_t i = 0; i < n; ++i) P::kill(s.pkts[i]);
        }
    }

    // The first drop's chatter, as the replaced checker prints it
    // (checkipheader.cc:146, checkip6header.cc:93, checkudpheader.cc:77,
    // checktcpheader.cc:78).
    void drop_chatter(uint32_t reason) {
        if (_warned && !_verbose) return;
        _warned = true;
        std::string m;
        if (reason < 6) m = name + ": IP header check failed: " + kReasonTexts[reason];
        else if (reason == FCGPU_R_BAD_IP6) m = "IP6 header check failed";
        else if (reason >= FCGPU_R_L4_PROTO && reason <= FCGPU_R_L4_CKSUM) {
            static const char *const udp[3] = {"not UDP", "bad packet length", "bad UDP checksum"};
            static const char *const tcp[3] = {"not TCP", "bad packet length", "bad TCP checksum"};
            const uint32_t r = reason - FCGPU_R_L4_PROTO;
            m = _cfg.l4_mode == FCGPU_L4_UDP ? std::string("UDP header check failed: ") + udp[r]
                                             : name + ": TCP header check failed: " + tcp[r];
        } else {
            return;    // VLAN reject, TTL expiry: the replaced elements print nothing
        }
        P::chatter(m);
    }

    // Packets [b, e) of a completed slot: the device's results into each
    // packet (headers, trim, annotations, rewritten bytes, strip). Packets were
    // staged one batch ago, so their lines are prefetched well ahead.
    void annotate(Slot &s, uint32_t b, uint32_t e) {
        constexpr uint32_t kAhead = 16;
        const bool hashing = _cfg.hash_mode != FCGPU_HASH_NONE;
        const bool autom = _cfg.check_mode == FCGPU_CHECK_AUTO;
        // loop invariants in locals: the annotation stores below may alias
        // any member of a matching type, so the compiler reloads members
        const int color = _color;
        const bool strip = _strip;
        const int flow_anno = _flow_anno;
        const uint32_t offset = (uint32_t)_cfg.offset, n = s.n;
        const fcgpu_anno8 *const anno8 = s.anno8;
        const fcgpu_anno *const anno = s.anno;
        const uint16_t *const verdict = s.verdict;
        const uint32_t *const hash = s.hash, *const flowid = s.flowid, *const iprw = s.iprw;
        Packet **const pkts = s.pkts.data();
        for (uint32_t i = b; i < e && i < b + kAhead; ++i) prefetch_packet(pkts[i]);
        for (uint32_t i = b; i < e; ++i) {
            Packet *p = pkts[i];
            if (i + kAhead < n) prefetch_packet(pkts[i + kAhead]);
            fcgpu_anno a8v;
            if (anno8) {                                  // IPv4 chain: the 8-B form
                const fcgpu_anno8 &q = anno8[i];
                a8v = fcgpu_anno{q.dst_ip, q.length, 0, q.nh, (uint16_t)(q.nh + q.thl), 0, 4, 0};
            }
            const fcgpu_anno &a = anno8 ? a8v : anno[i];
            const uint32_t reason = verdict[i] & 0xff;
            if (color >= 0) P::set_anno_u8(p, P::kPaint, (uint8_t)color);       // SET_PAINT_ANNO
            if (autom && reason != FCGPU_R_VLAN_REJECT)
                P::set_anno_u16(p, P::kVlanTci, a.vlan_tci);                     // StripEtherVLANHeader
            if (reason == FCGPU_R_OK || reason >= FCGPU_R_NO_MATCH) {
                // DecIPTTL / SetIPChecksum: ip_rw holds every R_OK packet's bytes
                // 8..11 as they leave; only a changed word is written back
                if (iprw && reason == FCGPU_R_OK && memcmp(P::data(p) + a.nh + 8u, &iprw[i], 4) != 0) {
                    Packet *q = P::write_bytes(p, a.nh + 8u, &iprw[i], 4);
                    if (!q) {                                                    // uniqueify failed: freed
                        pkts[i] = nullptr;
                        s.holes = true;
                        continue;
                    }
                    pkts[i] = p = q;
                }
                P::set_headers(p, a.nh, a.th);                                   // set_ip_header / set_ip6_header
                if (a.length < P::length(p)) P::take(p, P::length(p) - a.length);
                if (a.ipver == 6) P::set_anno_u8(p, P::kIp6Nxt, a.ip6_nxt);
                else P::set_anno_u32(p, P::kDstIp, a.dst_ip);
                if (hashing && reason <= FCGPU_R_NO_MATCH)                       // AggregateHash (not after an L4 drop)
                    P::set_anno_u32(p, P::kAggregate, hash[i]);
                if (flowid && flowid[i] != FCGPU_FLOW_NONE && flowid[i] != FCGPU_FLOW_FULL)
                    P::set_anno_u32(p, flow_anno, flowid[i]);
                if (strip) P::pull(p, a.nh);
                if (reason > FCGPU_R_NO_MATCH) drop_chatter(reason);
            } else {
                drop_chatter(reason);
                // the replaced Strip / StripEtherVLANHeader ran before the checker
                if (strip && reason != FCGPU_R_VLAN_REJECT) P::pull(p, autom ? a.nh : offset);
            }
        }
    }
    // the Packet object's first three lines (header pointers, data/length,
    // annotations: FastClick's Packet is 168 B, packet.hh:874-941)
    static inline void prefetch_packet(const Packet *p) {
        const char *c = reinterpret_cast<const char *>(p);
        __builtin_prefetch(c, 1);
        __builtin_prefetch(c + 64, 1);
        __builtin_prefetch(c + 128, 1);
    }

    // Results of slot k back into its packets, then its output runs leave.
    template <class Emit>
    void complete(uint32_t k, Emit &emit) {
        Slot &s = _slot[k];
        const uint32_t n = s.n;
        fcgpu_block_layout L;
        bool failed = false;
        {
            std::lock_guard<std::mutex> g(_mu);
            int rc = fcgpu_span_wait(_ctx, k);
            s.inflight = false;
            if (rc != FCGPU_OK) {
                rc = resubmit(k);
                if (rc == FCGPU_OK) rc = fcgpu_span_wait(_ctx, k);
            }
            if (rc == FCGPU_OK) fcgpu_block_layout_for(_ctx, n, _outputs, _partition, &L);
            else failed = true;
        }
        if (failed) {
            fail_slot(s, emit);
            return;
        }
        s.holes = false;
        s.map(L, (_outputs & FCGPU_OUT_ANNO8) != 0);
        const uint32_t nb = _cfg.nports + 1;
        if (_partition == FCGPU_PART_GLOBAL) {
            annotate(s, 0, n);
            // one batch per output in port order, input order within a port
            for (uint32_t port = 0; port < nb; ++port)
                emit_run(s, port, s.start[port], s.start[port + 1], [&s](uint32_t j) { return s.perm[j]; }, emit);
        } else {
            // every FCGPU_TILE-packet tile is one classified PacketBatch: its
            // runs leave in port order, tiles in input order. A tile's packets
            // are annotated and linked into its output runs in one visit, while
            // their Packet lines are in the CPU cache (annotating the whole
            // batch first and linking after touched every Packet twice, 16K
            // packets apart: twice from DRAM once a few threads share an L3)
            const uint32_t ntiles = (n + FCGPU_TILE - 1) / FCGPU_TILE;
            for (uint32_t t = 0; t < ntiles; ++t) {
                const uint32_t base = t * FCGPU_TILE;
                annotate(s, base, base + FCGPU_TILE < n ? base + FCGPU_TILE : n);
                uint32_t b = base;
                auto idx = [&s, base](uint32_t j) { return base + s.tperm[j]; };
                const uint16_t *tc = s.tile_count + (size_t)t * nb;
                for (uint32_t port = 0; port < nb; ++port) {
                    const uint32_t c = tc[port];
                    if (c) emit_run(s, port, b, b + c, idx, emit);
                    b += c;
                }
            }
        }
        s.n = 0;
        s.used = 0;
    }

    // link the packets idx(b) .. idx(e-1) into PacketBatches of <= kMaxBatch
    template <class Idx, class Emit>
    void emit_run(Slot &s, uint32_t port, uint32_t b, uint32_t e, Idx idx, Emit &emit) {
        const bool nomatch = port == _cfg.nports && _cfg.classify == FCGPU_CLS_PROGRAM;
        const bool last = port == _cfg.nports;
        if (nomatch || (last && _cfg.rewrite) || s.flowid || s.holes) {
            // the last list mixes invalid packets (output N) and packets no
            // rule matched or SetIPChecksum rejected (killed); a full flow
            // table kills new flows. The rest keep input order.
            uint32_t w = 0;
            for (uint32_t j = b; j < e; ++j) {
                const uint32_t i = idx(j);
                Packet *p = s.pkts[i];
                const uint32_t r = s.verdict[i] & 0xff;
                if (!p) continue;                                     // freed by a failed uniqueify
                if ((nomatch && r == FCGPU_R_NO_MATCH) || (last && r == FCGPU_R_SETCKSUM_BAD)) {
                    P::kill(p);
                } else if (s.flowid && s.flowid[i] == FCGPU_FLOW_FULL) {
                    _flow_drops.fetch_add(1, std::memory_order_relaxed);
                    P::kill(p);
                } else {
                    s.keep[w++] = i;
                }
            }
            // FLOW_RUNS: consecutive packets of one flow leave as one batch
            // (the BatchBuilder of FlowIPManagerHMP::process and
            // VirtualFlowManagerIMP::process, flowipmanagerhmp.cc:101-117,
            // virtualflowmanager.hh:304-326); killed packets do not end a run
            const bool runs = _flow_runs && s.flowid && !last;
            for (uint32_t a = 0; a < w;) {
                uint32_t k = w - a < kMaxBatch ? w - a : kMaxBatch;
                if (runs) {
                    const uint32_t f = s.flowid[s.keep[a]];
                    uint32_t j = 1;
                    while (j < k && s.flowid[s.keep[a + j]] == f) ++j;
                    k = j;
                }
                Packet *head = s.pkts[s.keep[a]], *prev = head;
                for (uint32_t j = 1; j < k; ++j) {
                    Packet *q = s.pkts[s.keep[a + j]];
                    P::set_next(prev, q);
                    prev = q;
                }
                emit((int)port, P::make_batch(head, prev, k));
                a += k;
            }
            return;
        }
        while (b < e) {
            const uint32_t m = e - b < kMaxBatch ? e - b : kMaxBatch;
            Packet *head = s.pkts[idx(b)], *prev = head;
            for (uint32_t j = 1; j < m; ++j) {
                Packet *q = s.pkts[idx(b + j)];
                P::set_next(prev, q);
                prev = q;
            }
            emit((int)port, P::make_batch(head, prev, m));
            b += m;
        }
    }

    fcgpu_cfg _cfg;
    fcgpu_ctx *_ctx = nullptr;
    bool _lb_direct = false;          // LB_MODE hash (IPFlowID), not hash_agg
    uint32_t _cst_buckets = 0;        // CST_BUCKETS (0: 100 per output)
    ParsedProgram _prog;
    uint32_t _prog_kind = FCGPU_PROG_IPFILTER;
    bool _prog_jit = true;
    int _color = -1;
    uint32_t _flow_cap = 0;
    uint32_t _flow_mgr = FCGPU_FLOW_MGR_HMP, _flow_timeout = 0, _flow_recycle_ms = 1000;
    uint64_t _next_maint_ms = 0;     // the next maintainer run, ms on the element's clock
    bool _maint_armed = false;
    int _flow_anno = 28;
    bool _flow_runs = true;
    std::atomic<uint64_t> _flow_drops{0};       // read by handlers on other threads
    std::atomic<uint64_t> _gpu_errors{0}, _gpu_killed{0}, _gpu_retries{0};
    int _error_output = -1;                      // ERROR_OUTPUT (-1: kill)
    std::string _fail_msg;                       // the failure that caused the last re-submission (under _mu)
    int _device = 0;
    // BATCH auto: packets per batch while batches are copied, while they go
    // zero-copy, and zero-copy with compact records (half the PCIe bytes per
    // packet: bigger batches amortise the round trip; profiles/r04_crossover)
    static constexpr uint32_t kBatchCopy = 16384, kBatchZeroCopy = 4096, kBatchZeroCopyCompact = 8192;
    uint32_t _batch = kBatchCopy;
    bool _batch_auto = true;                     // BATCH auto (the default)
    uint32_t _eff_batch = kBatchCopy;            // packets per device batch now (BATCH auto: by the span path)
    int64_t _timer_us = 100;
    uint32_t _cap = 0;
    uint32_t _capture = fcgpu::kCaptureMin;
    fcgpu::StagePlan _plan;                      // compact records (capture.hh) when the chain allows them
    bool _compact = true;                        // COMPACT
    uint32_t _lead = 0;                          // compact: records start this far into the block
    bool _desc32 = false;                        // compact records: 4-B descriptors while they fit
    // DESC32 frame offsets reach 65535 x 8 B
    static constexpr size_t kDesc32Reach = 0xffffu * 8u;
    uint32_t _partition = FCGPU_PART_TILE;
    uint32_t _span_mode = FCGPU_SPAN_AUTO;       // ZEROCOPY: the kernels read/write the pinned slots in place
    uint32_t _outputs = 0;                       // FCGPU_OUT_* the element asks for
    bool _verbose = false, _details = false, _strip = false, _warned = false;
    std::string _error;                         // under _mu
    mutable std::mutex _mu;                     // the context and _error (see counters())
    Slot _slot[kMaxSlots];
    uint32_t _nslots = 2;
    uint32_t _cur = 0;
};

}  // namespace fcx
