#ifndef CLICK_GPUIPCHECKCLASSIFY_HH
#define CLICK_GPUIPCHECKCLASSIFY_HH
/*
 * GPUIPCheckClassify -- the MI355X receive-path element as a FastClick
 * package element (etc/samplepackage layout).
 *
 * A BatchElement (include/click/batchelement.hh:29-125) whose push_batch
 * replaces the CPU chain
 *     [Strip(14) | StripEtherVLANHeader] -> CheckIPHeader / CheckIP6Header
 *         -> AggregateHash -> FlowSwitch(LB_MODE hash) | HashSwitch | IPClassifier
 * by one batched pass on the GPU (libfcgpu.so, include/fastclick_gpu.h).
 * The element logic is fcx::RxCore (fastclick_amd/csrc/host/gpu_core.hh),
 * the same code the repository's tests drive through the harness model;
 * ClickPolicy below maps its packet operations onto FastClick's Packet and
 * PacketBatch (include/click/packet.hh, packetbatch.hh).
 *
 * Threads: one RxCore -- one GPU context, two pinned staging slots, one
 * Timer -- per Click thread that pushes into the element (per_thread<>,
 * include/click/sync.hh:56), as FastClick keeps per-thread element state;
 * counters are summed on read (PER_THREAD_SUM, sync.hh:384). Accumulation and
 * the TIMER flush follow MinBatch (elements/standard/minbatch.cc:35,57-76).
 *
 * Keyword arguments and handlers: see gpu_core.hh.
 *
 * =c
 * GPUIPCheckClassify(KEYWORDS)
 * =s ip
 * checks IP headers, hashes flows and classifies packets on an AMD GPU
 */
#include <click/batchelement.hh>
#include <click/packet.hh>
#include <click/packet_anno.hh>
#include <click/packetbatch.hh>
#include <click/timer.hh>
#include <click/timestamp.hh>
#include <click/sync.hh>
#include "gpu_core.hh"   // -I fastclick_amd/csrc/host (Makefile)
CLICK_DECLS

struct ClickPolicy {
    typedef ::Packet Packet;
    typedef ::PacketBatch Batch;
    static constexpr int kAnnoSize = Packet::anno_size;
    static constexpr int kDstIp = DST_IP_ANNO_OFFSET, kIp6Nxt = IP6_NXT_ANNO_OFFSET,
                         kPaint = PAINT_ANNO_OFFSET, kVlanTci = VLAN_TCI_ANNO_OFFSET,
                         kAggregate = AGGREGATE_ANNO_OFFSET;
    static const uint8_t *data(Packet *p) { return p->data(); }
    static uint32_t length(Packet *p) { return p->length(); }
    static Packet *next(Packet *p) { return p->next(); }
    static void set_next(Packet *p, Packet *q) { p->set_next(q); }
    static void kill(Packet *p) { p->kill(); }
    static void set_anno_u8(Packet *p, int o, uint8_t v) { p->set_anno_u8(o, v); }
    static void set_anno_u16(Packet *p, int o, uint16_t v) { p->set_anno_u16(o, v); }
    static void set_anno_u32(Packet *p, int o, uint32_t v) { p->set_anno_u32(o, v); }
    // set_ip_header / set_ip6_header (packet.hh:2493-2516): network header
    // at nh, transport header at th
    static void set_headers(Packet *p, uint32_t nh, uint32_t th) {
        p->set_network_header(p->data() + nh, th - nh);
    }
    static void take(Packet *p, uint32_t n) { p->take(n); }
    static void pull(Packet *p, uint32_t n) { p->pull(n); }
    // DecIPTTL / SetIPChecksum write the header: uniqueify first (a shared
    // packet is copied; null = freed on failure), as those elements do
    static Packet *write_bytes(Packet *p, uint32_t off, const void *src, uint32_t len) {
        WritablePacket *q = p->uniqueify();
        if (!q) return 0;
        memcpy(q->data() + off, src, len);
        return q;
    }
    static Batch *make_batch(Packet *h, Packet *t, unsigned n) {
        return PacketBatch::make_from_simple_list(h, t, n);
    }
    static uint64_t now_ns() { return (uint64_t)Timestamp::now_steady().nsecval(); }
    static void chatter(const std::string &m) { click_chatter("%s", m.c_str()); }
};

class GPUIPCheckClassify : public BatchElement { public:

    GPUIPCheckClassify() CLICK_COLD;
    ~GPUIPCheckClassify() CLICK_COLD;

    const char *class_name() const override { return "GPUIPCheckClassify"; }
    const char *port_count() const override { return "1/1-"; }
    const char *processing() const override { return PUSH; }

    int configure(Vector<String> &conf, ErrorHandler *errh) override CLICK_COLD;
    int initialize(ErrorHandler *errh) override CLICK_COLD;
    void cleanup(CleanupStage stage) override CLICK_COLD;
    void add_handlers() override CLICK_COLD;

    void push_batch(int port, PacketBatch *batch) override;
    void push(int port, Packet *p) override;
    void run_timer(Timer *timer) override;

  private:
    typedef fcx::RxCore<ClickPolicy> Core;
    struct State {
        Core *core;
        Timer *timer;
        State() : core(0), timer(0) {}
    };
    struct Emit {
        GPUIPCheckClassify *e;
        void operator()(int port, PacketBatch *b) const { e->checked_output_push_batch(port, b); }
        int noutputs() const { return e->noutputs(); }
    };

    int make_state(int thread, ErrorHandler *errh);
    void arm(State &s);
    static String read_handler(Element *e, void *thunk);

    per_thread<State> _state;
    std::vector<std::string> _conf;
    int64_t _timer_us;
    int _error_output;
};

CLICK_ENDDECLS
#endif
