// gpu_element.hh -- GPUIPCheckClassify on the test harness's packet model.
//
// The element logic is RxCore (gpu_core.hh), shared with the FastClick
// element (fastclick_pkg/gpuipcheckclassify.{hh,cc}); ModelPolicy maps its
// Packet/PacketBatch operations onto click_model.hh, which mirrors the
// FastClick data model (include/click/packet.hh, packetbatch.hh). This class
// is what libfcclick.so drives in the tests and the host-rate benchmark.
#pragma once
#include <atomic>
#include <chrono>
#include <string>
#include <vector>

#include "click_model.hh"
#include "gpu_core.hh"

namespace fcx {

struct ModelPolicy {
    using Packet = fcx::Packet;
    using Batch = fcx::PacketBatch;
    static constexpr int kAnnoSize = ANNO_SIZE;
    static constexpr int kDstIp = DST_IP_ANNO_OFFSET, kIp6Nxt = IP6_NXT_ANNO_OFFSET, kPaint = PAINT_ANNO_OFFSET,
                         kVlanTci = VLAN_TCI_ANNO_OFFSET, kAggregate = AGGREGATE_ANNO_OFFSET;
    static const uint8_t *data(Packet *p) { return p->data(); }
    static uint32_t length(Packet *p) { return p->length(); }
    static Packet *next(Packet *p) { return p->next(); }
    static void set_next(Packet *p, Packet *q) { p->set_next(q); }
    static void kill(Packet *p) { p->kill(); }
    static void set_anno_u8(Packet *p, int o, uint8_t v) { p->set_anno_u8(o, v); }
    static void set_anno_u16(Packet *p, int o, uint16_t v) { p->set_anno_u16(o, v); }
    static void set_anno_u32(Packet *p, int o, uint32_t v) { p->set_anno_u32(o, v); }
    static void set_headers(Packet *p, uint32_t nh, uint32_t th) { p->set_network_header((int)nh, (int)th); }
    static void take(Packet *p, uint32_t n) { p->take(n); }
    static void pull(Packet *p, uint32_t n) { p->pull(n); }
    // the harness's packets are never shared: written in place
    static Packet *write_bytes(Packet *p, uint32_t off, const void *src, uint32_t len) {
        memcpy(p->data() + off, src, len);
        return p;
    }
    static Batch *make_batch(Packet *h, Packet *t, unsigned n) { return PacketBatch::make_from_list(h, t, n); }
    // the harness's clock: steady_clock, or the virtual time a clocked run
    // sets before each burst (fcclick_run_clocked)
    static inline std::atomic<uint64_t> virtual_ns{0};
    static uint64_t now_ns() {
        const uint64_t v = virtual_ns.load(std::memory_order_relaxed);
        if (v) return v;
        return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                   std::chrono::steady_clock::now().time_since_epoch()).count();
    }
    static void chatter(const std::string &m) { fprintf(stderr, "%s\n", m.c_str()); }
};

class GPUIPCheckClassify : public Element {
  public:
    const char *class_name() const override { return "GPUIPCheckClassify"; }
    int configure(const std::vector<std::string> &conf, std::string &errh) override {
        _core.name = class_name();
        return _core.configure(conf, errh);
    }
    int initialize(std::string &errh) override { return _core.initialize(errh); }
    void push_batch(int, PacketBatch *batch) override { _core.push_list(batch->first(), emitter()); }
    // A non-batch upstream (Element::push, lib/element.cc:3141-3147): the
    // packet is staged like any other
    void push(int, Packet *p) override {
        p->set_next(nullptr);
        _core.push_one(p, emitter());
    }
    void flush() override { _core.flush(emitter()); }
    bool run_timer(uint64_t now_ns) override { return _core.run_timer(now_ns, emitter()); }
    uint32_t held() const override { return _core.held(); }
    uint32_t max_held() const override { return _core.max_held(); }
    std::string read_handler(const std::string &h) override { return _core.read_handler(h); }
    const fcgpu_cfg &device_cfg() const { return _core.device_cfg(); }

  private:
    struct Emit {          // RxCore hands each output run here
        GPUIPCheckClassify *e;
        void operator()(int port, PacketBatch *b) const { e->checked_output_push_batch(port, b); }
        int noutputs() const { return e->noutputs(); }
    };
    Emit emitter() { return Emit{this}; }
    RxCore<ModelPolicy> _core;
};

}  // namespace fcx
