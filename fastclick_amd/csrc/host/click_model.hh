// click_model.hh -- minimal Click-shaped packet/batch/element model (host C++).
//
// Just enough of FastClick's data model for the GPU element to be driven the
// way FastClick drives a BatchElement, with the same semantics:
//   - Packet: data/length with headroom, 48-byte annotation area, network and
//     transport header marks; pull()/take() as include/click/packet.hh:2122-2207
//     (take clamps to the length).
//   - PacketBatch: a singly linked list threaded through the packets; the head
//     carries the count (BATCH_COUNT_ANNO, 16-bit, packet_anno.hh:90-93) and
//     the tail (the head's prev), as include/click/packetbatch.hh:413-476.
//   - Element / Port: push_batch(port, batch) dispatch along connections,
//     checked_output_push_batch kills batches sent to a missing output
//     (include/click/batchelement.hh:54-62).
// Annotation offsets follow include/click/packet_anno.hh: DST_IP @0 (4),
// IP6_NXT @16 (1), VLAN_TCI @20 (2), AGGREGATE @20 (4), BATCH_COUNT @24 (2).
#pragma once
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <string>
#include <vector>
#include <atomic>

#include "click_args.hh"

namespace fcx {

enum { ANNO_SIZE = 48, DST_IP_ANNO_OFFSET = 0, IP6_NXT_ANNO_OFFSET = 16, PAINT_ANNO_OFFSET = 17,
       VLAN_TCI_ANNO_OFFSET = 20, AGGREGATE_ANNO_OFFSET = 20, BATCH_COUNT_ANNO_OFFSET = 24 };

class PacketPool;

class Packet {
  public:
    uint8_t *buffer() const { return _buf; }
    uint32_t buffer_length() const { return _cap; }
    uint8_t *data() const { return _buf + _data; }
    uint32_t length() const { return _len; }
    uint32_t headroom() const { return _data; }
    uint32_t tailroom() const { return _cap - _data - _len; }
    const uint8_t *end_data() const { return data() + _len; }

    // Packet::pull (packet.hh:2122-2140): clamps to the length
    void pull(uint32_t n) {
        if (n > _len) n = _len;
        _data += n;
        _len -= n;
        _nh = _nh >= (int)n ? _nh - (int)n : -1;
        _th = _th >= (int)n ? _th - (int)n : -1;
    }
    void push(uint32_t n) { _data -= n; _len += n; if (_nh >= 0) _nh += n; if (_th >= 0) _th += n; }
    // Packet::take (packet.hh:2189-2207): clamps to the length
    void take(uint32_t n) { _len -= (n > _len ? _len : n); }

    // header marks (offsets from data(); -1 = unset)
    bool has_network_header() const { return _nh >= 0; }
    bool has_transport_header() const { return _th >= 0; }
    const uint8_t *network_header() const { return _nh >= 0 ? data() + _nh : nullptr; }
    const uint8_t *transport_header() const { return _th >= 0 ? data() + _th : nullptr; }
    int network_header_offset() const { return _nh; }
    int transport_header_offset() const { return _th; }
    void set_network_header(int nh, int th) { _nh = nh; _th = th; }

    uint8_t *anno_u8() { return _anno; }
    uint8_t anno_u8(int o) const { return _anno[o]; }
    uint16_t anno_u16(int o) const { uint16_t v; memcpy(&v, _anno + o, 2); return v; }
    uint32_t anno_u32(int o) const { uint32_t v; memcpy(&v, _anno + o, 4); return v; }
    void set_anno_u8(int o, uint8_t v) { _anno[o] = v; }
    void set_anno_u16(int o, uint16_t v) { memcpy(_anno + o, &v, 2); }
    void set_anno_u32(int o, uint32_t v) { memcpy(_anno + o, &v, 4); }
    void clear_annotations() { memset(_anno, 0, sizeof(_anno)); }

    Packet *next() const { return _next; }
    Packet *prev() const { return _prev; }
    void set_next(Packet *p) { _next = p; }
    void set_prev(Packet *p) { _prev = p; }

    uint32_t id = 0;   // harness-only: index of the packet in its input trace

    void kill();

  private:
    friend class PacketPool;
    uint8_t *_buf = nullptr;
    uint32_t _cap = 0, _data = 0, _len = 0;
    int _nh = -1, _th = -1;
    Packet *_next = nullptr, *_prev = nullptr;
    PacketPool *_pool = nullptr;
    alignas(8) uint8_t _anno[ANNO_SIZE] = {};
};

// Fixed pool of packets with private buffers (headroom + data).
class PacketPool {
  public:
    PacketPool(uint32_t n, uint32_t bufsize, uint32_t headroom = 128)
        : _pk(n), _store((size_t)n * bufsize), _headroom(headroom) {
        for (uint32_t i = 0; i < n; ++i) {
            _pk[i]._buf = _store.data() + (size_t)i * bufsize;
            _pk[i]._cap = bufsize;
            _pk[i]._pool = this;
            _free.push_back(&_pk[i]);
        }
    }
    Packet *make(const uint8_t *frame, uint32_t len) {
        if (_free.empty()) return nullptr;
        Packet *p = _free.back();
        _free.pop_back();
        p->_data = _headroom;
        p->_len = len;
        if (frame) memcpy(p->data(), frame, len);
        p->_nh = p->_th = -1;
        p->_next = p->_prev = nullptr;
        p->clear_annotations();
        return p;
    }
    void recycle(Packet *p) { _free.push_back(p); }
    size_t available() const { return _free.size(); }

  private:
    std::vector<Packet> _pk;
    std::vector<uint8_t> _store;
    std::vector<Packet *> _free;
    uint32_t _headroom;
};

inline void Packet::kill() {
    if (_pool) _pool->recycle(this);
}

// PacketBatch: the head packet; count in BATCH_COUNT_ANNO, tail in head->prev.
class PacketBatch {
  public:
    static PacketBatch *start_head(Packet *p) { return reinterpret_cast<PacketBatch *>(p); }
    Packet *first() { return reinterpret_cast<Packet *>(this); }
    Packet *tail() { return first()->prev(); }
    void set_tail(Packet *t) { first()->set_prev(t); }
    unsigned count() { return first()->anno_u16(BATCH_COUNT_ANNO_OFFSET); }
    void set_count(unsigned c) { first()->set_anno_u16(BATCH_COUNT_ANNO_OFFSET, (uint16_t)c); }
    void append_packet(Packet *p) {
        tail()->set_next(p);
        set_tail(p);
        set_count(count() + 1);
    }
    // make_from_simple_list (packetbatch.hh): link [head..tail] of count packets
    static PacketBatch *make_from_list(Packet *head, Packet *tail, unsigned count) {
        PacketBatch *b = start_head(head);
        tail->set_next(nullptr);
        b->set_tail(tail);
        b->set_count(count);
        return b;
    }
    void kill() {
        Packet *p = first();
        while (p) {
            Packet *n = p->next();
            p->kill();
            p = n;
        }
    }
};

class Element;

struct Port {
    Element *e = nullptr;
    int port = 0;
};

class Element {
  public:
    virtual ~Element() {}
    virtual const char *class_name() const = 0;
    virtual int configure(const std::vector<std::string> &conf, std::string &errh) = 0;
    virtual int initialize(std::string &) { return 0; }
    virtual void push_batch(int port, PacketBatch *batch) = 0;
    // Per-packet entry for non-batch upstreams (Element::push, lib/element.cc:3141-3147;
    // with batching on, Port::push hands a lone packet to a batch element the same way,
    // include/click/element.hh:765-790). Default: a one-packet batch.
    virtual void push(int port, Packet *p) {
        push_batch(port, PacketBatch::make_from_list(p, p, 1));
    }
    virtual std::string read_handler(const std::string &) { return std::string(); }
    virtual void flush() {}
    // A Timer firing at now_ns (Element::run_timer); true = reschedule it.
    virtual bool run_timer(uint64_t) { return false; }
    // packets the element holds (staged or on the device)
    virtual uint32_t held() const { return 0; }
    // the most packets the element may hold at once (staged + in flight)
    virtual uint32_t max_held() const { return 0; }

    int noutputs() const { return (int)_out.size(); }
    void connect_output(int i, Element *e, int port) {
        if ((int)_out.size() <= i) _out.resize(i + 1);
        _out[i].e = e;
        _out[i].port = port;
    }
    void set_noutputs(int n) { _out.resize(n); }
    void output_push_batch(int i, PacketBatch *b) {
        if (_out[i].e) _out[i].e->push_batch(_out[i].port, b);
        else b->kill();
    }
    // batchelement.hh:54-62
    void checked_output_push_batch(int i, PacketBatch *b) {
        if ((unsigned)i < (unsigned)noutputs()) output_push_batch(i, b);
        else b->kill();
    }

  protected:
    std::vector<Port> _out;
};

}  // namespace fcx
