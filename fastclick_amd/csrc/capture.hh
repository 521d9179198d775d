// capture.hh -- how many leading bytes of each frame a host-resident batch
// must hand to the device (host code shared by fcgpu_process_host and the
// GPUIPCheckClassify element's staging).
//
// The device reads a frame's header window and, past it, whatever the
// configured chain looks at; bytes beyond that never decide a verdict, an
// annotation or an output. Staging only the reach (rounded up to whole 64-B
// slots, at least 128 B) keeps the PCIe copy at ~64-128 B per packet.
#pragma once
#include <stdint.h>
#include "../../include/fastclick_gpu.h"

namespace fcgpu {

constexpr uint32_t kCaptureWhole = 0xffffffffu;
constexpr uint32_t kCaptureMin = 128;

// Bytes from the frame start a decision program may read (IPFilter offsets
// >= 512 are transport-relative, >= 256 network-relative, else MAC - 2,
// elements/ip/ipfilter.hh:393-481; Classifier offsets are frame-relative).
// `l3` is the farthest a network header can start; `l4` the farthest a
// transport header can start.
inline uint32_t program_reach(uint32_t kind, const fcgpu_step *steps, uint32_t n, uint32_t l3, uint32_t l4) {
    uint32_t r = 0;
    for (uint32_t k = 0; k < n; ++k) {
        const int32_t o = steps[k].offset;
        uint32_t end;
        if (kind == FCGPU_PROG_IPFILTER)
            end = o >= 512 ? l4 + (uint32_t)(o - 512) + 4 : o >= 256 ? l3 + (uint32_t)(o - 256) + 4
                                                                   : (o > 2 ? (uint32_t)o - 2 : 0u) + 4;
        else
            end = (o > 0 ? (uint32_t)o : 0u) + 4;
        r = end > r ? end : r;
    }
    return r;
}

// prog_reach: program_reach() of the installed program (0 without one).
inline uint32_t capture_bytes(const fcgpu_cfg &c, uint32_t prog_reach) {
    // the L4 checksum covers the segment, PROCESS_EH follows any number of
    // extension headers: whole frames
    if (c.l4_mode != FCGPU_L4_NONE && c.l4_checksum) return kCaptureWhole;
    const bool autom = c.check_mode == FCGPU_CHECK_AUTO;
    if (autom && c.process_eh) return kCaptureWhole;
    const uint32_t l3 = (uint32_t)c.offset + (autom ? 18u : 0u);   // StripEtherVLANHeader: 14 or 18
    // IPv4: up to 60 B of header then the L4 words the checks and hashes read
    // (ports, UDP length/checksum, TCP offset: 16 B); IPv6: 40 B + the same
    const uint32_t l4 = l3 + 60;
    uint32_t need = l4 + 16;
    if (c.classify == FCGPU_CLS_HASHSWITCH) {
        const uint32_t e = (uint32_t)c.hs_offset + (uint32_t)c.hs_length;
        need = e > need ? e : need;
    }
    if (c.classify == FCGPU_CLS_HASH_IP && need < 34) need = 34;
    if (prog_reach > need) need = prog_reach;
    need = (need + 63) & ~63u;
    return need < kCaptureMin ? kCaptureMin : need;
}

// Records start on kStageAlign-byte boundaries: the device reads a record
// through 16-B aligned windows wherever it starts, and the PCIe bytes per
// packet are the records' bytes (neighbouring records share the window
// lines), so the finer the packing, the fewer bytes cross (C2: 24-B records
// instead of 32). Rest-of-frame records (L4 checksums) keep 16-B packing:
// with every frame then at the same place in its 16-B aligned window, a small
// datagram lies inside the window the device loads and is summed there
// instead of read again (k_rx win_l4_sum).
constexpr uint32_t kStageAlign = 8;

// Compact staging (the element's block records). For the IPv4 chains whose
// reads all fall in [start, o + max(hl, 20) + tail) of each frame -- CheckIPHeader /
// MarkIPHeader at OFFSET o (header, options, addresses), the ports IPFlowID /
// IPFlow5ID read at th = o + hl (AggregateHash, FlowSwitch LB hash / hash_crc,
// the flow table), CheckUDPHeader / CheckTCPHeader's length words without
// their checksum (tail 16), DecIPTTL / SetIPChecksum (header), LB hash_ip's
// bytes 26..33 and HashSwitch's range -- a record holds only those bytes: the
// descriptor points `start` bytes before the record, so the device finds
// every byte it reads at its frame offset, and bytes outside the range (the
// neighbouring records) are never part of a decision. A 60-B UDP frame then
// stages 24 B instead of 64. With CheckUDPHeader / CheckTCPHeader's checksum
// (the datagram, whatever its length) a record holds the frame from OFFSET to
// its end: 46 of a 60-B frame's bytes. Chains that read anywhere in the frame
// (AUTO with VLAN / IPv6, decision programs) keep whole captures.
struct StagePlan {
    bool compact = false;
    bool rest = false;        // the record runs to the frame's end (L4 checksums)
    uint32_t align = 8;       // record packing (rest-of-frame records: 16, see stage_record_size)
    uint32_t start = 0;       // first frame byte any stage reads
    uint32_t fixed_end = 0;   // frame bytes every packet needs up to (hash_ip, HashSwitch)
    uint32_t tail = 4;        // bytes past th: ports (4) or the L4 length checks' words (16)
};
inline StagePlan stage_plan(const fcgpu_cfg &c) {
    StagePlan p;
    const bool ip4 = c.check_mode == FCGPU_CHECK_IP4 || c.check_mode == FCGPU_MARK_IP4;
    if (!ip4 || c.classify == FCGPU_CLS_PROGRAM) return p;
    p.compact = true;
    p.rest = c.l4_mode != FCGPU_L4_NONE && c.l4_checksum;
    p.align = p.rest ? 16u : kStageAlign;
    p.start = (uint32_t)c.offset;
    p.tail = c.l4_mode != FCGPU_L4_NONE ? 16u : 4u;
    if (c.classify == FCGPU_CLS_HASH_IP) {
        p.start = p.start < 26u ? p.start : 26u;
        p.fixed_end = 34;
    } else if (c.classify == FCGPU_CLS_HASHSWITCH) {
        const uint32_t o = (uint32_t)c.hs_offset, e = o + (uint32_t)c.hs_length;
        p.start = p.start < o ? p.start : o;
        p.fixed_end = e;
    }
    return p;
}
// The frame bytes [plan.start, end) a packet's record must hold.
inline uint32_t stage_end(const StagePlan &p, uint32_t offset, const uint8_t *frame, uint32_t len) {
    if (p.rest) return len;
    uint32_t end = p.fixed_end;
    if (len > offset) {
        // th + tail, and never less than the 20-B header: MarkIPHeader takes
        // any hl, and IPFlowID / DST_IP read the addresses at o + 12..19
        const uint32_t hl = (uint32_t)(frame[offset] & 15) << 2;
        const uint32_t e = offset + (hl > 20u ? hl : 20u) + (hl >= 20u ? p.tail : 0u);
        const uint32_t ep = offset + hl + p.tail;
        end = e > end ? e : end;
        end = ep > end ? ep : end;
    }
    return end < len ? end : len;
}
constexpr uint32_t kStageLead = 256;   // records start this far into the block (descriptor offsets >= 0)


// One packet's compact record: copy cp bytes from frame + src_off; the record
// takes the returned size (a multiple of p.align, at least p.align)
// and the packet's descriptor offset is the record's offset minus p.start.
inline uint32_t stage_record_size(const StagePlan &p, uint32_t offset, const uint8_t *frame, uint32_t len,
                                  uint32_t &src_off, uint32_t &cp) {
    const uint32_t end = stage_end(p, offset, frame, len);
    cp = end > p.start ? end - p.start : 0u;
    src_off = cp ? p.start : 0u;
    return cp ? (cp + p.align - 1) & ~(p.align - 1) : p.align;
}

}  // namespace fcgpu
