// fcgpu_device.hh -- device code of the receive-path element library (gfx950).
//
// One lane per packet, 64 packets per wave, 256 packets per workgroup tile.
// Each wave gathers the first 64 bytes of its 64 frames into LDS with four
// 1-KiB LDS-DMA instructions (global_load_lds_dwordx4, per-lane source address
// = arena + frame offset), so four consecutive lanes fetch one frame's 64 B as
// one contiguous 64-B segment. Chunks are XOR-swizzled per row so that the
// b128 lane groups hit distinct LDS slots. Each lane then parses its own row
// with 4-B LDS reads at runtime offsets (IP header offset, transport offset),
// falling back to aligned global loads for bytes past the 64-B window (IPv4
// options, large OFFSET): correctness never depends on the window size.
//
// Integer/byte work only; no MFMA. The kernel is bound by HBM read bytes:
// 8 B descriptor + 64 B window per packet.
#pragma once
#ifndef __HIPCC_RTC__   // hiprtc provides the HIP runtime declarations itself
#include <hip/hip_runtime.h>
#include <stdint.h>
#endif
#include "../../include/fastclick_gpu.h"

namespace fcgpu {

constexpr int kWave = 64;
constexpr int kTile = 256;                  // packets per workgroup (4 waves)
constexpr int kWin = 64;                    // header window bytes staged in LDS
constexpr int kMaxBins = FCGPU_MAX_PORTS + 1 + FCGPU_NREASON_SLOTS;

struct DevCfg {
    int32_t offset;
    uint32_t nports;
    uint32_t lb_magic;       // ceil(2^32 / nports): x % nports for x < 2^16 (fastmod)
    uint32_t hash_mode;
    uint32_t classify;
    int32_t hs_offset;
    int32_t hs_length;
    int32_t native_vlan;
    uint32_t vlan_tpid;       // tag protocol as the 16-bit little-endian load of its bytes
    uint32_t nbadsrc;
    uint32_t ngooddst;
    uint32_t nbad6;
    uint32_t badsrc[FCGPU_MAX_ADDRS];
    uint32_t gooddst[FCGPU_MAX_ADDRS];
    uint32_t bad6[FCGPU_MAX_ADDRS][4];
    uint32_t process_eh;
    uint32_t l4_mode;
    uint32_t l4_checksum;
    uint32_t rewrite;         // FCGPU_RW_*
    uint32_t ttl_multicast;
    const uint4 *prog;        // decision program (FCGPU_CLS_PROGRAM), 16 B per step, then tables
    uint32_t prog_n;          // steps (table-step fallback copies included)
    uint32_t prog_q;          // uint4 words of steps + tables
    uint32_t prog_tab;        // uint4 index where the int16 jump tables start
    uint32_t prog_kind;
    int32_t prog_all;         // >= 0: empty program, every packet -> this output
    const uint4 *crc_tab;     // FCGPU_CLS_LB_CRC: 2 x 256 u32 slicing tables (1 KB each)
    const uint8_t *lb_tab;    // FCGPU_CLS_LB_TABLE: bucket -> output ((lb_tab_n + 15) & ~15 bytes, zero-padded)
    uint32_t lb_tab_n;        // buckets (<= 65536: the folded hash is < 2^16)
    uint32_t lb_tab_magic;    // ceil(2^32 / lb_tab_n) for lb_port's fastmod
};

// Device step: x = (u16)offset | flags << 16, y = value, z = mask,
// w = (u16)yes | (u16)no << 16 (signed 16-bit jumps).
// Table step (flag kStepTable, built by fcgpu_set_program from a run of steps
// that all test the word at one offset): when the word is inside the packet,
// the run's outcome is tab[y + ((bswap(word) >> (z & 31)) & ((1 << (z >> 8)) - 1))]
// (an int16 jump), else the walk continues at step w, a copy of the original
// step, so short packets keep the step-by-step length-checked semantics.
constexpr int32_t kProgUnmatched = 0x7fff;
constexpr uint32_t kStepTable = 2u;       // in the flags (x >> 16)

// Flow table state (fcgpu_flow_configure). Slot = {saddr, daddr, ports, tag}
// with tag = proto | (flow id + 1) << 8; tag 0 = empty. Linear probing, never
// more than half full (max_flows <= slots / 2), no deletions between
// maintainer runs (an IMP run with timeouts rebuilds the table without the
// flows it expired, k_flow_rebuild).
struct FlowArgs {
    uint4 *slots;
    uint32_t mask;           // slots - 1
    uint32_t max_flows;
    uint32_t *claim;         // [slots] claiming miss packet + 1 (this batch)
    uint32_t *first;         // [slots] min packet index of the claiming flow
    // per packet of the batch, meaningful where its missmask bit is set
    uint4 *miss_key;         // [max_batch]
    uint32_t *miss_slot;     // [max_batch]
    uint32_t *miss_first;    // [max_batch]
    uint64_t *missmask;      // [words64] bit i: packet i missed (every wave writes its word)
    uint64_t *firstmask;     // [words64] bit i: packet i is a new flow's first packet
    uint32_t *wordpre;       // [words64] exclusive popcount prefix of firstmask
    uint32_t *state;         // kFs* words below
    uint32_t *host_hint;     // mapped host word: size class of the last batch's misses (kHint*)
    uint32_t *flowid;        // [n] output (may be null)
    uint32_t *missed;        // the word a wave with misses stamps with the epoch (state + kFsMissed)
    uint32_t epoch;          // this batch's number (never 0)
    // IMP managers (fcgpu_flow.hh, "IMP"): null stack = HMP (IDs 0, 1, 2, ...)
    uint32_t *stack;         // free IDs; [0, max_flows - state[kFsNext]) hold them, top last
    uint32_t *lastseen;      // [wstride] ms of the last batch with a packet of the flow (null: no timeout)
    uint32_t *wheel;         // [wmask + 1][wstride] timer-wheel buckets, IDs in scheduling order
    uint32_t *wheel_len;     // [wmask + 1]
    uint32_t wstride;        // the table's capacity (IDs 0 .. wstride - 1)
    uint32_t wmask;          // wheel buckets - 1
    uint32_t te;             // timeout in maintainer epochs
    uint32_t now;            // this batch's time (ms, fcgpu_flow_set_time)
    uint32_t ls_mode;        // lastseen stamps (kLs*): per run, per run if the stored time differs, per packet
};
constexpr uint32_t kFsNext = 0;   // HMP: next flow ID; IMP: IDs out of the stack (max_flows - stack size)
constexpr uint32_t kFsBase = 1;   // the ID base of the batch being finished (grid-wide finish)
constexpr uint32_t kFsMissed = 2; // epoch of the last batch with a miss (FlowArgs::missed, one batch per launch)
constexpr uint32_t kFsHint = 3;   // the hint last published
constexpr uint32_t kFsIndex = 4;  // IMP: timer-wheel index (maintainer runs so far)
constexpr uint32_t kFsWBase = 5;  // IMP: the new-flow bucket's length when the batch began (grid-wide finish)
constexpr uint32_t kFsQlen = 6;   // IMP: IDs the last maintainer run released (pushed back by the next)
// The maintainer runs of IMP with timeouts (fcgpu_flow.hh k_maint_*).
struct MaintArgs {
    uint32_t *qbsr;          // [wstride] IDs released by the last run, in release order
    uint32_t *dead;          // [wstride] run number that released the ID
    uint32_t *counts;        // [chunks][te + 1] per-chunk counts, then offsets
    uint16_t *rbuf;          // [wstride] each walk entry's destination
    uint32_t now, to_ms, ri_ms, eps, seq;
};
constexpr uint32_t kLsRun = 0, kLsCheck = 1, kLsPacket = 2;   // FlowArgs::ls_mode
constexpr uint32_t kFlowMiss = 0xfffffffdu;
constexpr uint32_t kSlotNone = 0xffffffffu;

// A batch's descriptor and annotation layouts (RxArgs::layout, RxJob::layout):
// kLayDesc32 -- FCGPU_SUBMIT_DESC32 descriptors, one uint32 per packet (offset
// / 8 in bits 0-15, length in bits 16-31) instead of {u32 off, u32 len};
// kLayAnno8 -- FCGPU_OUT_ANNO8 annotations, the 8-B fcgpu_anno8 instead of
// fcgpu_anno. Any other bit is refused by the host launch guard.
constexpr uint32_t kLayDesc32 = 1u;
constexpr uint32_t kLayAnno8 = 2u;
constexpr uint32_t kLayKnown = kLayDesc32 | kLayAnno8;

struct RxArgs {
    const uint8_t *arena;
    const uint2 *desc;
    uint32_t n;
    uint32_t ntiles;
    uint16_t *verdict;
    uint32_t *hash;
    fcgpu_anno *anno;
    uint32_t *tilecnt;     // [nports+1][ntiles] (kPartGlobal)
    uint32_t *perm;        // [n] tile-local partition (kPartTile)
    uint16_t *tile_count;  // [ntiles][nports+1] (kPartTile)
    uint8_t *tile_perm;    // [n] tile-local partition (kPartTile)
    unsigned long long *ctr;   // [FCGPU_CTR_SHARDS][FCGPU_NCOUNTERS]
    FlowArgs fl;               // FLOW instances only
    uint32_t *ip_rw;           // [n] rewritten IP header bytes 8..11 (cfg.rewrite)
    uint32_t layout;           // kLay* bits: how desc and anno are laid out
    // a count on the device (fcgpu_process_counted, one batch per launch):
    // packets i >= *n_dev - n_base are not processed (n is then the bound the
    // grid covers); null: all n are
    const uint32_t *n_dev;
    uint32_t n_base;
    DevCfg cfg;
};

__device__ __forceinline__ uint32_t bswap16(uint32_t x) { return ((x & 0xff) << 8) | ((x >> 8) & 0xff); }
__device__ __forceinline__ uint32_t rotl32(uint32_t v, uint32_t r) {
    // v_alignbit_b32 funnel shift; shift count is taken mod 32, so r = 0 -> v
    return __builtin_amdgcn_alignbit(v, v, (32u - r) & 31u);
}

// One lane's view of its frame: 64-B window in LDS (swizzled 16-B chunks),
// beyond that aligned global loads from the arena.
struct FrameView {
    const uint8_t *row;       // this lane's 64-B LDS row
    const uint8_t *gwin;      // arena address of window byte 0 (16-B aligned)
    uint32_t sw;              // chunk swizzle of this row
    uint32_t shift;           // frame byte b lives at window byte b + shift

    // aligned dword at window byte x (x % 4 == 0)
    __device__ __forceinline__ uint32_t wdw(uint32_t x) const {
        if (x < (uint32_t)kWin)
            return *reinterpret_cast<const uint32_t *>(row + ((((x >> 4) ^ sw) << 4) | (x & 15)));
        return *reinterpret_cast<const uint32_t *>(gwin + x);
    }
    // little-endian 32-bit value at frame byte b (any alignment)
    __device__ __forceinline__ uint32_t rd32(uint32_t b) const {
        const uint32_t x = b + shift;
        const uint32_t lo = wdw(x & ~3u), hi = wdw((x & ~3u) + 4);
        return __builtin_amdgcn_alignbyte(hi, lo, x & 3u);
    }
    // K consecutive little-endian dwords starting at frame byte b
    template <int K>
    __device__ __forceinline__ void run(uint32_t b, uint32_t (&out)[K]) const {
        const uint32_t x = b + shift, a = x & ~3u, r = x & 3u;
        uint32_t w[K + 1];
#pragma unroll
        for (int j = 0; j <= K; ++j) w[j] = wdw(a + 4 * j);
#pragma unroll
        for (int j = 0; j < K; ++j) out[j] = __builtin_amdgcn_alignbyte(w[j + 1], w[j], r);
    }
    __device__ __forceinline__ uint32_t rd8(uint32_t b) const {
        const uint32_t x = b + shift;
        return (wdw(x & ~3u) >> (8 * (x & 3u))) & 0xff;
    }
    // rd8 for a frame byte inside the window: one LDS read
    __device__ __forceinline__ uint32_t rd8_win(uint32_t b) const {
        const uint32_t x = b + shift, a = x & ~3u;
        const uint32_t w = *reinterpret_cast<const uint32_t *>(row + ((((a >> 4) ^ sw) << 4) | (a & 15)));
        return (w >> (8 * (x & 3u))) & 0xff;
    }
    // rd32 for a frame byte whose dword pair lies in the window (x + 8 <= kWin):
    // LDS reads only. (wdw's choice between the LDS row and the arena compiles
    // to flat loads, which go through the vector-memory path and wait on it.)
    __device__ __forceinline__ uint32_t rd32_win(uint32_t b) const {
        const uint32_t x = b + shift, a = x & ~3u;
        const uint32_t lo = *reinterpret_cast<const uint32_t *>(row + ((((a >> 4) ^ sw) << 4) | (a & 15)));
        const uint32_t a4 = a + 4;
        const uint32_t hi = *reinterpret_cast<const uint32_t *>(row + ((((a4 >> 4) ^ sw) << 4) | (a4 & 15)));
        return __builtin_amdgcn_alignbyte(hi, lo, x & 3u);
    }
};

// click_in_cksum(hdr, hlen) == 0  <=>  the end-around-carry sum of the header's
// 16-bit words folds to 0xffff (lib/in_cksum.c:20-51). Summing little-endian
// dwords and folding is the same one's-complement sum (RFC 1071 associativity).
__device__ __forceinline__ bool cksum_ok(const FrameView &f, uint32_t o, uint32_t hlen,
                                         const uint32_t (&h)[5]) {
    uint64_t s = (uint64_t)h[0] + h[1] + h[2] + h[3] + h[4];
    for (uint32_t j = 20; j < hlen; j += 4) s += f.rd32(o + j);
    s = (s & 0xffffffffu) + (s >> 32);
    s = (s & 0xffffffffu) + (s >> 32);
    uint32_t t = (uint32_t)s;
    t = (t & 0xffff) + (t >> 16);
    t = (t & 0xffff) + (t >> 16);
    return t == 0xffff;
}

// ((h >> 16) ^ (h & 0xffff)) % n (loadbalancer.hh:580-584). The folded value is
// < 2^16, so with m = ceil(2^32 / n): q = (x * m) >> 32 is exact (x * (m*n - 2^32)
// ceil error e = m*n - 2^32 < n, and x*e < 2^16 * 64 < 2^32 keeps the quotient
// exact; n = 1 is special-cased (m would not fit). Checked exhaustively in
// tests/test_abi.py::test_lb_fastmod_exhaustive).
__device__ __forceinline__ int lb_port(uint32_t h, uint32_t n, uint32_t m) {
    const uint32_t x = (h >> 16) ^ (h & 0xffff);
    const uint32_t q = __umulhi(x, m);
    return n == 1 ? 0 : (int)(x - q * n);
}

// LoadBalancer constant_hash_agg (loadbalancer.hh:585-589): the ring's entry
// at ((h >> 16) ^ (h & 0xffff)) % buckets (lb_port's fastmod is exact for any
// buckets <= 2^16: x * e < 2^16 * 2^16), from the workgroup's LDS copy when the
// table is there (dyn != nullptr), else from global memory
// (Two plain branches: a select of the two pointers became one flat load,
// whose pending count made every later store of the tile wait for all earlier
// ones -- 4 % on the headline kernel, which never takes this path. The wait
// after the global load keeps its count from reaching the join.)
__device__ __forceinline__ uint32_t lb_table_port(const DevCfg &c, const uint4 *dyn, uint32_t h) {
    const uint32_t b = (uint32_t)lb_port(h, c.lb_tab_n, c.lb_tab_magic);
    if (dyn) return reinterpret_cast<const uint8_t *>(dyn)[b];
    const uint32_t p = c.lb_tab[b];
    __builtin_amdgcn_s_waitcnt(0x0F70);      // vmcnt(0), expcnt / lgkmcnt left alone
    return p;
}

// rte_hash_crc_4byte(data, crc) (DPDK rte_hash_crc.h: _mm_crc32_u32(crc, data)):
// CRC32-C, reflected polynomial 0x82F63B78, no inversion -- a reflected CRC
// takes the 32-bit word at once (xor) and shifts it through bit by bit.
__device__ __forceinline__ uint32_t crc32c_u32(uint32_t data, uint32_t crc) {
    crc ^= data;
#pragma unroll
    for (int k = 0; k < 32; ++k) crc = (crc >> 1) ^ (0x82F63B78u & (0u - (crc & 1u)));
    return crc;
}
// The same through byte-sliced tables: the 32 shifts are linear over GF(2),
// and 16 of them take y to (y >> 16) ^ G(y & 0xffff), with G(v) = U0[v & 0xff]
// ^ U1[v >> 8] and U_k[b] = 16 shift steps of b << 8k -- so a word is two
// rounds of two LDS reads. The tables (2 KB) are built on the host
// (fcgpu_configure) and copied to LDS by the workgroups of an LB_CRC launch:
// 2 KB keeps 8 workgroups per CU, where four 32-step tables (4 KB) kept 7.
__device__ __forceinline__ uint32_t crc32c_u32_tab(const uint32_t *t, uint32_t data, uint32_t crc) {
    uint32_t y = crc ^ data;
    y = (y >> 16) ^ t[y & 0xff] ^ t[256 + ((y >> 8) & 0xff)];
    y = (y >> 16) ^ t[y & 0xff] ^ t[256 + ((y >> 8) & 0xff)];
    return y;
}
// ipv4_hash_crc(IPFlow5ID, 0) (include/click/dpdk_glue.hh:13-27): proto, saddr,
// daddr, then the ports word; a non-first fragment's IPFlow5ID has zero
// addresses and (here) zero ports (lib/ipflowid.cc:34-38)
__device__ __forceinline__ uint32_t flow5_crc(const uint4 *dyn, uint32_t proto, uint32_t sa, uint32_t da,
                                              uint32_t ports) {
    if (dyn) {
        const uint32_t *t = reinterpret_cast<const uint32_t *>(dyn);
        return crc32c_u32_tab(t, ports, crc32c_u32_tab(t, da, crc32c_u32_tab(t, sa, crc32c_u32_tab(t, proto, 0u))));
    }
    return crc32c_u32(ports, crc32c_u32(da, crc32c_u32(sa, crc32c_u32(proto, 0u))));
}

// HashSwitch::process / LoadBalancer::hash_ip byte-sum (hashswitch.cc:50-66,
// loadbalancer.hh:227-243)
__device__ __forceinline__ int bytesum_port(const FrameView &f, uint32_t len, int o, int l, uint32_t n) {
    if ((int)len < o + l) return 0;
    int d = 0;
    for (int i = 0; i < l; ++i) d += (int)f.rd8((uint32_t)(o + i));
    if (n == 2 || n == 4 || n == 8) return (d ^ (d >> 4)) & (int)(n - 1);
    return d % (int)n;
}

// The same byte sum over frame bytes [o, o + l) inside the lane's LDS window
// (o + l + shift <= kWin): aligned window dwords, bytes outside the range
// masked, four bytes summed per v_sad_u8; d < 2^16, so lb_port's fastmod
// (m = ceil(2^32 / n)) takes d % n exactly.
__device__ __forceinline__ uint32_t win_bytesum_port(const FrameView &f, uint32_t len, uint32_t o, uint32_t l,
                                                     uint32_t n, uint32_t m) {
    if (len < o + l) return 0u;
    const uint32_t x0 = o + f.shift, x1 = x0 + l;
    uint32_t d = 0;
    for (uint32_t a = x0 & ~3u; a < x1; a += 4) {
        const uint32_t w = *reinterpret_cast<const uint32_t *>(f.row + ((((a >> 4) ^ f.sw) << 4) | (a & 15)));
        uint32_t k = 0xffffffffu;                          // bytes of [x0, x1) in this dword
        if (a < x0) k &= 0xffffffffu << (8 * (x0 - a));
        if (a + 4 > x1) k &= 0xffffffffu >> (8 * (a + 4 - x1));
        d = __builtin_amdgcn_sad_u8(w & k, 0u, d);
    }
    if (n == 2 || n == 4 || n == 8) return (d ^ (d >> 4)) & (n - 1);
    return n == 1 ? 0u : d - __umulhi(d, m) * n;
}

// A decision program over one valid packet (IPFilter::match, ipfilter.hh:393-481
// with length_checked_match, ipfilter.cc:1415-1474; Classifier: Program::match,
// classification.hh:372-392 / classification.cc:1146-1176). Every step is
// length-checked, which is what the reference's unchecked fast loop computes
// whenever the packet is at least the program's safe length. Bytes before the
// frame start (MAC header - 2) read as zero.
__device__ __forceinline__ uint32_t prog_word(const FrameView &f, int b) {
    if (b >= 0) return f.rd32((uint32_t)b);
    if (b <= -4) return 0u;
    return f.rd32(0) << (8 * (-b));
}

template <class Steps>
__device__ __forceinline__ uint32_t run_program_on(const DevCfg &c, const FrameView &f, const fcgpu_anno &an,
                                                   const Steps &prog) {
    if (c.prog_all >= 0) return (uint32_t)c.prog_all;
    const bool ipf = c.prog_kind == FCGPU_PROG_IPFILTER;
    int plen;
    if (ipf) {
        const int nl = (int)an.length - (int)an.nh, nhl = (int)an.th - (int)an.nh;
        plen = nl > nhl ? nl + 512 - nhl : nl + 256;
    } else {
        plen = (int)an.length;
    }
    int pos = 0;
    // consecutive steps mostly test the same word (a rule's fields, a range
    // split into mask tests): keep the last one instead of re-reading it
    int lastb = INT32_MIN;
    uint32_t lastw = 0;
    const uint16_t *tab = reinterpret_cast<const uint16_t *>(prog + c.prog_tab);
    for (uint32_t it = 0; it <= c.prog_n; ++it) {
        const uint4 st = prog[pos];
        const int off = (int16_t)(st.x & 0xffff);
        const uint32_t m = st.z;
        const bool table = (st.x >> 16) & kStepTable;
        bool avail = off + 4 <= plen;
        if (table && !avail) {            // short word: the original steps decide
            pos = (int)st.w;
            continue;
        }
        if (!avail && off < plen) {
            const int a = plen - off;
            avail = !((m >> 24) || (((m >> 16) & 0xff) && a <= 2) || (((m >> 8) & 0xff) && a == 1));
        }
        int j;
        if (avail) {
            const int b = !ipf ? off : off >= 512 ? (int)an.th + off - 512 : off >= 256 ? (int)an.nh + off - 256 : off - 2;
            if (b != lastb) {
                lastw = prog_word(f, b);
                lastb = b;
            }
            if (table) {
                const uint32_t idx = (__builtin_bswap32(lastw) >> (m & 31)) & ((1u << (m >> 8)) - 1u);
                j = (int16_t)tab[st.y + idx];
            } else {
                const uint32_t data = lastw & m;
                j = data == st.y ? (int16_t)(st.w & 0xffff) : (int16_t)(st.w >> 16);
            }
        } else {
            j = ((st.x >> 16) & FCGPU_STEP_SHORT_YES) ? (int16_t)(st.w & 0xffff) : (int16_t)(st.w >> 16);
        }
        if (j <= 0) return (uint32_t)(-j);
        pos = j;
    }
    return (uint32_t)kProgUnmatched;   // malformed (cyclic) program
}

// Steps come from the workgroup's LDS copy when the program fits (sprog !=
// nullptr, block-uniform), else from global memory.
// Steps + tables cached in LDS: <= 2.5 KiB keeps 8 workgroups (17.6 KB of
// header windows and counts each) within a CU's 160 KB.
constexpr uint32_t kProgLdsQ = 160;
__host__ __device__ inline bool prog_in_lds(const DevCfg &c) {
#ifdef FCGPU_JIT_PROGRAM
    return false;                 // the program is code: no steps to cache
#else
    return c.classify == FCGPU_CLS_PROGRAM && c.prog_all < 0 && c.prog_q <= kProgLdsQ;
#endif
}
// dynamic LDS of a k_rx launch: only program mode pays for the step cache,
// only LB_CRC for its 2-KB slicing tables, only LB_TABLE for its table (its
// buckets rounded up to 16 B) when it has at most 4096 buckets. Up to 2,944
// bytes keep 8 workgroups per CU (17.5 KB of windows and counts each); the
// default ring, 100 buckets per output, fits for up to 29 outputs
constexpr uint32_t kCrcTabQ = 128;          // 2 x 256 u32 = 128 uint4
constexpr uint32_t kTabLdsBytes = 4096;     // = kTile x 16 B: one uint4 per thread
__host__ __device__ inline bool crc_in_lds(const DevCfg &c) { return c.classify == FCGPU_CLS_LB_CRC && c.crc_tab; }
__host__ __device__ inline bool tab_in_lds(const DevCfg &c) {
    return c.classify == FCGPU_CLS_LB_TABLE && c.lb_tab && c.lb_tab_n <= kTabLdsBytes;
}
inline size_t prog_lds_bytes(const DevCfg &c) {
    return prog_in_lds(c) ? sizeof(uint4) * c.prog_q : crc_in_lds(c) ? sizeof(uint4) * kCrcTabQ
         : tab_in_lds(c) ? (c.lb_tab_n + 15u) & ~15u : 0;
}
#ifdef FCGPU_JIT_PROGRAM
// The installed program compiled to straight-line code (fcgpu_program_jit,
// prog_jit.hh jit_program_source): defined by the generated source after this header.
__device__ __forceinline__ uint32_t jit_program(const FrameView &f, const fcgpu_anno &an);
#endif
__device__ __forceinline__ uint32_t run_program(const DevCfg &c, const FrameView &f, const fcgpu_anno &an,
                                                const uint4 *sprog) {
#ifdef FCGPU_JIT_PROGRAM
    return jit_program(f, an);
#else
    if (sprog) return run_program_on(c, f, an, sprog);
    return run_program_on(c, f, an, c.prog);
#endif
}

struct PktResult {
    uint32_t reason;
    uint32_t port;
    uint32_t hash;
    fcgpu_anno an;
};

// CheckIPHeader::valid (elements/ip/checkipheader.cc:163-226); ip header at o.
template <bool CK>
__device__ __forceinline__ uint32_t check_ip4(const DevCfg &c, const FrameView &f, uint32_t len,
                                              uint32_t o, uint32_t (&h)[5], fcgpu_anno &an) {
    const uint32_t plen = len - o;
    if ((int)plen < 20) return FCGPU_R_MINISCULE;
    f.run<5>(o, h);
    an.ipver = 4;
    const uint32_t b0 = h[0] & 0xff;
    if ((b0 >> 4) != 4) return FCGPU_R_BAD_VERSION;
    const uint32_t hlen = (b0 & 15) << 2;
    if (hlen < 20) return FCGPU_R_BAD_HLEN;
    const uint32_t L = bswap16(h[0] >> 16);
    if (L > plen || L < hlen) return FCGPU_R_BAD_IP_LEN;
    if (CK && !cksum_ok(f, o, hlen, h)) return FCGPU_R_BAD_CKSUM;
    if (c.nbadsrc) {
        bool bad = false, good = false;
        for (uint32_t j = 0; j < c.nbadsrc; ++j) bad |= (c.badsrc[j] == h[3]);
        for (uint32_t j = 0; j < c.ngooddst; ++j) good |= (c.gooddst[j] == h[4]);
        if (bad && !good) return FCGPU_R_BAD_SADDR;
    }
    an.nh = (uint16_t)o;
    an.th = (uint16_t)(o + hlen);
    an.length = (uint16_t)(plen > L ? len - (plen - L) : len);
    an.dst_ip = h[4];
    return FCGPU_R_OK;
}

// CheckIP6Header::simple_action (elements/ip6/checkip6header.cc:105-168)
__device__ __forceinline__ uint32_t check_ip6(const DevCfg &c, const FrameView &f, uint32_t len,
                                              uint32_t o, fcgpu_anno &an) {
    const uint32_t plen = len - o;
    an.ipver = 6;
    if ((int)plen < 40) return FCGPU_R_BAD_IP6;
    uint32_t h[2];
    f.run<2>(o, h);
    if (((h[0] & 0xff) >> 4) != 6) return FCGPU_R_BAD_IP6;
    const uint32_t pl6 = bswap16(h[1] & 0xffff);
    if (pl6 > plen - 40) return FCGPU_R_BAD_IP6;
    if (c.nbad6) {
        uint32_t s[4];
        f.run<4>(o + 8, s);
        for (uint32_t j = 0; j < c.nbad6; ++j)
            if (s[0] == c.bad6[j][0] && s[1] == c.bad6[j][1] && s[2] == c.bad6[j][2] &&
                s[3] == c.bad6[j][3])
                return FCGPU_R_BAD_IP6;
    }
    uint32_t nxt = (h[1] >> 16) & 0xff, tot = 40;
    if (c.process_eh) {
        // ip6_follow_eh (include/click/ip6address.hh:417-448) from the first
        // extension header to the end of the (untrimmed) packet: the last
        // header visited gives IP6_NXT and the transport header offset
        uint32_t eh = 40, t = nxt;
        while (eh < plen) {
            nxt = t;
            tot = eh;
            const uint32_t w = f.rd32(o + eh);          // eh->nxt, eh->len
            const uint32_t en = w & 0xff, el = (w >> 8) & 0xff;
            if (t == 0 || t == 43) eh += el * 8 + 8;            // hop-by-hop, routing
            else if (t == 51) eh += ((el + 2) * 4 + 7) & ~7u;   // AH: round_up((len+2)*4, 8)
            else if (t == 44) eh += 8;                          // fragment
            else break;                                         // no next header / upper layer
            t = en;
        }
    }
    an.nh = (uint16_t)o;
    an.th = (uint16_t)(o + tot);
    an.ip6_nxt = (uint8_t)nxt;
    an.length = (uint16_t)(pl6 < plen - tot ? len - (plen - tot - pl6) : len);
    return FCGPU_R_OK;
}

template <int CM, bool CK, bool PROG>
__device__ __forceinline__ void process_packet(const DevCfg &c, const FrameView &f, uint32_t len,
                                               PktResult &r, const uint4 *sprog) {
    fcgpu_anno &an = r.an;
    uint32_t o = (uint32_t)c.offset;
    uint32_t h[5] = {0, 0, 0, 0, 0};
    bool v6 = false;
    r.hash = 0;
    if (CM == FCGPU_CHECK_AUTO) {
        // StripEtherVLANHeader::simple_action (stripethervlanheader.cc:48-61)
        const uint32_t e = f.rd32(o + 12);        // bytes 12..15: type, tci
        if ((e & 0xffff) == c.vlan_tpid) {        // be16 == 0x8100 (or VLANDecap ETHERTYPE)
            an.vlan_tci = (uint16_t)(e >> 16);    // raw network-order tci
            o += 18;
        } else if (c.native_vlan >= 0) {
            an.vlan_tci = (uint16_t)bswap16((uint32_t)c.native_vlan);
            o += 14;
        } else {
            r.reason = FCGPU_R_VLAN_REJECT;
            r.port = c.nports;
            return;
        }
        an.nh = (uint16_t)o;                       // the pull() StripEtherVLANHeader did
        v6 = ((int)(len - o) >= 1) && ((f.rd8(o) >> 4) == 6);
        r.reason = v6 ? check_ip6(c, f, len, o, an) : check_ip4<CK>(c, f, len, o, h, an);
    } else if (CM == FCGPU_MARK_IP6) {
        // MarkIP6Header::simple_action (markip6header.cc:43-48): set_ip6_header(o, 40)
        an.nh = (uint16_t)o;
        an.th = (uint16_t)(o + 40);
        an.length = (uint16_t)len;
        an.ipver = 6;
        v6 = true;
        r.reason = FCGPU_R_OK;
    } else if (CM == FCGPU_MARK_IP4) {
        // MarkIPHeader::simple_action (markipheader.cc:43-48)
        f.run<5>(o, h);
        an.nh = (uint16_t)o;
        an.th = (uint16_t)(o + ((h[0] & 15) << 2));
        an.length = (uint16_t)len;
        an.ipver = 4;
        r.reason = FCGPU_R_OK;
    } else {
        r.reason = check_ip4<CK>(c, f, len, o, h, an);
    }
    if (r.reason != FCGPU_R_OK) {
        r.port = c.nports;
        return;
    }
    uint32_t hv = 0;
    if (c.hash_mode != FCGPU_HASH_NONE) {
        const uint32_t pd = f.rd32(an.th);              // sport, dport (network order)
        const uint32_t s = bswap16(pd & 0xffff), d = bswap16(pd >> 16);
        if (v6) {
            // IP6FlowID::hashcode (ip6flowid.hh:220-230), IP6Address::hashcode
            const uint32_t sa = (f.rd32(an.nh + 16) << 1) + f.rd32(an.nh + 20);
            const uint32_t da = (f.rd32(an.nh + 32) << 1) + f.rd32(an.nh + 36);
            hv = rotl32(sa, s & 15) ^ rotl32(da, 31 - (d & 15)) ^ ((d << 16) | s);
        } else {
            // IPFlowID(p) (lib/ipflowid.cc:29-46): non-first fragments -> zero flow
            const bool first = (bswap16(h[1] >> 16) & 0x1fff) == 0;
            if (first) hv = rotl32(h[3], (s & 15) + 1) ^ rotl32(h[4], 31 - (d & 15)) ^ ((d << 16) | s);
            if (c.hash_mode == FCGPU_HASH_FLOW5ID) hv ^= (h[2] >> 8) & 0xff;
        }
    }
    r.hash = hv;
    switch (c.classify) {
    case FCGPU_CLS_LB_HASH: r.port = (uint32_t)lb_port(hv, c.nports, c.lb_magic); break;
    case FCGPU_CLS_LB_CRC: {
        const uint32_t w1 = f.rd32(an.nh + 4), w2 = f.rd32(an.nh + 8);
        const bool first = (bswap16(w1 >> 16) & 0x1fff) == 0;
        const uint32_t crc = flow5_crc(sprog, (w2 >> 8) & 0xff, first ? f.rd32(an.nh + 12) : 0u,
                                       first ? f.rd32(an.nh + 16) : 0u, first ? f.rd32(an.th) : 0u);
        r.port = (uint32_t)lb_port(crc, c.nports, c.lb_magic);
        break;
    }
    case FCGPU_CLS_LB_TABLE: r.port = lb_table_port(c, sprog, hv); break;
    case FCGPU_CLS_HASH_IP: r.port = (uint32_t)bytesum_port(f, an.length, 26, 8, c.nports); break;
    case FCGPU_CLS_HASHSWITCH:
        r.port = (uint32_t)bytesum_port(f, an.length, c.hs_offset, c.hs_length, c.nports);
        break;
    case FCGPU_CLS_PROGRAM: {
        if (!PROG) { r.port = 0; break; }    // not launched this way (launch_rx_any)
        const uint32_t out = run_program(c, f, an, sprog);
        if (out >= c.nports) {            // no output: CLASSIFY_EACH_PACKET kills it
            r.reason = FCGPU_R_NO_MATCH;
            r.port = c.nports;
        } else {
            r.port = out;
        }
        break;
    }
    default: r.port = 0;
    }
}

// Straight-line IPv4 fast path (CheckIPHeader -> AggregateHash -> classify) for
// the common shape: IP header + first L4 word inside the 64-B LDS window and
// no IP options. Reads 7 LDS dwords, no global loads, no data-dependent
// branches except the (wave-uniform) configuration. Returns false when this
// lane needs the general path (options, header beyond the window, hash modes
// or classifiers it does not cover); the caller then runs process_packet.
template <bool CK, bool PROG>
__device__ __forceinline__ bool ip4_fast(const DevCfg &c, const FrameView &f, uint32_t len, uint32_t o, PktResult &r,
                                         const uint4 *sprog) {
    const uint32_t x = f.shift + o, a = x & ~3u, sh = x & 3u;
    const bool inwin = a + 28 <= (uint32_t)kWin;
    const uint32_t ab = inwin ? a : 0u;   // keep the LDS reads in the row either way
    uint32_t w[7];
#pragma unroll
    for (int j = 0; j < 7; ++j)
        w[j] = *reinterpret_cast<const uint32_t *>(f.row + (((((ab + 4 * j) >> 4) ^ f.sw) << 4) | ((ab + 4 * j) & 15)));
    uint32_t h[6];
#pragma unroll
    for (int j = 0; j < 6; ++j) h[j] = __builtin_amdgcn_alignbyte(w[j + 1], w[j], sh);
    // CheckIPHeader::valid reason chain, computed as predicates (no divergent
    // branches); the first failing check wins, as in the reference
    const uint32_t plen = len - o;
    const uint32_t b0 = h[0] & 0xff, hlen = (b0 & 15) << 2, L = bswap16(h[0] >> 16);
    const bool tiny = (int)plen < 20, badv = (b0 >> 4) != 4, badhl = hlen < 20;
    const bool badlen = L > plen || L < hlen;
    bool ckbad = false;
    if (CK) {
        uint64_t sum = (uint64_t)h[0] + h[1] + h[2] + h[3] + h[4];
        uint32_t t = (uint32_t)sum + (uint32_t)(sum >> 32);      // fold the carries
        t = (t < (uint32_t)sum) ? t + 1 : t;                       // end-around carry
        t = (t & 0xffff) + (t >> 16);
        t = (t & 0xffff) + (t >> 16);
        ckbad = t != 0xffff;
    }
    bool srcbad = false;
    if (c.nbadsrc) {   // wave-uniform
        bool bad = false, good = false;
        for (uint32_t j = 0; j < c.nbadsrc; ++j) bad |= (c.badsrc[j] == h[3]);
        for (uint32_t j = 0; j < c.ngooddst; ++j) good |= (c.gooddst[j] == h[4]);
        srcbad = bad && !good;
    }
    const uint32_t early = tiny ? FCGPU_R_MINISCULE : badv ? FCGPU_R_BAD_VERSION
                         : badhl ? FCGPU_R_BAD_HLEN : badlen ? FCGPU_R_BAD_IP_LEN : FCGPU_R_OK;
    // decline: header not in the window, or IP options deciding checksum/ports
    if (!inwin || (early == FCGPU_R_OK && hlen != 20)) return false;
    const uint32_t reason = early != FCGPU_R_OK ? early
                          : ckbad ? FCGPU_R_BAD_CKSUM : srcbad ? FCGPU_R_BAD_SADDR : FCGPU_R_OK;
    const bool ok = reason == FCGPU_R_OK;
    uint32_t hv = 0;
    if (c.hash_mode != FCGPU_HASH_NONE) {   // wave-uniform
        const uint32_t sp = bswap16(h[5] & 0xffff), dp = bswap16(h[5] >> 16);
        const bool first = (bswap16(h[1] >> 16) & 0x1fff) == 0;
        hv = first ? rotl32(h[3], (sp & 15) + 1) ^ rotl32(h[4], 31 - (dp & 15)) ^ ((dp << 16) | sp) : 0u;
        if (c.hash_mode == FCGPU_HASH_FLOW5ID) hv ^= (h[2] >> 8) & 0xff;
    }
    uint32_t port = 0;
    if (c.classify == FCGPU_CLS_LB_HASH) {
        port = (uint32_t)lb_port(hv, c.nports, c.lb_magic);
    } else if (c.classify == FCGPU_CLS_LB_CRC) {       // wave-uniform
        const bool first = (bswap16(h[1] >> 16) & 0x1fff) == 0;
        const uint32_t crc = flow5_crc(sprog, (h[2] >> 8) & 0xff, first ? h[3] : 0u, first ? h[4] : 0u,
                                       first ? h[5] : 0u);
        port = (uint32_t)lb_port(crc, c.nports, c.lb_magic);
    } else if (c.classify == FCGPU_CLS_LB_TABLE) {
        port = lb_table_port(c, sprog, hv);
    } else if (c.classify == FCGPU_CLS_HASH_IP || c.classify == FCGPU_CLS_HASHSWITCH) {   // wave-uniform
        // LoadBalancer::hash_ip (loadbalancer.hh:227-243) = HashSwitch(26, 8),
        // HashSwitch::process (hashswitch.cc:50-66) over the trimmed packet
        const uint32_t bo = c.classify == FCGPU_CLS_HASH_IP ? 26u : (uint32_t)c.hs_offset;
        const uint32_t bl = c.classify == FCGPU_CLS_HASH_IP ? 8u : (uint32_t)c.hs_length;
        if (f.shift + bo + bl > (uint32_t)kWin) return false;   // bytes past the window: general path
        const uint32_t tl = plen > L ? len - (plen - L) : len;
        port = win_bytesum_port(f, tl, bo, bl, c.nports, c.lb_magic);
    } else if (c.classify != FCGPU_CLS_NONE && (!PROG || c.classify != FCGPU_CLS_PROGRAM)) {
        return false;
    }
    r.reason = reason;
    r.hash = ok ? hv : 0u;
    fcgpu_anno &an = r.an;
    an.ipver = early == FCGPU_R_MINISCULE ? 0 : 4;
    an.nh = (uint16_t)(ok ? o : 0u);
    an.th = (uint16_t)(ok ? o + 20 : 0u);
    an.length = (uint16_t)(ok ? (plen > L ? len - (plen - L) : len) : 0u);
    an.dst_ip = ok ? h[4] : 0u;
    if (PROG && ok) {                                  // FCGPU_CLS_PROGRAM
        port = run_program(c, f, an, sprog);
        if (port >= c.nports) r.reason = FCGPU_R_NO_MATCH;
    }
    r.port = ok && port < c.nports ? port : c.nports;
    return true;
}

// One LDS dword of the lane's window at frame byte b (any alignment); the
// caller guarantees shift + b + 8 <= kWin (two aligned dwords in the row).
__device__ __forceinline__ uint32_t win32(const FrameView &f, uint32_t b) {
    const uint32_t x = f.shift + b, a = x & ~3u;
    const uint32_t lo = *reinterpret_cast<const uint32_t *>(f.row + ((((a >> 4) ^ f.sw) << 4) | (a & 15)));
    const uint32_t hi = *reinterpret_cast<const uint32_t *>(f.row + (((((a + 4) >> 4) ^ f.sw) << 4) | ((a + 4) & 15)));
    return __builtin_amdgcn_alignbyte(hi, lo, x & 3u);
}

// StripEtherVLANHeader / VLANDecap at OFFSET, then the version dispatch of
// CHECK_AUTO, straight-line for frames whose headers sit in the window;
// rejected untagged frames (NATIVE_VLAN < 0) and PROCESS_EH take the general
// path. IPv4 and IPv6 lanes share one wave, so both checks run branch-free on
// one read of the window (12 dwords from the IP header) and each lane keeps
// its version's result: CheckIPHeader as ip4_fast, CheckIP6Header
// (checkip6header.cc:105-150) and IP6FlowID::hashcode (ip6flowid.hh:220-230)
// for the IPv6 header and first L4 word; same outputs as process_packet.
template <bool CK, bool PROG>
__device__ __forceinline__ bool auto_fast(const DevCfg &c, const FrameView &f, uint32_t len, PktResult &r,
                                          const uint4 *sprog) {
    const uint32_t o = (uint32_t)c.offset;
    // the tag word at o+12 and the version byte at o+18 as two aligned dwords each
    if (c.process_eh || f.shift + o + 26 > (uint32_t)kWin) return false;
    const uint32_t e = win32(f, o + 12);                     // type, tci
    const bool tagged = (e & 0xffff) == c.vlan_tpid;
    if (!tagged && c.native_vlan < 0) return false;
    const uint32_t x = o + (tagged ? 18u : 14u);
    const uint32_t xa = f.shift + x, a = xa & ~3u, sh = xa & 3u;
    // dwords past the row wrap into it (their lanes decline below)
    const uint32_t sw4 = f.sw << 4;
    uint32_t w[12];
#pragma unroll
    for (int j = 0; j < 12; ++j)
        w[j] = *reinterpret_cast<const uint32_t *>(f.row + (((a + 4 * j) & (uint32_t)(kWin - 1)) ^ sw4));
    uint32_t h[11];
#pragma unroll
    for (int j = 0; j < 11; ++j) h[j] = __builtin_amdgcn_alignbyte(w[j + 1], w[j], sh);
    const uint32_t plen = len - x;
    const bool v6 = (int)plen >= 1 && (h[0] & 0xf0) == 0x60;
    // classifiers the straight line covers (wave-uniform)
    const bool prog = PROG && c.classify == FCGPU_CLS_PROGRAM;
    // byte sums (hash_ip = HashSwitch(26, 8)) over frame bytes inside the window
    const bool bsum = c.classify == FCGPU_CLS_HASH_IP || c.classify == FCGPU_CLS_HASHSWITCH;
    const uint32_t bo = c.classify == FCGPU_CLS_HASH_IP ? 26u : (uint32_t)c.hs_offset;
    const uint32_t bl = c.classify == FCGPU_CLS_HASH_IP ? 8u : (uint32_t)c.hs_length;
    const bool bwin = !bsum || f.shift + bo + bl <= (uint32_t)kWin;
    const bool cls4 = c.classify == FCGPU_CLS_LB_HASH || c.classify == FCGPU_CLS_LB_CRC ||
                      c.classify == FCGPU_CLS_LB_TABLE || c.classify == FCGPU_CLS_NONE || prog || bsum;
    const bool cls6 = c.classify == FCGPU_CLS_LB_HASH || c.classify == FCGPU_CLS_LB_TABLE || prog || bsum;
    // CheckIPHeader::valid's reason chain as predicates (ip4_fast)
    const uint32_t b0 = h[0] & 0xff, hlen = (b0 & 15) << 2, L = bswap16(h[0] >> 16);
    const bool tiny = (int)plen < 20, badv = (b0 >> 4) != 4, badhl = hlen < 20;
    const bool badlen = L > plen || L < hlen;
    bool ckbad = false;
    if (CK) {
        uint64_t sum = (uint64_t)h[0] + h[1] + h[2] + h[3] + h[4];
        uint32_t t = (uint32_t)sum + (uint32_t)(sum >> 32);
        t = (t < (uint32_t)sum) ? t + 1 : t;
        t = (t & 0xffff) + (t >> 16);
        t = (t & 0xffff) + (t >> 16);
        ckbad = t != 0xffff;
    }
    bool srcbad = false;
    if (c.nbadsrc) {   // wave-uniform
        bool bad = false, good = false;
        for (uint32_t j = 0; j < c.nbadsrc; ++j) bad |= (c.badsrc[j] == h[3]);
        for (uint32_t j = 0; j < c.ngooddst; ++j) good |= (c.gooddst[j] == h[4]);
        srcbad = bad && !good;
    }
    const uint32_t early = tiny ? FCGPU_R_MINISCULE : badv ? FCGPU_R_BAD_VERSION
                         : badhl ? FCGPU_R_BAD_HLEN : badlen ? FCGPU_R_BAD_IP_LEN : FCGPU_R_OK;
    // CheckIP6Header: length, payload length, bad source addresses
    const uint32_t pl6 = bswap16(h[1] & 0xffff);
    bool bad6 = (int)plen < 40 || pl6 > plen - 40;
    for (uint32_t j = 0; j < c.nbad6; ++j)   // wave-uniform
        bad6 |= h[2] == c.bad6[j][0] && h[3] == c.bad6[j][1] && h[4] == c.bad6[j][2] && h[5] == c.bad6[j][3];
    // decline: header (+ first L4 word) not in the window, IP options, or a
    // classifier of the general path
    const bool take = bwin && (v6 ? (a + 48 <= (uint32_t)kWin && cls6)
                                  : (a + 28 <= (uint32_t)kWin && !(early == FCGPU_R_OK && hlen != 20) && cls4));
    if (!take) return false;
    const uint32_t reason = v6 ? (bad6 ? FCGPU_R_BAD_IP6 : FCGPU_R_OK)
                          : early != FCGPU_R_OK ? early
                          : ckbad ? FCGPU_R_BAD_CKSUM : srcbad ? FCGPU_R_BAD_SADDR : FCGPU_R_OK;
    const bool ok = reason == FCGPU_R_OK;
    uint32_t hv = 0;
    if (c.hash_mode != FCGPU_HASH_NONE) {   // wave-uniform
        const uint32_t pw = v6 ? h[10] : h[5];              // sport, dport
        const uint32_t sp = bswap16(pw & 0xffff), dp = bswap16(pw >> 16);
        // IPFlowID: non-first fragments hash as the zero flow; IP6Address::hashcode
        const bool first = (bswap16(h[1] >> 16) & 0x1fff) == 0;
        const uint32_t sa = v6 ? (h[4] << 1) + h[5] : h[3], da = v6 ? (h[8] << 1) + h[9] : h[4];
        const uint32_t rs = v6 ? (sp & 15) : (sp & 15) + 1;
        hv = rotl32(sa, rs) ^ rotl32(da, 31 - (dp & 15)) ^ ((dp << 16) | sp);
        hv = v6 || first ? hv : 0u;
        if (c.hash_mode == FCGPU_HASH_FLOW5ID && !v6) hv ^= (h[2] >> 8) & 0xff;
    }
    uint32_t port = 0;
    if (c.classify == FCGPU_CLS_LB_HASH) {
        port = (uint32_t)lb_port(hv, c.nports, c.lb_magic);
    } else if (c.classify == FCGPU_CLS_LB_CRC) {   // IPv4 lanes only (cls6)
        const bool first = (bswap16(h[1] >> 16) & 0x1fff) == 0;
        const uint32_t crc = flow5_crc(sprog, (h[2] >> 8) & 0xff, first ? h[3] : 0u, first ? h[4] : 0u,
                                       first ? h[5] : 0u);
        port = (uint32_t)lb_port(crc, c.nports, c.lb_magic);
    } else if (c.classify == FCGPU_CLS_LB_TABLE) {
        port = lb_table_port(c, sprog, hv);
    }
    const uint32_t cut = v6 ? (pl6 < plen - 40 ? plen - 40 - pl6 : 0u) : (plen > L ? plen - L : 0u);
    if (bsum) port = win_bytesum_port(f, len - cut, bo, bl, c.nports, c.lb_magic);
    r.reason = reason;
    r.hash = ok ? hv : 0u;
    fcgpu_anno &an = r.an;
    an.ipver = v6 ? 6 : early == FCGPU_R_MINISCULE ? 0 : 4;
    an.nh = (uint16_t)x;                                     // the pull() the strip did
    an.th = (uint16_t)(ok ? x + (v6 ? 40u : 20u) : 0u);
    an.length = (uint16_t)(ok ? len - cut : 0u);
    an.dst_ip = ok && !v6 ? h[4] : 0u;
    an.ip6_nxt = (uint8_t)(ok && v6 ? (h[1] >> 16) & 0xff : 0u);
    an.vlan_tci = tagged ? (uint16_t)(e >> 16) : (uint16_t)bswap16((uint32_t)c.native_vlan);
    if (prog && ok) {
        port = run_program(c, f, an, sprog);
        if (port >= c.nports) r.reason = FCGPU_R_NO_MATCH;
    }
    r.port = ok && port < c.nports ? port : c.nports;
    return true;
}

// ---- CheckUDPHeader / CheckTCPHeader ----------------------

// Lengths and protocol (checkudpheader.cc:96-111, checktcpheader.cc:96-111).
// Returns the verdict; l4len = segment length, want_sum = checksum to verify.
// WIN: every byte it reads is in the LDS window (l4_stage checks it per wave).
template <bool WIN>
__device__ __forceinline__ uint32_t l4_check(const DevCfg &c, const FrameView &f, const fcgpu_anno &an,
                                             uint32_t &l4len, bool &want_sum) {
    auto rd = [&](uint32_t b) { return WIN ? f.rd32_win(b) : f.rd32(b); };
    const uint32_t w0 = rd(an.nh), w2 = rd(an.nh + 8);
    const uint32_t hl = (w0 & 15) << 2, proto = (w2 >> 8) & 0xff;
    want_sum = false;
    if (c.l4_mode == FCGPU_L4_UDP) {
        if (proto != 17) return FCGPU_R_L4_PROTO;
        const uint32_t u = rd(an.th + 4);                     // uh_ulen, uh_sum
        const uint32_t len = bswap16(u & 0xffff);
        if (len < 8 || (uint32_t)an.length < len + hl + an.nh) return FCGPU_R_L4_LENGTH;
        l4len = len;
        want_sum = c.l4_checksum && (u >> 16) != 0;            // uh_sum == 0: not checked
    } else {
        if (proto != 6) return FCGPU_R_L4_PROTO;
        const uint32_t len = bswap16(w0 >> 16) - hl;          // unsigned, as the reference
        const uint32_t toff = ((rd(an.th + 12) >> 4) & 15) << 2;       // th_off
        if (toff < 20 || len < toff || (uint32_t)an.length < len + hl + an.nh) return FCGPU_R_L4_LENGTH;
        l4len = len;
        want_sum = c.l4_checksum != 0;
    }
    return FCGPU_R_OK;
}

// bytes [lo, hi) of the dword at byte offset off
__device__ __forceinline__ uint32_t dw_masked(uint32_t w, uint32_t off, uint32_t lo, uint32_t hi) {
    if (off >= lo && off + 4 <= hi) return w;
    if (off + 4 <= lo || off >= hi) return 0u;
    uint32_t m = 0xffffffffu;
    if (lo > off) m &= 0xffffffffu << (8 * (lo - off));
    if (hi < off + 4) m &= 0xffffffffu >> (8 * (off + 4 - hi));
    return w & m;
}

// One's-complement sums of the L4 segments of the lanes in `need`: 16 lanes
// per segment read 256 contiguous bytes per step (coalesced, each byte once),
// four segments per wave step. Each owner lane gets the 16-bit sum of its
// segment as ~click_in_cksum(seg, len) & 0xffff (lib/in_cksum.c:20-51): the sum
// of little-endian 16-bit words from the 16-B aligned base, byte-swapped when
// the segment starts at an odd address (RFC 1071 byte-order independence).
__device__ __forceinline__ uint32_t wave_l4_sum(const uint8_t *seg, uint32_t len, uint64_t need) {
    const uint32_t lane = threadIdx.x & 63, g = lane >> 4, j = lane & 15;
    const uint64_t sa = (uint64_t)seg;
    uint32_t mine = 0;
    uint64_t m = need;
    while (m) {
        uint32_t own[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            own[k] = m ? (uint32_t)__builtin_ctzll(m) : 64u;
            m = m ? m & (m - 1) : 0ull;
        }
        const uint32_t src = g == 0 ? own[0] : g == 1 ? own[1] : g == 2 ? own[2] : own[3];
        const int sl = (int)(src & 63);
        const uint32_t alo = __shfl((uint32_t)sa, sl), ahi = __shfl((uint32_t)(sa >> 32), sl);
        const uint32_t L = __shfl(len, sl);
        const uint64_t a = ((uint64_t)ahi << 32) | alo;
        uint64_t acc = 0;
        if (src < 64) {
            const uint32_t lo = (uint32_t)(a & 15), hi = lo + L;
            const uint8_t *base = reinterpret_cast<const uint8_t *>(a & ~15ull);
            for (uint32_t o = 16 * j; o < hi; o += 256) {
                const uint4 v = *reinterpret_cast<const uint4 *>(base + o);
                acc += (uint64_t)dw_masked(v.x, o, lo, hi) + dw_masked(v.y, o + 4, lo, hi) +
                       dw_masked(v.z, o + 8, lo, hi) + dw_masked(v.w, o + 12, lo, hi);
            }
        }
        uint32_t alo2 = (uint32_t)acc, ahi2 = (uint32_t)(acc >> 32);
#pragma unroll
        for (int o = 8; o >= 1; o >>= 1) {
            const uint32_t xl = __shfl_xor(alo2, o), xh = __shfl_xor(ahi2, o);
            const uint64_t t = ((uint64_t)ahi2 << 32 | alo2) + ((uint64_t)xh << 32 | xl);
            alo2 = (uint32_t)t;
            ahi2 = (uint32_t)(t >> 32);
        }
        uint32_t t = alo2 + ahi2;
        t += (t < alo2) ? 1u : 0u;
        t = (t & 0xffff) + (t >> 16);
        t = (t & 0xffff) + (t >> 16);
        if (a & 1) t = bswap16(t);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t v = __shfl(t, 16 * k);
            if (lane == own[k]) mine = v;
        }
    }
    return mine;
}

// The same 16-bit sum for a segment inside the lane's LDS window (frame bytes
// [b, b + len) with b + len + shift <= kWin): the window's aligned dwords,
// bytes outside the segment masked. Window byte 0 is 16-B aligned in the
// arena, so the segment's address parity is that of its window byte. Reading
// the window instead of the arena matters when the arena is host memory read
// over PCIe (zero-copy): the datagram of a small frame is already in LDS.
__device__ __forceinline__ uint32_t win_l4_sum(const FrameView &f, uint32_t b, uint32_t len) {
    const uint32_t x0 = b + f.shift, x1 = x0 + len;
    uint64_t acc = 0;
    for (uint32_t a = x0 & ~3u; a < x1; a += 4) {
        const uint32_t w = *reinterpret_cast<const uint32_t *>(f.row + ((((a >> 4) ^ f.sw) << 4) | (a & 15)));
        acc += dw_masked(w, a, x0, x1);
    }
    uint32_t t = (uint32_t)acc + (uint32_t)(acc >> 32);
    t += (t < (uint32_t)acc) ? 1u : 0u;
    t = (t & 0xffff) + (t >> 16);
    t = (t & 0xffff) + (t >> 16);
    return (x0 & 1) ? bswap16(t) : t;
}

// click_in_cksum_pseudohdr (include/clicknet/ip.h:156-163, lib/in_cksum.c:53-111):
// the final destination of an SSRR/LSRR option replaces ip_dst. True = bad.
template <bool WIN>
__device__ __forceinline__ bool l4_cksum_bad(const FrameView &f, const fcgpu_anno &an, uint32_t dsum,
                                             uint32_t len) {
    auto rd = [&](uint32_t b) { return WIN ? f.rd32_win(b) : f.rd32(b); };
    auto rd8 = [&](uint32_t b) { return WIN ? f.rd8_win(b) : f.rd8(b); };
    const uint32_t w0 = rd(an.nh), hl = (w0 & 15) << 2;
    const uint32_t proto = (rd(an.nh + 8) >> 8) & 0xff;
    const uint32_t src = rd(an.nh + 12);
    uint32_t dst = rd(an.nh + 16);
    if (hl != 20) {
        uint32_t opt = an.nh + 20;
        const uint32_t end = an.nh + hl;
        while (opt < end) {
            const uint32_t b = rd8(opt);
            if (b == 1) { ++opt; continue; }                // IPOPT_NOP
            if (b == 0) break;                              // IPOPT_EOL
            if (opt + 1 >= end) break;
            const uint32_t l = rd8(opt + 1);
            if (l < 2 || opt + l > end) break;
            if ((b == 137 || b == 131) && l >= 7) {         // IPOPT_SSRR, IPOPT_LSRR
                dst = rd(opt + l - 4);
                break;
            }
            opt += l;
        }
    }
    uint32_t c = dsum + (src & 0xffff) + (src >> 16) + (dst & 0xffff) + (dst >> 16) + bswap16(len) + (proto << 8);
    c = (c & 0xffff) + (c >> 16);
    return ((~(c + (c >> 16))) & 0xffffu) != 0;
}

// The L4 stage of k_rx for IPv4-accepted lanes (valid or no program match):
// length/protocol per lane, then the wave-cooperative checksum. WIN: every
// header byte it reads lies in the LDS window for every such lane of the wave.
template <bool WIN>
__device__ __forceinline__ void l4_stage_t(const DevCfg &c, const FrameView &f, const uint8_t *frame, bool live,
                                           PktResult &r) {
    uint32_t l4len = 0;
    bool want = false;
    if (live && (r.reason == FCGPU_R_OK || r.reason == FCGPU_R_NO_MATCH)) {
        const uint32_t lr = l4_check<WIN>(c, f, r.an, l4len, want);
        if (lr != FCGPU_R_OK) {
            r.reason = lr;
            r.port = c.nports;
            r.hash = 0;
        }
    }
    // segments inside the LDS window are summed there, the rest by the wave
    const bool inwin = want && r.an.th + l4len + f.shift <= (uint32_t)kWin;
    const uint64_t need = __ballot(want && !inwin);
    if (need || __ballot(inwin)) {
        uint32_t dsum = need ? wave_l4_sum(frame + r.an.th, l4len, need) : 0u;
        if (inwin) dsum = win_l4_sum(f, r.an.th, l4len);
        if (want && l4_cksum_bad<WIN>(f, r.an, dsum, l4len)) {
            r.reason = FCGPU_R_L4_CKSUM;
            r.port = c.nports;
            r.hash = 0;
        }
    }
}
// The header reads from the LDS window when, for every lane of the wave that
// reaches them, the IP header and the first 20 bytes of the L4 header are
// there (the general reads compile to flat loads, which wait on the
// vector-memory path): IPv4 puts th right after the options, so th + 20
// bounds every read of l4_check and l4_cksum_bad.
__device__ __forceinline__ void l4_stage(const DevCfg &c, const FrameView &f, const uint8_t *frame, bool live,
                                         PktResult &r) {
    const bool elig = live && (r.reason == FCGPU_R_OK || r.reason == FCGPU_R_NO_MATCH);
    const bool inw = (uint32_t)r.an.th + f.shift + 20u <= (uint32_t)kWin;
    if (!__ballot(elig && !inw)) l4_stage_t<true>(c, f, frame, live, r);
    else l4_stage_t<false>(c, f, frame, live, r);
}

// Header windows are read once per launch: non-temporal (cpol nt = 2) keeps
// them from evicting the outputs and descriptors from L2/MALL -- 5 % shorter
// k_rx than the default policy (profiles/r01_kernel_experiments).
constexpr int kWinCpol = 2;
__device__ __forceinline__ void glds16(const uint8_t *src, uint8_t *lds) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                     (__attribute__((address_space(3))) void *)lds, 16, 0, kWinCpol);
}

// Packet i's (offset, length) descriptor, read in the batch's layout
// (kLayDesc32: one uint32 per packet; the layout is uniform over a batch).
__device__ __forceinline__ uint2 load_desc(const uint2 *desc, uint32_t i, uint32_t layout) {
    if (layout & kLayDesc32) {
        const uint32_t w = reinterpret_cast<const uint32_t *>(desc)[i];
        return make_uint2((w & 0xffffu) << 3, w >> 16);
    }
    return desc[i];
}
// The per-packet outputs (verdict, hash, tile permutation, flow ID) are
// stored non-temporally: nothing in the launch reads them again, and under
// the default policy they shared L2 with the descriptors and the next
// workgroups' lines (same box, interleaved, profiles/r05_nt/: C2 13.3 ->
// 12.7 us per 1M batch; the descriptors read non-temporally too, or the
// tile counts, permutation and ip_rw words stored so, measured slower).
template <class T>
__device__ __forceinline__ void st_nt(T *p, T v) { __builtin_nontemporal_store(v, p); }

// Packet i's annotation: fcgpu_anno, or (kLayAnno8, IPv4 check modes) the
// 8-B fcgpu_anno8.
__device__ __forceinline__ void store_anno(fcgpu_anno *a, uint32_t i, const fcgpu_anno &an, uint32_t layout) {
    if (layout & kLayAnno8) {
        reinterpret_cast<uint2 *>(a)[i] =
            make_uint2(an.dst_ip, (uint32_t)an.length | ((uint32_t)(an.nh & 0xffu) << 16) |
                                      ((uint32_t)((an.th - an.nh) & 0xffu) << 24));
        return;
    }
    a[i] = an;
}

// Inclusive prefix sum over the 64 lanes of a wave by DPP (gfx9 row shifts
// within 16-lane rows, then row_bcast:15 / row_bcast:31 across rows): six
// VALU ops instead of six ds_bpermute round trips.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);   // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);   // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);   // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);   // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);   // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);   // row_bcast:31
    return x;
}

__host__ __device__ __forceinline__ uint32_t reason_slot(uint32_t r) { return r < 6 ? r : r - 1; }

// Lanes of this wave whose `key` equals mine, among the lanes in `live`
// (a match-any built from one ballot per key bit: the cost depends on the key
// width, not on how many distinct keys the wave holds).
__device__ __forceinline__ uint64_t match_any(uint32_t key, uint32_t nbits, uint64_t live) {
    uint64_t m = live;
    for (uint32_t k = 0; k < nbits; ++k) {
        const uint64_t bk = __ballot((key >> k) & 1u);
        m &= ((key >> k) & 1u) ? bk : ~bk;
    }
    return m;
}

// A workgroup barrier for LDS data only: this wave's LDS operations complete,
// then s_barrier. __syncthreads() is a workgroup release/acquire fence on all
// memory, which on gfx9 means s_waitcnt vmcnt(0) before the barrier: every
// wave of the tile would first wait for its outstanding global loads (the
// flow-table probe k_rx issues early to hide its latency) and for its
// verdict/hash stores to be acknowledged. Nothing after rx_tile's barrier
// reads global memory another wave of the workgroup wrote, so the LDS
// counters are all the barrier has to publish.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Partition modes of k_rx
constexpr int kPartNone = 0;     // counters only
constexpr int kPartGlobal = 1;   // + per-tile port histogram for k_scan/k_part (dense perm)
constexpr int kPartTile = 2;     // + stable partition of each 256-packet tile, in-kernel

// Source of a wave's header-window gather: 4 x (16 frames x 64 B); lane l of
// instruction k fetches 16-B chunk (l & 3) ^ swizzle of frame 16k + l/4.
__device__ __forceinline__ const uint8_t *win_src(const uint8_t *arena, uint32_t doff, uint32_t lane, int k) {
    const uint32_t p = k * 16 + (lane >> 2);
    const uint32_t poff = __shfl(doff, (int)p);
    const uint32_t c = (lane & 3) ^ ((p >> 2) & 3);
    return arena + (poff & ~15u) + c * 16;
}

// ---- flow table lookup (FlowIPManagerHMP::process, flowipmanagerhmp.cc:96-126) ----
__device__ __forceinline__ uint32_t flow_slot_hash(const uint4 &k) {
    // placement only (any mix works; IDs do not depend on it): murmur3 fmix32
    uint32_t h = k.x * 0x9E3779B1u ^ rotl32(k.y, 13) * 0x85EBCA77u ^ rotl32(k.z, 7) * 0xC2B2AE3Du ^ k.w;
    h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13; h *= 0xC2B2AE35u; h ^= h >> 16;
    return h;
}
__device__ __forceinline__ bool flow_key_eq(const uint4 &s, const uint4 &k) {
    return s.x == k.x && s.y == k.y && s.z == k.z && (s.w & 0xffu) == k.w;
}
// tag = proto | (id + 1) << 8; kTagFull marks a flow that arrived when the
// table was full (it stays FCGPU_FLOW_FULL: no timeouts, as in HMP)
constexpr uint32_t kTagFull = 0xffffffu;
__device__ __forceinline__ uint32_t flow_tag_id(uint32_t tag) {
    return (tag >> 8) == kTagFull ? FCGPU_FLOW_FULL : (tag >> 8) - 1u;
}
// IPFlow5ID(p) (lib/ipflowid.cc:29-46,91-94): saddr, daddr, the first L4 word
// (sport, dport), ip_p. A non-first fragment returns before assign(): its
// addresses stay 0 (IPAddress(), ipaddress.hh:21-22) and its ports unset
// (defined as 0), so it keys on ip_p alone.
__device__ __forceinline__ uint4 flow_key(const FrameView &f, const fcgpu_anno &an, bool live) {
    uint4 k;
    uint32_t w1, w2, sa, da, pt;
    // the header and the first L4 word inside the window for every lane of
    // the wave (the common case): LDS reads only; else the general reads
    const bool inwin = an.th + f.shift + 8 <= (uint32_t)kWin && an.nh + f.shift + 24 <= (uint32_t)kWin;
    if (!__ballot(live && !inwin)) {
        w1 = f.rd32_win(an.nh + 4);
        w2 = f.rd32_win(an.nh + 8);
        sa = f.rd32_win(an.nh + 12);
        da = f.rd32_win(an.nh + 16);
        pt = f.rd32_win(an.th);
    } else {
        w1 = f.rd32(an.nh + 4);                     // id, frag offset
        w2 = f.rd32(an.nh + 8);                     // ttl, proto, sum
        sa = f.rd32(an.nh + 12);
        da = f.rd32(an.nh + 16);
        pt = f.rd32(an.th);
    }
    const bool first = (bswap16(w1 >> 16) & 0x1fff) == 0;
    k.x = first ? sa : 0u;
    k.y = first ? da : 0u;
    k.z = first ? pt : 0u;
    k.w = (w2 >> 8) & 0xffu;
    return k;
}

// Packets past the checks get the ID of their flow, or a miss entry for the
// batch's new-flow pass (k_flow_finish). The first slot is loaded early
// (flow_issue, right after the checks) and examined late (flow_resolve, after
// the histogram and partition), so its latency hides behind that work.
struct FlowProbe {
    uint4 key;
    uint4 sl;        // first probed slot
    uint32_t pos;
    bool want;
};
__device__ __forceinline__ FlowProbe flow_issue(const FlowArgs &F, const FrameView &f, bool live,
                                                const PktResult &r) {
    FlowProbe q;
    q.want = live && r.an.ipver == 4 && (r.reason == FCGPU_R_OK || r.reason == FCGPU_R_NO_MATCH);
    q.key = make_uint4(0, 0, 0, 0);
    q.sl = make_uint4(0, 0, 0, 0);
    q.pos = 0;
    if (q.want) {
        q.key = flow_key(f, r.an, true);
        q.pos = flow_slot_hash(q.key) & F.mask;
        q.sl = F.slots[q.pos];
    }
    return q;
}
__device__ __forceinline__ void flow_resolve(const FlowArgs &F, FlowProbe &q, bool live, uint32_t i, bool word) {
    uint32_t id = FCGPU_FLOW_NONE;
    if (q.want) {
        id = kFlowMiss;
        for (uint32_t p = 0; p <= F.mask; ++p) {
            if (q.sl.w == 0) break;
            if (flow_key_eq(q.sl, q.key)) { id = flow_tag_id(q.sl.w); break; }
            q.pos = (q.pos + 1) & F.mask;
            q.sl = F.slots[q.pos];
        }
    }
    // IMP with timeouts: a flow with a packet in the batch is stamped with the
    // batch's time once per run of its packets (kLsRun), as the reference's
    // BatchBuilder stamps each run it pushes (update_lastseen at every run
    // boundary, virtualflowmanager.hh:236-239,304-313): the first packet of
    // a run of one flow in the wave stores (lane 0 always: a run crossing a
    // wave boundary is stamped twice with the same time). With kLsCheck the
    // stored time is read first and only a different one is written: one
    // store per flow and batch instead of per run (tables small enough to
    // stay in the caches). New flows are stamped by their first packet in
    // the new-flow pass. (kLsPacket, every packet stamping, is round 5's way,
    // kept for same-box A/B runs: FCGPU_LASTSEEN=packet.)
    if (F.lastseen) {
        const uint32_t prev = __shfl_up(id, 1);
        const bool head = (threadIdx.x & 63) == 0 || prev != id || F.ls_mode == kLsPacket;
        if (head && id < kTagFull && (F.ls_mode != kLsCheck || F.lastseen[id] != F.now)) F.lastseen[id] = F.now;
    }
    // The lookup only reads the table: a miss keeps its record (key, and the
    // empty slot its probe stopped at) at its packet index for the new-flow
    // pass, which looks it up again and places it in batch order
    // (fcgpu_flow.hh). The wave writes its 64-bit miss word (also a wave with
    // no live lane inside a counted launch's bound: `word`, so the new-flow
    // pass over the bound reads no stale word), and a wave with misses stamps
    // the batch's epoch -- plain stores: only the next launch
    // reads them. (An atomic on one miss counter per wave with misses
    // serialised at ~30 ns each at the memory: 10k misses cost 300 us.)
    const uint64_t mm = __ballot(id == kFlowMiss), lv = __ballot(live);
    if ((threadIdx.x & 63) == 0 && (lv || word)) {
        F.missmask[i >> 6] = mm;
        if (mm) *F.missed = F.epoch;
    }
    if (id == kFlowMiss) {
        F.miss_key[i] = q.key;
        F.miss_slot[i] = q.pos;
    }
    if (live && F.flowid) st_nt(F.flowid + i, id);
}

// ---- header rewrites after the classifier ----------------
// DecIPTTL::simple_action (elements/ip/decipttl.cc:52-78): ttl <= 1 leaves on
// output 1; else --ttl and the RFC 1624 update of the checksum,
//   sum = (~ntohs(ip_sum) & 0xFFFF) + 0xFEFF; ip_sum = ~htons(sum + (sum >> 16)).
// SetIPChecksum::simple_action (elements/ip/setipchecksum.cc:38-58): the full
// click_in_cksum of the header with ip_sum = 0; kills a packet whose header
// does not fit (only reachable in MARK mode). The packet's IP header bytes
// 8..11 after the rewrites go to ip_rw for every packet that leaves with
// R_OK (and, when changed, to the arena with FCGPU_RW_INPLACE).
template <bool WIN>
__device__ __forceinline__ void rw_stage_t(const DevCfg &c, const FrameView &f, uint8_t *frame, bool live,
                                           PktResult &r, uint32_t *ip_rw, uint32_t i) {
    auto rd = [&](uint32_t b) { return WIN ? f.rd32_win(b) : f.rd32(b); };
    uint32_t w = 0;
    bool changed = false;
    if (live && r.reason == FCGPU_R_OK && r.an.ipver == 4) {
        const uint32_t nh = r.an.nh;
        w = rd(nh + 8);                         // ttl, proto, sum (network order)
        if (c.rewrite & FCGPU_RW_DECTTL) {
            const bool mcast = (rd(nh + 16) & 0xf0u) == 0xe0u;   // IPAddress::is_multicast
            if (c.ttl_multicast || !mcast) {
                const uint32_t ttl = w & 0xffu;
                if (ttl <= 1) {
                    r.reason = FCGPU_R_TTL_EXPIRED;
                    r.port = c.nports;
                } else {
                    const uint32_t old = bswap16(w >> 16);
                    const uint32_t sum = (~old & 0xffffu) + 0xfeffu;
                    const uint32_t nsum = ~(sum + (sum >> 16)) & 0xffffu;
                    w = (w & 0xff00u) | (ttl - 1) | (bswap16(nsum) << 16);
                    changed = true;
                }
            }
        }
        if ((c.rewrite & FCGPU_RW_SETCKSUM) && r.reason == FCGPU_R_OK) {
            const uint32_t plen = (uint32_t)r.an.length - nh, hl = (rd(nh) & 15u) << 2;
            if (plen < 20 || hl < 20 || hl > plen) {
                r.reason = FCGPU_R_SETCKSUM_BAD;
                r.port = c.nports;
            } else {
                uint64_t s = (uint64_t)rd(nh) + rd(nh + 4) + (w & 0xffffu);
                for (uint32_t j = 12; j < hl; j += 4) s += rd(nh + j);
                s = (s & 0xffffffffu) + (s >> 32);
                s = (s & 0xffffffffu) + (s >> 32);
                uint32_t t = (uint32_t)s;
                t = (t & 0xffff) + (t >> 16);
                t = (t & 0xffff) + (t >> 16);
                w = (w & 0xffffu) | ((~t & 0xffffu) << 16);
                changed = true;
            }
        }
        changed = changed && r.reason == FCGPU_R_OK;   // a killed packet keeps nothing
        if (changed && (c.rewrite & FCGPU_RW_INPLACE)) {
            uint8_t *p = frame + nh + 8;
            p[0] = (uint8_t)w;
            p[2] = (uint8_t)(w >> 16);
            p[3] = (uint8_t)(w >> 24);
        }
    }
    // every packet that leaves with R_OK reports its bytes 8..11 as they leave
    // (rewritten or not), so a rewritten word of 0 (ttl 0, proto 0, sum 0 after
    // SetIPChecksum) is told apart from "no rewrite"; the rest report 0
    if (live && ip_rw) ip_rw[i] = r.reason == FCGPU_R_OK ? w : 0u;
}
// The header reads from the LDS window when every rewriting lane of the wave
// has its IP header there (the general reads compile to flat loads that wait
// on the vector-memory path).
__device__ __forceinline__ void rw_stage(const DevCfg &c, const FrameView &f, uint8_t *frame, bool live,
                                         PktResult &r, uint32_t *ip_rw, uint32_t i) {
    const bool elig = live && r.reason == FCGPU_R_OK && r.an.ipver == 4;
    bool inw = true;
    if (elig) {
        const uint32_t x = r.an.nh + f.shift;
        inw = x + 8 <= (uint32_t)kWin;
        if (inw) {
            const uint32_t hl = (f.rd32_win(r.an.nh) & 15u) << 2;
            inw = x + (hl > 20u ? hl : 20u) + 4 <= (uint32_t)kWin;
        }
    }
    if (!__ballot(elig && !inw)) rw_stage_t<true>(c, f, frame, live, r, ip_rw, i);
    else rw_stage_t<false>(c, f, frame, live, r, ip_rw, i);
}

// The batch a workgroup works on: RxArgs' per-batch pointers, or (fused
// launch) its job's. Plain scalars, so they stay in SGPRs.
struct RxView {
    const uint8_t *arena;
    const uint2 *desc;
    uint16_t *verdict;
    uint32_t *hash;
    fcgpu_anno *anno;
    uint32_t *perm;
    uint16_t *tile_count;
    uint8_t *tile_perm;
    uint32_t *tilecnt;       // kPartGlobal: [nports+1][ntiles]
    uint32_t *ip_rw;         // cfg.rewrite: the rewritten header bytes
    unsigned long long *ctr; // the batch's context's counter replicas
    uint32_t n, ntiles;
    uint32_t layout;         // kLay* bits
};
__device__ __forceinline__ RxView rx_view(const RxArgs &A) {
    return RxView{A.arena, A.desc, A.verdict, A.hash, A.anno, A.perm, A.tile_count, A.tile_perm, A.tilecnt,
                  A.ip_rw, A.ctr, A.n, A.ntiles, A.layout};
}

// One 256-packet tile once its header window is in LDS: fused
// [StripEtherVLANHeader ->] CheckIPHeader/CheckIP6Header -> AggregateHash ->
// classify; per-wave histogram by ballots; counters by sharded atomics;
// optionally the tile's stable per-output partition (CLASSIFY_EACH_PACKET on a
// 256-packet PacketBatch).
template <int CM, bool CK, int PART, bool PROG, bool L4, bool FAST, bool FLOW>
__device__ __forceinline__ void rx_tile(const RxArgs &A, const RxView &V, const FlowArgs &FL, uint32_t tile, uint2 d,
                                        const uint8_t *wl,
                                        uint32_t (*s_cnt)[kMaxBins], const uint4 *sprog) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t i = tile * kTile + threadIdx.x;
    const bool live = i < V.n;
    FrameView f;
    f.row = wl + lane * kWin;
    f.sw = (lane >> 2) & 3;
    f.shift = d.x & 15;
    f.gwin = V.arena + (d.x & ~15u);

    PktResult r;
    r.an = fcgpu_anno{};
    uint32_t bin = 0xffffffffu, rslot = 0xffffffffu;
    if (FAST && CM == FCGPU_CHECK_IP4) {
        bool done = !live;
        if (live) done = ip4_fast<CK, PROG>(A.cfg, f, d.y, (uint32_t)A.cfg.offset, r, sprog);
        if (__ballot(!done)) {
            if (!done) {
                r.an = fcgpu_anno{};
                process_packet<CM, CK, PROG>(A.cfg, f, d.y, r, sprog);
            }
        }
    } else if (FAST && CM == FCGPU_CHECK_AUTO) {
        bool done = !live;
        if (live) done = auto_fast<CK, PROG>(A.cfg, f, d.y, r, sprog);
        if (__ballot(!done)) {
            if (!done) {
                r.an = fcgpu_anno{};
                process_packet<CM, CK, PROG>(A.cfg, f, d.y, r, sprog);
            }
        }
    } else if (live) {
        process_packet<CM, CK, PROG>(A.cfg, f, d.y, r, sprog);
    }
    if (L4) l4_stage(A.cfg, f, V.arena + d.x, live, r);
    FlowProbe fq;
    if (FLOW) fq = flow_issue(FL, f, live, r);
    if (A.cfg.rewrite)   // launch-uniform
        rw_stage(A.cfg, f, const_cast<uint8_t *>(V.arena) + d.x, live, r, V.ip_rw, i);
    if (live) {
        if (V.verdict) st_nt(V.verdict + i, (uint16_t)(r.reason | (r.port << 8)));
        if (V.hash) st_nt(V.hash + i, r.hash);
        if (V.anno) store_anno(V.anno, i, r.an, V.layout);
        bin = r.port;
        if (r.reason != FCGPU_R_OK) rslot = reason_slot(r.reason);
    }

    // per-wave histogram: outputs 0..nports (nports = invalid list) by
    // match-any; each group's first lane writes its count, absent outputs 0
    const uint32_t nb = A.cfg.nports + 1;
    const uint32_t nbits = 32 - __clz(nb - 1 | 1);
    const uint64_t lt = (1ull << lane) - 1ull;
    const uint64_t mlive = __ballot(live);
    const uint64_t grp = match_any(bin, nbits, mlive);
    const uint32_t rank = (uint32_t)__popcll(grp & lt);
    for (uint32_t b = lane; b < nb + FCGPU_NREASON_SLOTS; b += 64) s_cnt[wave][b] = 0;
    __builtin_amdgcn_wave_barrier();
    if (live && rank == 0) s_cnt[wave][bin] = (uint32_t)__popcll(grp);
    const uint64_t mbad = __ballot(rslot != 0xffffffffu);
    if (mbad) {   // rare: per-reason counts
        const uint64_t g2 = match_any(rslot, 4, mbad);
        if (rslot != 0xffffffffu && __popcll(g2 & lt) == 0) s_cnt[wave][nb + rslot] = (uint32_t)__popcll(g2);
    }
    lds_barrier();
    const uint32_t nbt = nb + FCGPU_NREASON_SLOTS;
    const uint32_t t = threadIdx.x;
    uint32_t tot = 0;
    if (t < nbt) tot = s_cnt[0][t] + s_cnt[1][t] + s_cnt[2][t] + s_cnt[3][t];
    if (PART == kPartGlobal && t < nb) V.tilecnt[(size_t)t * V.ntiles + tile] = tot;
    if (PART == kPartTile) {
        if (t < nb) V.tile_count[(size_t)tile * nb + t] = (uint16_t)tot;
        // every wave scans the tile's output totals in registers (lane = output,
        // nb <= 65: output 64 rides in lane 63's inclusive sum) and adds the
        // counts of the waves before it, then each lane fetches its output's
        // start with one lane shuffle -- no second block barrier, no LDS base
        uint32_t v = 0, wpre = 0;
        if (lane < nb) {
#pragma unroll
            for (uint32_t w = 0; w < 4; ++w) {
                const uint32_t c = s_cnt[w][lane];
                v += c;
                wpre += w < wave ? c : 0u;
            }
        }
        const uint32_t incl = wave_incl_scan(v);
        const uint32_t start = incl - v + wpre;   // lane b: start of output b for this wave
        uint32_t mine = __shfl(start, (int)(bin & 63));
        if (nb > 64) {   // output 64 (nports == 64): base = sum of outputs 0..63
            uint32_t w64 = 0;
            for (uint32_t w = 0; w < wave; ++w) w64 += s_cnt[w][64];
            const uint32_t s64 = __shfl(incl, 63) + w64;
            if (bin == 64) mine = s64;
        }
        // each lane stores its own permutation entry (scattered within the
        // tile's 256-entry run; staging the run in LDS for coalesced stores
        // measured 1 % slower, profiles/r01_kernel_experiments)
        if (live) {
            const size_t pos = (size_t)tile * kTile + mine + rank;
            if (V.perm) V.perm[pos] = i;
            if (V.tile_perm) st_nt(V.tile_perm + pos, (uint8_t)threadIdx.x);
        }
    }
    if (FLOW) flow_resolve(FL, fq, live, i, A.n_dev != nullptr && (i & ~63u) < A.n);
    // counters: one atomic per non-zero bin per tile, sharded by tile. "count"
    // and "drops" are not kept here: both follow from these bins on read
    // (fcgpu_counters_derive), which saves an atomic per tile (-0.4 us / 1M).
    if (t < nbt) {
        unsigned long long *ctr = V.ctr + (size_t)(tile & (FCGPU_CTR_SHARDS - 1)) * FCGPU_NCOUNTERS;
        if (tot) {
            if (t < nb) atomicAdd(&ctr[FCGPU_CTR_PORT + t], (unsigned long long)tot);
            else atomicAdd(&ctr[FCGPU_CTR_REASON + (t - nb)], (unsigned long long)tot);
        }
    }
}


// The receive-path kernel: one 256-packet tile per workgroup (grid = ntiles).
// (Two tiles per workgroup with the second window prefetched into VGPRs
// while the first is processed measured 10-15 % slower: one resident round
// of workgroups instead of two loses the natural load/compute skew.)
//
// One launch may carry several batches (fcgpu_process_jobs on one stream,
// RxLaunch::njobs > 1): the grid is the batches' tiles end to end and each
// workgroup takes its batch's pointers from the launch arguments. A queue of
// batches then pays one launch ramp and tail instead of one per batch; the
// batches are independent (no in-place rewrite: jobs may share an arena;
// the flow table and the whole-batch partition keep per-batch scratch).
constexpr uint32_t kMaxFuse = 24;
constexpr uint32_t kMaxFuseJobs = kMaxFuse;   // ScanMulti / PartMulti
struct RxJob {
    const uint8_t *arena;
    const uint2 *desc;
    uint16_t *verdict;
    uint32_t *hash;
    fcgpu_anno *anno;
    uint32_t *perm;
    uint16_t *tile_count;
    uint8_t *tile_perm;
    uint32_t *flowid;
    uint32_t *tilecnt;       // kPartGlobal: the batch's per-tile counts (its own scratch)
    uint32_t *ip_rw;         // cfg.rewrite (not in place): the batch's rewritten header bytes
    unsigned long long *ctr; // the counter replicas of the batch's context (a launch may carry
                             // the batches of several contexts with one configuration)
    uint32_t n, tile0;       // packets; first workgroup of the batch in the grid
    uint32_t layout;         // kLay* bits of this batch (batches of one launch may differ)
};
struct RxLaunch {
    RxArgs A;                // njobs == 1: the batch; else the shared configuration
    uint32_t njobs;
    uint32_t job_tiles;      // every job's tile count when they are all equal, else 0
    // flow table, several batches: batch j's miss records at j x flow_stride
    // packets (j x flow_words mask words, missed + j) past A.fl's
    uint32_t flow_stride, flow_words;
    RxJob job[kMaxFuse];
};

template <int CM, bool CK, int PART, bool PROG, bool L4, bool FLOW = false,
          bool FAST = (CM == FCGPU_CHECK_IP4 || CM == FCGPU_CHECK_AUTO)>
__global__ __launch_bounds__(kTile, 8) void k_rx(RxLaunch L) {
    __shared__ __attribute__((aligned(16))) uint8_t s_win[4 * kWave * kWin];
    __shared__ uint32_t s_cnt[4][kMaxBins];
    extern __shared__ uint4 s_prog[];           // prog_lds_bytes(cfg) at launch: program steps, CRC or LB tables
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const RxArgs &A = L.A;
    RxView V = rx_view(A);
    FlowArgs FL = A.fl;
    uint32_t tile = blockIdx.x;
    if (L.njobs > 1) {   // workgroup-uniform
        // equal batches: a division; ragged ones: a walk over the jobs' first
        // tiles (kernel-argument loads the workgroup waits for)
        uint32_t j = 0, t = 0;
        if (L.job_tiles) {
            j = blockIdx.x / L.job_tiles;
            t = blockIdx.x - j * L.job_tiles;
        } else {
            for (uint32_t k = 1; k < L.njobs; ++k) j = blockIdx.x >= L.job[k].tile0 ? k : j;
            t = blockIdx.x - L.job[j].tile0;
        }
        const RxJob &J = L.job[j];
        V.arena = J.arena;
        V.desc = J.desc;
        V.verdict = J.verdict;
        V.hash = J.hash;
        V.anno = J.anno;
        V.perm = J.perm;
        V.tile_count = J.tile_count;
        V.tile_perm = J.tile_perm;
        V.tilecnt = J.tilecnt;
        V.ip_rw = J.ip_rw;
        V.ctr = J.ctr;
        V.n = J.n;
        V.ntiles = (J.n + kTile - 1) / kTile;
        V.layout = J.layout;
        tile = t;
        if (FLOW) {
            FL.miss_key += (size_t)j * L.flow_stride;
            FL.miss_slot += (size_t)j * L.flow_stride;
            FL.missmask += (size_t)j * L.flow_words;
            FL.missed += j;
            FL.flowid = J.flowid;
            FL.epoch += j;
        }
    }
    if (A.n_dev) {   // counted launch (one batch): the live packets are the first *n_dev - n_base
        const uint32_t c = *A.n_dev;
        V.n = c > A.n_base ? (c - A.n_base < V.n ? c - A.n_base : V.n) : 0u;
    }
    const uint32_t i = tile * kTile + threadIdx.x;
    uint2 d = make_uint2(0, 0);
    if (i < V.n) d = load_desc(V.desc, i, V.layout);
    uint8_t *wl = s_win + wave * (kWave * kWin);
#pragma unroll
    for (int k = 0; k < 4; ++k) glds16(win_src(V.arena, d.x, lane, k), wl + k * 1024);
    // decision program: the block's LDS copy when it fits (block-uniform)
    const bool prog_lds = PROG && prog_in_lds(A.cfg);
    const bool crc_lds = !PROG && crc_in_lds(A.cfg);          // block-uniform
    const bool tab_lds = !PROG && tab_in_lds(A.cfg);          // block-uniform
    if (prog_lds && threadIdx.x < A.cfg.prog_q) s_prog[threadIdx.x] = A.cfg.prog[threadIdx.x];
    if (crc_lds && threadIdx.x < kCrcTabQ) s_prog[threadIdx.x] = A.cfg.crc_tab[threadIdx.x];
    if (tab_lds && threadIdx.x * 16u < A.cfg.lb_tab_n)
        s_prog[threadIdx.x] = reinterpret_cast<const uint4 *>(A.cfg.lb_tab)[threadIdx.x];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // (every wave copying the whole table by LDS-DMA instead, with no block
    // barrier, measured the same: profiles/r05_lb/nobarrier_*)
    const bool dyn = prog_lds || crc_lds || tab_lds;
    if (dyn) __syncthreads();
    rx_tile<CM, CK, PART, PROG, L4, FAST, FLOW>(A, V, FL, tile, d, wl, s_cnt, dyn ? s_prog : nullptr);
}


}  // namespace fcgpu
