// fcgpu_exchange.hh -- device side of the flow re-shard across GPUs
// (SURVEY 8(f) #1 over 8(e); fcgpu_exchange_* in include/fastclick_gpu.h).
//
// FastClick keeps one flow table per core and lets the NIC's RSS hash send
// every packet of a flow to one core (FlowIPManagerHMP / VirtualFlowManagerIMP
// per thread, include/click/flow/virtualflowmanager.hh:249-330). When packets
// reach the GPUs unsharded, each rank's device pass classifies every packet to
// its owner rank (LB_MODE hash over `world` outputs, the FlowSwitch formula on
// the IPFlowID hash) with the whole-batch partition: perm lists the packets
// grouped by owner in input order, port_start[d] .. port_start[d+1] is owner
// d's run, and port_start[world] ends the packets that leave (invalid ones,
// output `world`, stay). These kernels turn that partition into the send
// buffer of one all-to-all:
//
//   k_xsum   per 1024-packet block of perm (4 consecutive packets a
//            thread): bytes its frames take (16-B slots), and the block's
//            partial sum at every segment boundary that falls inside it
//   k_xscan  one workgroup: exclusive scan of the block sums; each owner's
//            segment start = its block's scan value + that partial sum
//   k_xmeta  per packet of perm: its 16-B record {offset within its owner's
//            segment, length, source index, source rank}, staged in LDS and
//            written coalesced; the frame's arena offset into plan scratch
//   k_xpack  the frames into their segments, LPF lanes per frame moving 16 B
//            each (4 / 16 / 64 lanes by the mean frame size): each frame
//            starts 16-B aligned, the bytes of its slot past its length are
//            zero
//   k_xunpack (receiver) records -> descriptors into the received buffer
// Every per-packet load a thread needs is issued before the first barrier
// (perm, then the descriptors it names), so a block waits for memory once.
//
// Byte and index work only: HBM-bound (a frame's bytes read once and written
// once; perm/desc/records read twice), no MFMA.
#pragma once

#include <stdint.h>

#include "fastclick_gpu.h"

namespace fcgpu {

constexpr uint32_t kXThreads = 256;
constexpr uint32_t kXPer = 4;                     // packets per thread per plan block
constexpr uint32_t kXItems = kXThreads * kXPer;   // packets per plan block

// 4-B aligned vectors: the ABI's buffers are only dword-aligned
typedef uint32_t xu4 __attribute__((ext_vector_type(4), aligned(4)));
typedef uint32_t xu2 __attribute__((ext_vector_type(2), aligned(4)));
// Frame bytes read through global-address-space pointers: a pointer rebuilt
// from an integer (the dword-aligned base of a frame) is generic, its loads
// compile to flat loads, which also count on lgkmcnt -- then every LDS wait of
// the workgroup (the tile sort, the chunk search) waits for them and for the
// stores too: 199.5 -> see DESIGN section 6.
typedef const __attribute__((address_space(1))) uint32_t xg32;
typedef const __attribute__((address_space(1))) xu4 xg4;
__device__ __forceinline__ xg32 *xgbase(const uint8_t *p, uint32_t sh) {
    return (xg32 *)(p - sh);        // an address-space cast (no-op for global)
}

// A frame's slot in the send buffer: its length rounded up to 16 B, so every
// slot starts 16-B aligned and is written in whole aligned 16-B stores
// (4-B slots, round 4's format, left a segment's lines to be written by two
// frames' lanes with misaligned stores: k_xbuild 42.8 -> see DESIGN section 6).
constexpr uint32_t kXSlotAlign = 16;
__device__ __forceinline__ uint64_t xslot(uint32_t len) {
    return ((uint64_t)len + (kXSlotAlign - 1)) & ~(uint64_t)(kXSlotAlign - 1);
}

struct XPlan {
    const uint32_t *desc;
    const uint32_t *perm;
    const uint32_t *port_start;
    uint32_t n, world, rank, nblk;
    uint4 *meta;                    // fcgpu_xmeta [n] (dword-aligned)
    unsigned long long *bsum;       // [nblk + 1] block sums -> exclusive scan (+ total)
    unsigned long long *part;       // [world + 1] block-local sum before port_start[d]
    unsigned long long *base;       // [world + 1] segment starts in the send buffer
    unsigned long long *seg_bytes;  // [world]
    uint32_t *src;                  // [n] arena offset of perm[j]'s frame (for k_xpack)
};

__device__ __forceinline__ uint32_t xsend_count(const XPlan &P) {
    const uint32_t m = P.port_start[P.world];
    return m < P.n ? m : P.n;
}

// exclusive 64-bit scan over a 256-thread block, in thread order; *total = sum
__device__ __forceinline__ uint64_t xblock_excl(uint64_t v, unsigned long long *s_w, uint64_t *total) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint64_t incl = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t u = __shfl_up(incl, d);
        if (lane >= (uint32_t)d) incl += u;
    }
    __syncthreads();
    if (lane == 63) s_w[wave] = incl;
    __syncthreads();
    uint64_t pre = 0, t = 0;
    for (uint32_t w = 0; w < kXThreads / 64; ++w) {
        const uint64_t x = s_w[w];
        if (w < wave) pre += x;
        t += x;
    }
    *total = t;
    return pre + incl - v;
}

// this thread's kXPer consecutive packets of perm: indices, then their (offset,
// length) descriptors -- all loads in flight together
__device__ __forceinline__ void xload(const XPlan &P, uint32_t j0, uint32_t m, uint32_t (&pk)[kXPer],
                                       uint2 (&dl)[kXPer]) {
    static_assert(kXPer % 4 == 0, "perm is loaded 4 indices at a time");
    if (j0 + kXPer <= m) {
#pragma unroll
        for (uint32_t k = 0; k < kXPer; k += 4) {
            const xu4 a = *reinterpret_cast<const xu4 *>(P.perm + j0 + k);
            pk[k] = a.x, pk[k + 1] = a.y, pk[k + 2] = a.z, pk[k + 3] = a.w;
        }
    } else {
#pragma unroll
        for (uint32_t k = 0; k < kXPer; ++k) pk[k] = j0 + k < m ? P.perm[j0 + k] : 0u;
    }
#pragma unroll
    for (uint32_t k = 0; k < kXPer; ++k) {
        xu2 v = {0u, 0u};
        if (j0 + k < m) v = *reinterpret_cast<const xu2 *>(P.desc + 2 * (size_t)pk[k]);
        dl[k] = make_uint2(v.x, v.y);
    }
}

__global__ __launch_bounds__(kXThreads) void k_xsum(XPlan P) {
    __shared__ unsigned long long s_w[kXThreads / 64];
    __shared__ uint32_t s_ps[FCGPU_MAX_PORTS + 1];
    const uint32_t m = xsend_count(P);
    const uint32_t j0 = blockIdx.x * kXItems + kXPer * threadIdx.x;
    uint32_t pk[kXPer];
    uint2 dl[kXPer];
    xload(P, j0, m, pk, dl);
    for (uint32_t d = threadIdx.x; d <= P.world; d += kXThreads) {
        const uint32_t ps = P.port_start[d];
        s_ps[d] = ps < m ? ps : m;
    }
    uint64_t sl[kXPer], tsum = 0;
#pragma unroll
    for (uint32_t k = 0; k < kXPer; ++k) {
        sl[k] = xslot(dl[k].y);
        tsum += sl[k];
    }
    uint64_t tot;
    const uint64_t excl = xblock_excl(tsum, s_w, &tot);   // syncs: s_ps ready
    if (threadIdx.x == 0) P.bsum[blockIdx.x] = tot;
    for (uint32_t d = 0; d <= P.world; ++d) {
        const uint32_t ps = s_ps[d];
        if (ps >= j0 && ps < j0 + kXPer) {
            uint64_t v = excl;
#pragma unroll
            for (uint32_t k = 0; k < kXPer; ++k)
                if (j0 + k < ps) v += sl[k];
            P.part[d] = v;
        }
    }
}

// One workgroup of 1024 threads: bsum[0..nblk) -> exclusive scan, bsum[nblk]
// = total; base[d] = the scan value at packet port_start[d] (d = 0..world),
// seg_bytes[d] = base[d+1] - base[d].
__global__ __launch_bounds__(1024) void k_xscan(XPlan P) {
    __shared__ unsigned long long s_w[16];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t per = (P.nblk + 1023) / 1024;
    const uint32_t beg = threadIdx.x * per;
    uint64_t sum = 0;
    for (uint32_t k = 0; k < per; ++k)
        if (beg + k < P.nblk) sum += P.bsum[beg + k];
    uint64_t incl = sum;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t u = __shfl_up(incl, d);
        if (lane >= (uint32_t)d) incl += u;
    }
    if (lane == 63) s_w[wave] = incl;
    __syncthreads();
    uint64_t pre = 0, total = 0;
    for (uint32_t w = 0; w < 16; ++w) {
        const uint64_t x = s_w[w];
        if (w < wave) pre += x;
        total += x;
    }
    uint64_t run = pre + incl - sum;
    for (uint32_t k = 0; k < per; ++k)
        if (beg + k < P.nblk) {
            const uint64_t x = P.bsum[beg + k];
            P.bsum[beg + k] = run;
            run += x;
        }
    __syncthreads();
    const uint32_t m = xsend_count(P);
    auto base_at = [&](uint32_t d) -> uint64_t {
        uint32_t ps = P.port_start[d];
        ps = ps < m ? ps : m;
        const uint32_t blk = ps / kXItems;
        return blk >= P.nblk ? total : P.bsum[blk] + P.part[d];
    };
    const uint32_t d = threadIdx.x;
    if (d <= P.world) {
        const uint64_t b = base_at(d);
        P.base[d] = b;
        if (d < P.world) P.seg_bytes[d] = base_at(d + 1) - b;
    }
    if (threadIdx.x == 0) P.bsum[P.nblk] = total;
}

// the owner d of perm position j < m: the last d with port_start[d] <= j
__device__ __forceinline__ uint32_t xowner(const uint32_t *s_ps, uint32_t world, uint32_t j) {
    uint32_t lo = 0, hi = world;   // s_ps[lo] <= j < s_ps[hi] (s_ps[world] = m > j)
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (s_ps[mid] <= j) lo = mid;
        else hi = mid;
    }
    return lo;
}

__global__ __launch_bounds__(kXThreads) void k_xmeta(XPlan P) {
    __shared__ unsigned long long s_w[kXThreads / 64];
    __shared__ uint32_t s_ps[FCGPU_MAX_PORTS + 1];
    __shared__ unsigned long long s_base[FCGPU_MAX_PORTS + 1];
    __shared__ uint4 s_meta[kXItems];
    const uint32_t m = xsend_count(P);
    const uint32_t b0 = blockIdx.x * kXItems;
    const uint32_t j0 = b0 + kXPer * threadIdx.x;
    uint32_t pk[kXPer];
    uint2 dl[kXPer];
    xload(P, j0, m, pk, dl);
    for (uint32_t d = threadIdx.x; d <= P.world; d += kXThreads) {
        const uint32_t ps = P.port_start[d];
        s_ps[d] = ps < m ? ps : m;
        s_base[d] = P.base[d];
    }
    uint64_t tsum = 0;
#pragma unroll
    for (uint32_t k = 0; k < kXPer; ++k) tsum += xslot(dl[k].y);
    uint64_t tot;
    uint64_t at = P.bsum[blockIdx.x] + xblock_excl(tsum, s_w, &tot);   // syncs: s_ps, s_base ready
    if (j0 < m) {
        uint32_t d = xowner(s_ps, P.world, j0);
#pragma unroll
        for (uint32_t k = 0; k < kXPer; ++k) {
            const uint32_t j = j0 + k;
            if (j < m) {
                while (d + 1 < P.world && s_ps[d + 1] <= j) ++d;
                s_meta[kXPer * threadIdx.x + k] = make_uint4((uint32_t)(at - s_base[d]), dl[k].y, pk[k], P.rank);
                at += xslot(dl[k].y);
            }
        }
        if (j0 + kXPer <= m) {
#pragma unroll
            for (uint32_t k = 0; k < kXPer; k += 4)
                *reinterpret_cast<uint4 *>(P.src + j0 + k) = make_uint4(dl[k].x, dl[k + 1].x, dl[k + 2].x, dl[k + 3].x);
        } else {
#pragma unroll
            for (uint32_t k = 0; k < kXPer; ++k)
                if (j0 + k < m) P.src[j0 + k] = dl[k].x;
        }
    }
    __syncthreads();
    for (uint32_t q = threadIdx.x; q < kXItems && b0 + q < m; q += kXThreads) {
        const uint4 v = s_meta[q];
        *reinterpret_cast<xu4 *>(P.meta + b0 + q) = xu4{v.x, v.y, v.z, v.w};
    }
}

// One frame into its 16-B aligned slot (xslot) at dstp, lpf lanes (this one
// is q): 16 B per lane per step, four aligned dwords of the source and the
// next one funnel-shifted (v_alignbyte) into one aligned 16-B store (frames
// start anywhere in the arena; the ABI's 16 B of readable slack past a
// frame's end covers the fifth load). Slot bytes past the frame are zero;
// nothing is stored past the slot.
__device__ __forceinline__ void xcopy_frame(const uint8_t *src, uint32_t len, uint8_t *dstp, uint32_t q,
                                            uint32_t lpf) {
    const uint32_t sh = (uint32_t)(reinterpret_cast<uintptr_t>(src) & 3u);
    xg32 *al = xgbase(src, sh);
    uint32_t *out = reinterpret_cast<uint32_t *>(dstp);
    // four of the lane's chunks per round, their loads issued before any
    // store (a long frame's chunks then wait for memory together)
    constexpr uint32_t kU = 4;
    for (uint32_t w0 = 16 * q; w0 < len; w0 += 16 * lpf * kU) {
        xu4 a[kU];
        uint32_t e[kU];
#pragma unroll
        for (uint32_t k = 0; k < kU; ++k) {
            const uint32_t w = w0 + 16 * lpf * k;
            a[k] = xu4{0u, 0u, 0u, 0u};
            e[k] = 0u;
            if (w < len) {
                a[k] = *(xg4 *)(al + (w >> 2));
                // the fifth dword only when the frame reaches into it (so no
                // read goes further than 16 B past the frame's end)
                if (sh && w + 16 - sh < len) e[k] = al[(w >> 2) + 4];
            }
        }
#pragma unroll
        for (uint32_t k = 0; k < kU; ++k) {
            const uint32_t w = w0 + 16 * lpf * k;
            if (w >= len) break;
            uint32_t v0 = __builtin_amdgcn_alignbyte(a[k].y, a[k].x, sh);
            uint32_t v1 = __builtin_amdgcn_alignbyte(a[k].z, a[k].y, sh);
            uint32_t v2 = __builtin_amdgcn_alignbyte(a[k].w, a[k].z, sh);
            uint32_t v3 = __builtin_amdgcn_alignbyte(e[k], a[k].w, sh);
            const uint32_t rem = len - w;
            if (rem < 16) {
                // the slot's last 16 B: bytes past the frame zero
                auto cut = [rem](uint32_t v, uint32_t j) -> uint32_t {
                    if (rem <= 4 * j) return 0u;
                    const uint32_t keep = rem - 4 * j;
                    return keep >= 4 ? v : v & ((1u << (8 * keep)) - 1u);
                };
                v0 = cut(v0, 0), v1 = cut(v1, 1), v2 = cut(v2, 2), v3 = cut(v3, 3);
            }
            // the slot is 16-B aligned (xslot): one aligned 16-B store
            *reinterpret_cast<uint4 *>(out + (w >> 2)) = make_uint4(v0, v1, v2, v3);
        }
    }
}

struct XPack {
    const uint8_t *arena;
    const uint32_t *src;            // plan scratch: arena offset of each leaving frame
    const uint32_t *port_start;
    const uint4 *meta;
    const unsigned long long *seg_bytes;
    uint8_t *send;
    unsigned long long send_cap;
    uint32_t n, world;
};

// LPF lanes per frame (xcopy_frame), frames in perm order.
template <uint32_t LPF>
__global__ __launch_bounds__(kXThreads) void k_xpack(XPack X) {
    __shared__ uint32_t s_ps[FCGPU_MAX_PORTS + 1];
    __shared__ unsigned long long s_base[FCGPU_MAX_PORTS + 1];
    __shared__ unsigned long long s_big;     // owners whose segment is 4 GiB or more
    uint32_t m = X.port_start[X.world];
    m = m < X.n ? m : X.n;
    const uint32_t j = blockIdx.x * (kXThreads / LPF) + threadIdx.x / LPF;
    const uint32_t q = threadIdx.x % LPF;
    xu4 r = {0u, 0u, 0u, 0u};
    uint32_t so = 0;
    if (j < m) {
        r = *reinterpret_cast<const xu4 *>(X.meta + j);
        so = X.src[j];
    }
    if (threadIdx.x == 0) {
        unsigned long long b = 0, big = 0;
        for (uint32_t d = 0; d <= X.world; ++d) {
            const uint32_t ps = X.port_start[d];
            s_ps[d] = ps < m ? ps : m;
            s_base[d] = b;
            if (d < X.world) {
                b += X.seg_bytes[d];
                if (X.seg_bytes[d] > 0xffffffffull) big |= 1ull << d;
            }
        }
        s_big = big;
    }
    __syncthreads();
    if (j >= m) return;
    const uint32_t len = r.y;
    const uint64_t slot = xslot(len);
    const uint32_t own = xowner(s_ps, X.world, j);
    // the record's 32-bit offset within a segment past 4 GiB is truncated:
    // such a segment is not packed at all (the caller checks the plan's
    // segment sizes, fastclick_amd/device.py exchange_pack)
    if ((s_big >> own) & 1ull) return;
    const uint64_t dst = s_base[own] + r.x;
    if (dst + slot > X.send_cap) return;           // a send buffer smaller than the plan: nothing past it
    xcopy_frame(X.arena + so, len, X.send + dst, q, LPF);
}


// ---- one pass from the owner pass's verdicts (fcgpu_exchange_build) ---------
// The same records and send buffer as plan + pack, from a k_rx pass with
// LB_MODE hash over `world` outputs that wrote only its verdicts (no
// whole-batch partition, no owner-ordered gather of the descriptors): packet
// i leaves to owner d = verdict[i] >> 8 when d < world. Each 256-packet tile
// sorts its packets by owner in LDS (stable: a match-any rank per wave, the
// waves' counts in order), so tile t's packets of owner d follow the tile's
// earlier ones of d, and the tiles follow each other:
//
//   k_xbtile  per tile: packets and slot bytes of every owner
//             -> tcnt[d][t], tbyt[d][t]
//   k_xbscan  one workgroup per owner: exclusive scans of both over the
//             tiles (the tile's first record / byte within the owner's run),
//             seg_n[d], seg_bytes[d] (round 6 measured the scan folded into
//             k_xbtile's last blocks instead -- ticketed, two levels, no
//             third launch: 53.5 against 52.8 us for C4, 191.5 against 191.0
//             for C3, so the launch stays; profiles/r06_exchange/)
//   k_xbuild  per tile again: every leaving packet's record at its place in
//             owner order, then the tile's frames copied into their slots,
//             owner by owner (consecutive destinations), LPF lanes a frame
//
// Every per-packet load (verdict, descriptor) is coalesced in input order;
// the frames are read once and written once.
constexpr uint32_t kXTile = 256;

struct XBuild {
    const uint8_t *arena;
    const uint32_t *desc;           // [n][2]
    const uint16_t *verdict;        // [n] reason | port << 8
    uint32_t n, ntiles, world, rank;
    uint32_t *tcnt;                 // [world][ntiles] -> exclusive scan over t
    unsigned long long *tbyt;       // [world][ntiles] -> exclusive scan over t
    uint32_t *seg_n;                // [world]
    unsigned long long *seg_bytes;  // [world]
    uint4 *meta;                    // fcgpu_xmeta [m] (dword-aligned)
    uint8_t *send;
    unsigned long long send_cap;
    // fixed-capacity layout (fcgpu_exchange_build_fixed; 0: the counted one):
    // owner d's segment holds a header record and fix_recs records at meta
    // + d (fix_recs + 1), fix_bytes frame bytes at send + d fix_bytes; an
    // owner whose packets do not fit gets its header alone (overflow flag)
    uint32_t fix_recs;
    unsigned long long fix_bytes;
};

// inclusive scan of x over the 64 lanes of a wave
__device__ __forceinline__ uint32_t xwave_incl(uint32_t x) {
    const uint32_t lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t u = __shfl_up(x, d);
        if (lane >= (uint32_t)d) x += u;
    }
    return x;
}

// The tile's stable sort by owner (LDS). Outputs per lane: own (world =
// stays), pos (the lane's place among the tile's leaving packets in owner
// order; valid when own < world), intra (its slot's byte offset within the
// tile's run of its owner); in LDS: s_tcnt[d] / s_tstart[d] (the tile's
// packets of owner d and where they start), s_pre[k] (exclusive byte prefix
// in sorted order, s_pre[L] = the tile's leaving bytes). 256 threads.
struct XTileLds {
    uint32_t wc[4][FCGPU_MAX_PORTS + 1];     // per wave: packets of each owner
    uint32_t tcnt[FCGPU_MAX_PORTS + 1];
    uint32_t tstart[FCGPU_MAX_PORTS + 1];
    uint32_t slot[kXTile];
    uint32_t pre[kXTile + 1];
    uint32_t wsum[4];
};
__device__ __forceinline__ void xtile_sort(const XBuild &B, uint32_t t, XTileLds &L, uint32_t &own, uint32_t &len,
                                           uint32_t &src, uint32_t &pos, uint32_t &intra) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t i = t * kXTile + threadIdx.x;
    own = B.world;
    len = 0;
    src = 0;
    if (i < B.n) {
        const uint32_t d = (uint32_t)B.verdict[i] >> 8;
        const xu2 v = *reinterpret_cast<const xu2 *>(B.desc + 2 * (size_t)i);
        src = v.x;
        len = v.y;
        own = d < B.world ? d : B.world;
    }
    // rank among the wave's lanes with the same owner (match-any over its bits)
    const uint32_t nb = B.world + 1, nbits = 32 - __clz((nb - 1) | 1);
    uint64_t grp = ~0ull;
    for (uint32_t k = 0; k < nbits; ++k) {
        const uint64_t bk = __ballot((own >> k) & 1u);
        grp &= ((own >> k) & 1u) ? bk : ~bk;
    }
    const uint32_t rank = (uint32_t)__popcll(grp & ((1ull << lane) - 1ull));
    for (uint32_t b = lane; b < nb; b += 64) L.wc[wave][b] = 0;
    __builtin_amdgcn_wave_barrier();
    if (rank == 0) L.wc[wave][own] = (uint32_t)__popcll(grp);
    __syncthreads();
    // per owner: the tile's count; the owners' starts (only leaving owners, in order)
    if (wave == 0) {
        uint32_t c = 0;
        if (lane < B.world) c = L.wc[0][lane] + L.wc[1][lane] + L.wc[2][lane] + L.wc[3][lane];
        const uint32_t inc = xwave_incl(c);
        if (lane < B.world) {
            L.tcnt[lane] = c;
            L.tstart[lane] = inc - c;
        }
        if (lane == 63) L.tstart[B.world] = inc;           // = the tile's leaving packets
    }
    __syncthreads();
    pos = 0;
    if (own < B.world) {
        uint32_t wpre = 0;
        for (uint32_t w = 0; w < wave; ++w) wpre += L.wc[w][own];
        pos = L.tstart[own] + wpre + rank;
        L.slot[pos] = (uint32_t)xslot(len);
    }
    const uint32_t nl = L.tstart[B.world];
    __syncthreads();
    // exclusive byte prefix over the sorted slots
    const uint32_t v = threadIdx.x < nl ? L.slot[threadIdx.x] : 0u;
    const uint32_t inc = xwave_incl(v);
    if (lane == 63) L.wsum[wave] = inc;
    __syncthreads();
    uint32_t wp = 0;
    for (uint32_t w = 0; w < wave; ++w) wp += L.wsum[w];
    L.pre[threadIdx.x] = wp + inc - v;
    if (threadIdx.x == kXTile - 1) L.pre[kXTile] = wp + inc;
    __syncthreads();
    intra = own < B.world ? L.pre[pos] - L.pre[L.tstart[own]] : 0u;
}

// Per owner the tile's packets and slot bytes are sums, which the order the
// build sorts in does not change: LDS atomics and one barrier, no sort
// (the sort's five barriers per tile made this pass latency-bound). kXbTiles
// tiles per workgroup: four, their loads issued together, measured slower
// than one (6.4 against 5.3 us for 1M packets, profiles/r06_exchange/
// xbscan_regs: a quarter of the workgroups hides less latency).
constexpr uint32_t kXbTiles = 1;
__global__ __launch_bounds__(kXTile) void k_xbtile(XBuild B) {
    __shared__ uint32_t s_c[kXbTiles][FCGPU_MAX_PORTS], s_b[kXbTiles][FCGPU_MAX_PORTS];
    const uint32_t t0 = blockIdx.x * kXbTiles;
    for (uint32_t k = threadIdx.x; k < kXbTiles * FCGPU_MAX_PORTS; k += kXTile) {
        (&s_c[0][0])[k] = 0;
        (&s_b[0][0])[k] = 0;
    }
    uint32_t own[kXbTiles], slot[kXbTiles];
#pragma unroll
    for (uint32_t k = 0; k < kXbTiles; ++k) {
        const uint32_t i = (t0 + k) * kXTile + threadIdx.x;
        own[k] = B.world;
        slot[k] = 0;
        if (i < B.n) {
            const uint32_t d = (uint32_t)B.verdict[i] >> 8;
            if (d < B.world) {
                own[k] = d;
                slot[k] = (uint32_t)xslot(B.desc[2 * (size_t)i + 1]);
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < kXbTiles; ++k)
        if (own[k] < B.world) {
            atomicAdd(&s_c[k][own[k]], 1u);
            atomicAdd(&s_b[k][own[k]], slot[k]);
        }
    __syncthreads();
    for (uint32_t q = threadIdx.x; q < kXbTiles * B.world; q += kXTile) {
        const uint32_t k = q / B.world, d = q - k * B.world, t = t0 + k;
        if (t < B.ntiles) {
            B.tcnt[(size_t)d * B.ntiles + t] = s_c[k][d];
            B.tbyt[(size_t)d * B.ntiles + t] = s_b[k][d];
        }
    }
}

// owner d = blockIdx.x: exclusive scans over the tiles, in place; the totals
__global__ __launch_bounds__(1024) void k_xbscan(XBuild B) {
    __shared__ unsigned long long s_w[16];
    __shared__ uint32_t s_c[16];
    const uint32_t d = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t *cnt = B.tcnt + (size_t)d * B.ntiles;
    unsigned long long *byt = B.tbyt + (size_t)d * B.ntiles;
    const uint32_t per = (B.ntiles + 1023) / 1024, beg = threadIdx.x * per;
    // up to kScanRegs tiles a thread (a 1M batch: 4) stay in registers between
    // the sum and the offsets: one round trip to memory, not two
    constexpr uint32_t kScanRegs = 8;
    uint32_t rc[kScanRegs];
    uint64_t rb[kScanRegs];
    uint32_t cs = 0;
    uint64_t bs = 0;
    if (per <= kScanRegs) {
#pragma unroll
        for (uint32_t k = 0; k < kScanRegs; ++k) {
            const bool in = k < per && beg + k < B.ntiles;
            rc[k] = in ? cnt[beg + k] : 0u;
            rb[k] = in ? byt[beg + k] : 0ull;
            cs += rc[k];
            bs += rb[k];
        }
    } else {
        for (uint32_t k = 0; k < per; ++k)
            if (beg + k < B.ntiles) {
                cs += cnt[beg + k];
                bs += byt[beg + k];
            }
    }
    uint32_t ci = cs;
    uint64_t bi = bs;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t u = __shfl_up(ci, o);
        const uint64_t ub = __shfl_up(bi, o);
        if (lane >= (uint32_t)o) {
            ci += u;
            bi += ub;
        }
    }
    if (lane == 63) {
        s_c[wave] = ci;
        s_w[wave] = bi;
    }
    __syncthreads();
    uint32_t cp = 0, ct = 0;
    uint64_t bp = 0, bt = 0;
    for (uint32_t w = 0; w < 16; ++w) {
        if (w < wave) {
            cp += s_c[w];
            bp += s_w[w];
        }
        ct += s_c[w];
        bt += s_w[w];
    }
    uint32_t cr = cp + ci - cs;
    uint64_t br = bp + bi - bs;
    if (per <= kScanRegs) {
#pragma unroll
        for (uint32_t k = 0; k < kScanRegs; ++k)
            if (k < per && beg + k < B.ntiles) {
                cnt[beg + k] = cr;
                byt[beg + k] = br;
                cr += rc[k];
                br += rb[k];
            }
    } else {
        for (uint32_t k = 0; k < per; ++k)
            if (beg + k < B.ntiles) {
                const uint32_t c = cnt[beg + k];
                const uint64_t b = byt[beg + k];
                cnt[beg + k] = cr;
                byt[beg + k] = br;
                cr += c;
                br += b;
            }
    }
    if (threadIdx.x == 0) {
        B.seg_n[d] = ct;
        B.seg_bytes[d] = bt;
        if (B.fix_recs)      // the segment's header (fcgpu_xseg): packets, bytes, overflow
            *reinterpret_cast<xu4 *>(B.meta + (size_t)d * (B.fix_recs + 1)) =
                xu4{ct, (uint32_t)bt, (uint32_t)(bt >> 32), (ct > B.fix_recs || bt > B.fix_bytes) ? 1u : 0u};
    }
}

__global__ __launch_bounds__(kXTile) void k_xbuild(XBuild B) {
    __shared__ XTileLds L;
    __shared__ uint32_t s_src[kXTile], s_len[kXTile];
    __shared__ unsigned long long s_dst[kXTile];
    __shared__ uint32_t s_nbase[FCGPU_MAX_PORTS + 1];
    __shared__ unsigned long long s_bbase[FCGPU_MAX_PORTS + 1];
    __shared__ unsigned long long s_big;      // owners whose segment is 4 GiB or more: not packed
    __shared__ uint32_t s_tc[FCGPU_MAX_PORTS];              // the tile's first record / byte within each owner's run
    __shared__ unsigned long long s_tb[FCGPU_MAX_PORTS];
    const uint32_t t = blockIdx.x;
    // the tile's scanned bases (second wave) and the owners' record and byte
    // bases (first wave), loaded before the sort so their latency hides under it
    if (threadIdx.x >= 64 && threadIdx.x < 64 + B.world) {
        const uint32_t d = threadIdx.x - 64;
        s_tc[d] = B.tcnt[(size_t)d * B.ntiles + t];
        s_tb[d] = B.tbyt[(size_t)d * B.ntiles + t];
    }
    if (threadIdx.x < 64) {
        const uint32_t lane = threadIdx.x;
        const uint32_t c = lane < B.world ? B.seg_n[lane] : 0u;
        const uint64_t b = lane < B.world ? B.seg_bytes[lane] : 0ull;
        const uint32_t ci = xwave_incl(c);
        uint64_t bi = b;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint64_t u = __shfl_up(bi, o);
            if (lane >= (uint32_t)o) bi += u;
        }
        if (lane < B.world) {
            s_nbase[lane] = B.fix_recs ? lane * (B.fix_recs + 1) + 1 : ci - c;
            s_bbase[lane] = B.fix_recs ? lane * B.fix_bytes : bi - b;
        }
        // owners not packed: a segment of 4 GiB or more, or (fixed layout)
        // one that does not fit its capacity -- header only
        const bool over = B.fix_recs && (c > B.fix_recs || b > B.fix_bytes);
        const uint64_t big = __ballot(lane < B.world && (b > 0xffffffffull || over));
        if (lane == 0) s_big = big;
    }
    uint32_t own, len, src, pos, intra;
    xtile_sort(B, t, L, own, len, src, pos, intra);      // its barriers publish the bases too
    const uint32_t i = t * kXTile + threadIdx.x;
    if (own < B.world) {
        const uint32_t j = ((s_big >> own) & 1ull) ? ~0u : s_nbase[own] + s_tc[own] + (pos - L.tstart[own]);
        const uint64_t off = s_tb[own] + intra;
        if (j != ~0u) *reinterpret_cast<xu4 *>(B.meta + j) = xu4{(uint32_t)off, len, i, B.rank};
        s_src[pos] = src;
        s_len[pos] = len;
        s_dst[pos] = ((s_big >> own) & 1ull) ? ~0ull : s_bbase[own] + off;
    }
    __syncthreads();
    // The tile's leaving slots, in owner order, as one run of 16-B chunks
    // (L.pre: their byte prefix): lane k takes chunks k, k + 256, ..., four
    // at a time (loads before stores), each found by a binary search of
    // L.pre. Every lane moves data whatever the frame sizes, and a wave's
    // stores are 1 KB contiguous but at owner boundaries.
    const uint32_t nl = L.tstart[B.world];
    const uint32_t nch = L.pre[nl] >> 4;
    // (8 chunks in flight per lane, and non-temporal source loads, measured
    // slower: C4 55.7 / 55.3 / 59.6 against 52.4 us, profiles/r06_exchange/xcopy/)
    constexpr uint32_t kU = 4;
    for (uint32_t c0 = threadIdx.x; c0 < nch; c0 += kXTile * kU) {
        xu4 a[kU];
        uint32_t e[kU], fr[kU], off[kU];
#pragma unroll
        for (uint32_t k = 0; k < kU; ++k) {
            const uint32_t c = c0 + kXTile * k;
            a[k] = xu4{0u, 0u, 0u, 0u};
            e[k] = 0u;
            fr[k] = 0u;
            off[k] = 0u;
            if (c < nch) {
                // the last frame whose slot starts at or before byte 16c
                // (empty slots share their start with the next one)
                const uint32_t x = c << 4;
                uint32_t lo = 0;
#pragma unroll
                for (uint32_t step = kXTile / 2; step; step >>= 1)
                    if (lo + step < nl && L.pre[lo + step] <= x) lo += step;
                fr[k] = lo;
                off[k] = x - L.pre[lo];
                const uint32_t fl = s_len[lo];
                const uint8_t *p = B.arena + s_src[lo] + off[k];
                const uint32_t sh = (uint32_t)(reinterpret_cast<uintptr_t>(p) & 3u);
                xg32 *al = xgbase(p, sh);
                a[k] = *(xg4 *)al;
                // the fifth dword only when the frame reaches into it (so no
                // read goes further than 16 B past the frame's end)
                if (sh && off[k] + 16 - sh < fl) e[k] = al[4];
            }
        }
#pragma unroll
        for (uint32_t k = 0; k < kU; ++k) {
            const uint32_t c = c0 + kXTile * k;
            if (c >= nch) break;
            const uint32_t f = fr[k], fl = s_len[f];
            const uint64_t fd = s_dst[f];
            if (fd == ~0ull || fd + xslot(fl) > B.send_cap) continue;   // nothing past the buffer
            const uint32_t sh = (uint32_t)((reinterpret_cast<uintptr_t>(B.arena) + s_src[f]) & 3u);
            uint32_t v0 = __builtin_amdgcn_alignbyte(a[k].y, a[k].x, sh);
            uint32_t v1 = __builtin_amdgcn_alignbyte(a[k].z, a[k].y, sh);
            uint32_t v2 = __builtin_amdgcn_alignbyte(a[k].w, a[k].z, sh);
            uint32_t v3 = __builtin_amdgcn_alignbyte(e[k], a[k].w, sh);
            const uint32_t rem = fl - off[k];
            if (rem < 16) {
                // the slot's last 16 B: bytes past the frame zero
                auto cut = [rem](uint32_t v, uint32_t j) -> uint32_t {
                    if (rem <= 4 * j) return 0u;
                    const uint32_t keep = rem - 4 * j;
                    return keep >= 4 ? v : v & ((1u << (8 * keep)) - 1u);
                };
                v0 = cut(v0, 0), v1 = cut(v1, 1), v2 = cut(v2, 2), v3 = cut(v3, 3);
            }
            *reinterpret_cast<uint4 *>(B.send + fd + off[k]) = make_uint4(v0, v1, v2, v3);
        }
    }
}

struct XUnpack {
    const uint4 *meta;
    uint32_t *desc;
    uint32_t n, world;
    unsigned long long displ[FCGPU_MAX_PORTS];   // each source's segment start in the received buffer
};

__global__ __launch_bounds__(kXThreads) void k_xunpack(XUnpack U) {
    const uint32_t j = blockIdx.x * kXThreads + threadIdx.x;
    if (j >= U.n) return;
    const xu4 r = *reinterpret_cast<const xu4 *>(U.meta + j);
    const bool ok = r.w < U.world;
    const unsigned long long off = ok ? U.displ[r.w] + r.x : 0ull;
    U.desc[2 * (size_t)j] = (uint32_t)off;
    U.desc[2 * (size_t)j + 1] = ok ? r.y : 0u;
}

// The receive side of the fixed-capacity layout (fcgpu_exchange_unpack_fixed):
// source s's segment (header + records, frames at s x bytes) in place after
// the equal-split all-to-all. Block (c, s): records c*256 .. of source s ->
// descriptors at the exclusive prefix of the sources' packet counts, so the
// list is in (source rank, source order) as the counted exchange's. *count =
// the packets received; 0, with *stall = step (if it was 0), when any
// segment overflowed or an earlier step already stalled -- the flow pass
// that follows then processes nothing and the host replays the stalled steps
// through the counted exchange, in order (fastclick_amd.dist).
struct XUnpackFixed {
    const uint4 *meta;
    uint32_t *desc;
    uint32_t world, recs;
    unsigned long long bytes;
    uint32_t *count;
    uint32_t *stall;
    unsigned long long *total;   // optional: += the count (a running total, no host read per step)
    uint32_t step;
};
__global__ __launch_bounds__(kXThreads) void k_xunpack_fixed(XUnpackFixed U) {
    __shared__ uint32_t s_pre[FCGPU_MAX_PORTS + 1];
    __shared__ uint32_t s_bad;
    const uint32_t lane = threadIdx.x & 63;
    if (threadIdx.x < 64) {
        uint32_t c = 0;
        bool bad = false;
        if (lane < U.world) {
            const xu4 h = *reinterpret_cast<const xu4 *>(U.meta + (size_t)lane * (U.recs + 1));
            const uint64_t b = (uint64_t)h.z << 32 | h.y;
            bad = (h.w & 1u) || h.x > U.recs || b > U.bytes;
            c = bad ? 0u : h.x;
        }
        const uint32_t inc = xwave_incl(c);
        if (lane < U.world) s_pre[lane] = inc - c;
        if (lane == 63) s_pre[U.world] = inc;
        const bool any = __ballot(bad) != 0ull;
        if (lane == 0) s_bad = (any || *U.stall != 0u) ? 1u : 0u;
    }
    __syncthreads();
    const uint32_t s = blockIdx.y;
    if (s_bad) {
        if (blockIdx.x == 0 && s == 0 && threadIdx.x == 0) {
            *U.count = 0u;
            if (*U.stall == 0u) *U.stall = U.step;
        }
        return;
    }
    if (blockIdx.x == 0 && s == 0 && threadIdx.x == 0) {
        *U.count = s_pre[U.world];
        if (U.total) *U.total += s_pre[U.world];
    }
    const uint32_t k = blockIdx.x * kXThreads + threadIdx.x;
    const uint32_t ns = s_pre[s + 1] - s_pre[s];
    if (k >= ns) return;
    const xu4 r = *reinterpret_cast<const xu4 *>(U.meta + (size_t)s * (U.recs + 1) + 1 + k);
    const size_t j = (size_t)s_pre[s] + k;
    U.desc[2 * j] = (uint32_t)(s * U.bytes + r.x);
    U.desc[2 * j + 1] = r.y;
}

}  // namespace fcgpu
