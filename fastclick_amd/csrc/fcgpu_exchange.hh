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
//            thread): bytes its frames take (4-B slots), and the block's
//            partial sum at every segment boundary that falls inside it
//   k_xscan  one workgroup: exclusive scan of the block sums; each owner's
//            segment start = its block's scan value + that partial sum
//   k_xmeta  per packet of perm: its 16-B record {offset within its owner's
//            segment, length, source index, source rank}, staged in LDS and
//            written coalesced; the frame's arena offset into plan scratch
//   k_xpack  the frames into their segments, LPF lanes per frame moving 16 B
//            each (4 / 16 / 64 lanes by the mean frame size): each frame
//            starts 4-B aligned, the bytes of its last dword past its length
//            are zero
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

__device__ __forceinline__ uint64_t xslot(uint32_t len) { return ((uint64_t)len + 3u) & ~(uint64_t)3u; }

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

// LPF lanes per frame, 16 B each per step: four aligned dwords of the source
// and the next one funnel-shifted into four aligned destination dwords
// (frames start anywhere in the arena; the ABI's 16 B of readable slack past
// a frame's end covers the fifth load). Slot bytes past the frame are zero;
// nothing is stored past the slot.
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
    const uintptr_t sa = reinterpret_cast<uintptr_t>(X.arena + so);
    const uint32_t sh = (uint32_t)(sa & 3u);
    const uint32_t *al = reinterpret_cast<const uint32_t *>(sa & ~(uintptr_t)3);
    uint32_t *out = reinterpret_cast<uint32_t *>(X.send + dst);
    for (uint32_t w = 16 * q; w < len; w += 16 * LPF) {
        const xu4 a = *reinterpret_cast<const xu4 *>(al + (w >> 2));
        // the fifth dword only when the frame reaches into it (so no read
        // goes further than 16 B past the frame's end)
        const uint32_t e = sh && w + 16 - sh < len ? al[(w >> 2) + 4] : 0u;
        uint32_t v0 = __builtin_amdgcn_alignbyte(a.y, a.x, sh);
        uint32_t v1 = __builtin_amdgcn_alignbyte(a.z, a.y, sh);
        uint32_t v2 = __builtin_amdgcn_alignbyte(a.w, a.z, sh);
        uint32_t v3 = __builtin_amdgcn_alignbyte(e, a.w, sh);
        const uint32_t rem = len - w;
        if (rem >= 16) {
            xu4 o;
            o.x = v0, o.y = v1, o.z = v2, o.w = v3;
            *reinterpret_cast<xu4 *>(out + (w >> 2)) = o;
        } else {
            // the slot's last dwords: bytes past the frame zero, nothing past the slot
            auto cut = [rem](uint32_t v, uint32_t k) -> uint32_t {
                if (rem <= 4 * k) return 0u;
                const uint32_t keep = rem - 4 * k;
                return keep >= 4 ? v : v & ((1u << (8 * keep)) - 1u);
            };
            const uint32_t nd = (rem + 3) >> 2;
            out[(w >> 2)] = cut(v0, 0);
            if (nd > 1) out[(w >> 2) + 1] = cut(v1, 1);
            if (nd > 2) out[(w >> 2) + 2] = cut(v2, 2);
            if (nd > 3) out[(w >> 2) + 3] = cut(v3, 3);
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

}  // namespace fcgpu
