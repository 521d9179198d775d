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
//   k_xsum   per 2048-packet block of perm: bytes its frames take (4-B slots)
//   k_xscan  one workgroup: exclusive scan of the block sums, then each
//            owner's segment start (the scan at port_start[d])
//   k_xmeta  per packet of perm: its 16-B record {offset within its owner's
//            segment, length, source index, source rank}
//   k_xpack  the frames, 16 lanes per frame, into their segments: each frame
//            starts 4-B aligned, the bytes of its last dword past its length
//            are zero
//   k_xunpack (receiver) records -> descriptors into the received buffer
//
// Byte and index work only: HBM-bound (a frame's bytes read once and written
// once; perm/desc/records read twice), no MFMA.
#pragma once

#include <stdint.h>

#include "fastclick_gpu.h"

namespace fcgpu {

constexpr uint32_t kXThreads = 256;
constexpr uint32_t kXPer = 8;                     // packets per thread per plan block
constexpr uint32_t kXItems = kXThreads * kXPer;   // packets per plan block
constexpr uint32_t kXFramesPerBlock = kXThreads / 16;

__device__ __forceinline__ uint64_t xslot(uint32_t len) { return ((uint64_t)len + 3u) & ~(uint64_t)3u; }

struct XPlan {
    const uint32_t *desc;
    const uint32_t *perm;
    const uint32_t *port_start;
    uint32_t n, world, rank, nblk;
    uint4 *meta;                    // fcgpu_xmeta [n]
    unsigned long long *bsum;       // [nblk + 1] block sums -> exclusive scan (+ total)
    unsigned long long *base;       // [world + 1] segment starts in the send buffer
    unsigned long long *seg_bytes;  // [world]
};

__device__ __forceinline__ uint32_t xsend_count(const XPlan &P) {
    const uint32_t m = P.port_start[P.world];
    return m < P.n ? m : P.n;
}

// 64-bit sum over a 256-thread block (every thread gets it)
__device__ __forceinline__ uint64_t xblock_sum(uint64_t v, unsigned long long *s_w) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d);
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) s_w[wave] = v;
    __syncthreads();
    uint64_t t = 0;
    for (uint32_t w = 0; w < kXThreads / 64; ++w) t += s_w[w];
    return t;
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

__global__ __launch_bounds__(kXThreads) void k_xsum(XPlan P) {
    __shared__ unsigned long long s_w[kXThreads / 64];
    const uint32_t m = xsend_count(P);
    const uint32_t b0 = blockIdx.x * kXItems;
    uint64_t s = 0;
#pragma unroll
    for (uint32_t k = 0; k < kXPer; ++k) {
        const uint32_t j = b0 + k * kXThreads + threadIdx.x;
        if (j < m) s += xslot(P.desc[2 * (size_t)P.perm[j] + 1]);
    }
    s = xblock_sum(s, s_w);
    if (threadIdx.x == 0) P.bsum[blockIdx.x] = s;
}

// One workgroup of 1024 threads: bsum[0..nblk) -> exclusive scan, bsum[nblk]
// = total; then base[d] = scan value at packet port_start[d] (d = 0..world)
// and seg_bytes[d] = base[d+1] - base[d].
__global__ __launch_bounds__(1024) void k_xscan(XPlan P) {
    __shared__ unsigned long long s_w[16];
    __shared__ unsigned long long s_part;
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
    if (threadIdx.x == 0) P.bsum[P.nblk] = total;
    __syncthreads();
    // segment starts: the block's scan value plus the packets of that block
    // before port_start[d] (at most kXItems - 1 of them, 2 per thread)
    const uint32_t m = xsend_count(P);
    uint64_t prev = 0;
    for (uint32_t d = 0; d <= P.world; ++d) {
        uint32_t ps = P.port_start[d];
        ps = ps < m ? ps : m;
        const uint32_t blk = ps / kXItems;
        uint64_t part = 0;
        for (uint32_t j = blk * kXItems + threadIdx.x; j < ps; j += 1024) part += xslot(P.desc[2 * (size_t)P.perm[j] + 1]);
#pragma unroll
        for (int s = 32; s >= 1; s >>= 1) part += __shfl_xor(part, s);
        __syncthreads();
        if (lane == 0) s_w[wave] = part;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint64_t t = 0;
            for (uint32_t w = 0; w < 16; ++w) t += s_w[w];
            s_part = t;
        }
        __syncthreads();
        const uint64_t b = P.bsum[blk] + s_part;   // blk <= nblk: bsum[nblk] is the total
        if (threadIdx.x == 0) {
            P.base[d] = b;
            if (d) P.seg_bytes[d - 1] = b - prev;
        }
        prev = b;
    }
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
    const uint32_t m = xsend_count(P);
    for (uint32_t d = threadIdx.x; d <= P.world; d += kXThreads) {
        const uint32_t ps = P.port_start[d];
        s_ps[d] = ps < m ? ps : m;
        s_base[d] = P.base[d];
    }
    const uint32_t b0 = blockIdx.x * kXItems;
    uint64_t run = P.bsum[blockIdx.x];
    for (uint32_t k = 0; k < kXPer; ++k) {
        const uint32_t j = b0 + k * kXThreads + threadIdx.x;
        const bool live = j < m;
        const uint32_t i = live ? P.perm[j] : 0u;
        const uint32_t len = live ? P.desc[2 * (size_t)i + 1] : 0u;
        uint64_t tot;
        const uint64_t at = run + xblock_excl(live ? xslot(len) : 0u, s_w, &tot);   // syncs: s_ps ready
        run += tot;
        if (live) {
            const uint32_t d = xowner(s_ps, P.world, j);
            P.meta[j] = make_uint4((uint32_t)(at - s_base[d]), len, i, P.rank);
        }
    }
}

struct XPack {
    const uint8_t *arena;
    const uint32_t *desc;
    const uint32_t *port_start;
    const uint4 *meta;
    const unsigned long long *seg_bytes;
    uint8_t *send;
    unsigned long long send_cap;
    uint32_t n, world;
};

// 16 lanes per frame, a dword each per 64-B step: two aligned source loads
// funnel-shifted into one aligned store (frames start anywhere in the arena;
// the ABI's 16 B of readable slack past a frame's end covers the second load).
__global__ __launch_bounds__(kXThreads) void k_xpack(XPack X) {
    __shared__ uint32_t s_ps[FCGPU_MAX_PORTS + 1];
    __shared__ unsigned long long s_base[FCGPU_MAX_PORTS + 1];
    uint32_t m = X.port_start[X.world];
    m = m < X.n ? m : X.n;
    if (threadIdx.x == 0) {
        unsigned long long b = 0;
        for (uint32_t d = 0; d <= X.world; ++d) {
            const uint32_t ps = X.port_start[d];
            s_ps[d] = ps < m ? ps : m;
            s_base[d] = b;
            if (d < X.world) b += X.seg_bytes[d];
        }
    }
    __syncthreads();
    const uint32_t j = blockIdx.x * kXFramesPerBlock + (threadIdx.x >> 4);
    const uint32_t q = threadIdx.x & 15;
    if (j >= m) return;
    const uint4 r = X.meta[j];
    const uint32_t len = r.y;
    const uint64_t dst = s_base[xowner(s_ps, X.world, j)] + r.x;
    if (dst + xslot(len) > X.send_cap) return;     // a send buffer smaller than the plan: nothing past it
    const uint8_t *src = X.arena + X.desc[2 * (size_t)r.z];
    uint32_t *out = reinterpret_cast<uint32_t *>(X.send + dst);
    const uintptr_t sa = reinterpret_cast<uintptr_t>(src);
    const uint32_t sh = (uint32_t)(sa & 3u);
    const uint32_t *al = reinterpret_cast<const uint32_t *>(sa & ~(uintptr_t)3);
    for (uint32_t w = 4 * q; w < len; w += 64) {
        const uint32_t lo = al[w >> 2];
        const uint32_t hi = sh ? al[(w >> 2) + 1] : 0u;
        uint32_t v = __builtin_amdgcn_alignbyte(hi, lo, sh);
        if (len - w < 4) v &= (1u << (8 * (len - w))) - 1u;
        out[w >> 2] = v;
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
    const uint4 r = U.meta[j];
    const bool ok = r.w < U.world;
    const unsigned long long off = ok ? U.displ[r.w] + r.x : 0ull;
    U.desc[2 * (size_t)j] = (uint32_t)off;
    U.desc[2 * (size_t)j + 1] = ok ? r.y : 0u;
}

}  // namespace fcgpu
