// fcgpu_flow.hh -- the new-flow pass of the device flow table (gfx950).
//
// k_rx looks every checked packet up in the table (flow_stage) and appends the
// misses -- packets of flows the table has not seen -- to a miss list in
// arbitrary order. This pass gives each new flow its ID in order of first
// appearance in the batch, exactly as FlowIPManagerHMP's find_create +
// `_current.fetch_and_add(1)` does walking the batch on one thread
// (elements/research/flowipmanagerhmp.cc:96-126):
//
//   k_flow_claim   each miss probes for its key; the first miss of a key to
//                  reach an empty slot claims it (CAS), later misses of the
//                  same key find the claim and compare keys; atomicMin leaves
//                  the flow's first packet index in `first`.
//   k_flow_mark    the first packet of every new flow sets its bit in a
//                  per-batch bitmap over packet indices.
//   k_flow_scan    one block: exclusive popcount prefix over the bitmap words
//                  = rank of each first appearance; snapshots the ID base and
//                  the miss count (and empties the list), advances the ID
//                  counter, clears the other
//                  parity's bitmap for the next batch.
//   k_flow_assign  ID = base + rank of the flow's first packet; the first
//                  packet commits the slot (key + tag) and frees the claim.
//
// Integer work on a few bytes per new flow; with no new flows all four kernels
// exit at their first load.
#pragma once
#include "fcgpu_device.hh"

namespace fcgpu {

constexpr int kFlowBlock = 256;

__global__ __launch_bounds__(kFlowBlock) void k_flow_claim(FlowArgs F) {
    const uint32_t m = F.state[kFsMiss];
    const bool full = F.state[kFsNext] >= F.max_flows;   // no IDs left: no claims
    for (uint32_t e = blockIdx.x * kFlowBlock + threadIdx.x; e < m; e += gridDim.x * kFlowBlock) {
        const uint4 k = F.miss_key[e];
        uint32_t pos = flow_slot_hash(k) & F.mask, slot = kSlotNone;
        for (uint32_t p = 0; !full && p <= F.mask; ++p) {
            const uint4 sl = F.slots[pos];
            if (sl.w == 0) {
                const uint32_t old = atomicCAS(&F.claim[pos], 0u, e + 1);
                if (old == 0 || flow_key_eq(F.miss_key[old - 1], k)) { slot = pos; break; }
            }
            pos = (pos + 1) & F.mask;
        }
        F.miss_slot[e] = slot;
        if (slot != kSlotNone) atomicMin(&F.first[slot], F.miss_pkt[e]);
    }
}

__global__ __launch_bounds__(kFlowBlock) void k_flow_mark(FlowArgs F) {
    const uint32_t m = F.state[kFsMiss];
    uint32_t *bm = F.bitmap + (size_t)(F.state[kFsPar] & 1) * F.state[kFsWords];
    for (uint32_t e = blockIdx.x * kFlowBlock + threadIdx.x; e < m; e += gridDim.x * kFlowBlock) {
        const uint32_t slot = F.miss_slot[e];
        uint32_t fp = kSlotNone;
        if (slot != kSlotNone) {
            fp = F.first[slot];
            const uint32_t pkt = F.miss_pkt[e];
            if (fp == pkt) atomicOr(&bm[pkt >> 5], 1u << (pkt & 31));
        }
        F.miss_first[e] = fp;
    }
}

// One block of 1024 threads; nwords = ceil(n / 32) of this batch.
__global__ __launch_bounds__(1024) void k_flow_scan(FlowArgs F, uint32_t nwords) {
    __shared__ uint32_t s_w[16];
    __shared__ uint32_t s_m;
    const uint32_t t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const uint32_t par = F.state[kFsPar] & 1, W = F.state[kFsWords];
    if (t == 0) s_m = F.state[kFsMiss];
    // the previous batch's bitmap (other parity) is cleared for the next one
    const uint32_t prev = F.state[kFsPrevWords];
    uint32_t *other = F.bitmap + (size_t)(par ^ 1) * W;
    for (uint32_t w = t; w < prev; w += 1024) other[w] = 0;
    __syncthreads();
    const uint32_t m = s_m;
    if (m == 0) {
        if (t == 0) {
            F.state[kFsSnap] = 0;
            F.state[kFsBase] = F.state[kFsNext];
            F.state[kFsPrevWords] = 0;
            F.state[kFsPar] = par ^ 1;
        }
        return;
    }
    const uint32_t *bm = F.bitmap + (size_t)par * W;
    const uint32_t per = (nwords + 1023) / 1024, beg = t * per;
    uint32_t sum = 0;
    for (uint32_t j = 0; j < per; ++j)
        if (beg + j < nwords) sum += (uint32_t)__popc(bm[beg + j]);
    const uint32_t incl = wave_incl_scan(sum);
    if (lane == 63) s_w[wave] = incl;
    __syncthreads();
    uint32_t wpre = 0, total = 0;
    for (uint32_t w = 0; w < 16; ++w) {
        const uint32_t v = s_w[w];
        wpre += w < wave ? v : 0u;
        total += v;
    }
    uint32_t run = wpre + incl - sum;
    for (uint32_t j = 0; j < per; ++j) {
        if (beg + j < nwords) {
            F.wordpre[beg + j] = run;
            run += (uint32_t)__popc(bm[beg + j]);
        }
    }
    if (t == 0) {
        const uint32_t base = F.state[kFsNext];
        const uint32_t room = base < F.max_flows ? F.max_flows - base : 0u;
        F.state[kFsBase] = base;
        F.state[kFsSnap] = m;          // k_flow_assign's count; the list is
        F.state[kFsMiss] = 0;          // free for the next batch's k_rx
        F.state[kFsNext] = base + (total < room ? total : room);
        F.state[kFsPrevWords] = nwords;
        F.state[kFsPar] = par ^ 1;   // k_flow_assign reads this batch's bitmap as par
    }
}

__global__ __launch_bounds__(kFlowBlock) void k_flow_assign(FlowArgs F) {
    const uint32_t m = F.state[kFsSnap];
    if (m == 0) return;
    const uint32_t par = (F.state[kFsPar] & 1) ^ 1;   // flipped by k_flow_scan
    const uint32_t *bm = F.bitmap + (size_t)par * F.state[kFsWords];
    const uint32_t base = F.state[kFsBase];
    for (uint32_t e = blockIdx.x * kFlowBlock + threadIdx.x; e < m; e += gridDim.x * kFlowBlock) {
        const uint32_t pkt = F.miss_pkt[e], slot = F.miss_slot[e], fp = F.miss_first[e];
        uint32_t id = FCGPU_FLOW_FULL;
        if (slot != kSlotNone) {
            const uint32_t w = fp >> 5;
            const uint32_t rank = F.wordpre[w] + (uint32_t)__popc(bm[w] & ((1u << (fp & 31)) - 1u));
            if (base + rank < F.max_flows) id = base + rank;
            if (pkt == fp) {
                // commit; a flow the table had no ID left for is committed
                // as FULL too, so later lookups of keys probing past this
                // slot still find their own
                const uint4 k = F.miss_key[e];
                F.slots[slot] = make_uint4(k.x, k.y, k.z, k.w | ((id != FCGPU_FLOW_FULL ? id + 1u : kTagFull) << 8));
                F.claim[slot] = 0;
                F.first[slot] = 0xffffffffu;
            }
        }
        if (F.flowid) F.flowid[pkt] = id;
    }
}

}  // namespace fcgpu
