// fcgpu_flow.hh -- the new-flow pass of the device flow table (gfx950).
//
// FlowIPManagerHMP's find_create + `_current.fetch_and_add(1)` walked over a
// batch on one thread (elements/research/flowipmanagerhmp.cc:96-126) gives
// every flow, at its first packet, the next ID: IDs are the order of first
// appearance. On the device that is split in two:
//
//   k_rx (flow_issue / flow_resolve, fcgpu_device.hh): every checked packet
//     looks its IPFlow5ID up in the table. A miss -- a flow the table has not
//     seen -- appends (packet, key) to the batch's miss list and claims a slot
//     for its key: the first miss of a key to reach an empty slot claims it
//     (CAS on `claim`), later misses of the same key find the claim and compare
//     keys, so all misses of one key end on one slot; atomicMin leaves the
//     flow's first packet index in `first`.
//   k_flow_finish (one block, after k_rx): the first packet of each new flow
//     sets its bit in a bitmap over packet indices; an exclusive popcount
//     prefix over the bitmap words gives each first appearance its rank; ID =
//     next + rank. The first packet commits the slot (key + tag) and frees the
//     claim; every miss gets its flow's ID; the counter advances.
//
// With no new flows (steady state) k_flow_finish returns at its first load.
#pragma once
#include "fcgpu_device.hh"

namespace fcgpu {

constexpr int kFinishBlock = 1024;

__device__ __forceinline__ uint32_t ld_agent(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// nwords = ceil(n / 32) of this batch. One block of kFinishBlock threads.
__global__ __launch_bounds__(kFinishBlock) void k_flow_finish(FlowArgs F, uint32_t nwords) {
    __shared__ uint32_t s_w[kFinishBlock / 64];
    const uint32_t t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const uint32_t m = F.state[kFsMiss];
    if (m == 0) return;
    const uint32_t next = F.state[kFsNext];
    // mark the first appearance of every new flow
    for (uint32_t e = t; e < m; e += kFinishBlock) {
        const uint32_t slot = F.miss_slot[e];
        uint32_t fp = kSlotNone;
        if (slot != kSlotNone) {
            fp = ld_agent(&F.first[slot]);
            const uint32_t pkt = F.miss_pkt[e];
            if (fp == pkt) atomicOr(&F.bitmap[pkt >> 5], 1u << (pkt & 31));
        }
        F.miss_first[e] = fp;
    }
    __syncthreads();
    // exclusive popcount prefix over the words: thread t owns a contiguous chunk
    const uint32_t per = (nwords + kFinishBlock - 1) / kFinishBlock, w0 = t * per;
    uint32_t sum = 0;
    for (uint32_t j = 0; j < per; ++j)
        if (w0 + j < nwords) sum += (uint32_t)__popc(ld_agent(&F.bitmap[w0 + j]));
    const uint32_t incl = wave_incl_scan(sum);
    if (lane == 63) s_w[wave] = incl;
    __syncthreads();
    uint32_t run = incl - sum, total = 0;
    for (uint32_t w = 0; w < kFinishBlock / 64; ++w) {
        run += w < wave ? s_w[w] : 0u;
        total += s_w[w];
    }
    for (uint32_t j = 0; j < per; ++j) {
        if (w0 + j < nwords) {
            F.wordpre[w0 + j] = run;
            run += (uint32_t)__popc(ld_agent(&F.bitmap[w0 + j]));
        }
    }
    __syncthreads();
    // IDs; the first packet of a flow commits its slot. A flow the table had
    // no ID left for is committed as FULL too, so later lookups of keys that
    // probe past this slot still find their own.
    for (uint32_t e = t; e < m; e += kFinishBlock) {
        const uint32_t pkt = F.miss_pkt[e], slot = F.miss_slot[e], fp = F.miss_first[e];
        uint32_t id = FCGPU_FLOW_FULL;
        if (slot != kSlotNone) {
            const uint32_t w = fp >> 5;
            const uint32_t rank = ld_agent(&F.wordpre[w]) + (uint32_t)__popc(ld_agent(&F.bitmap[w]) & ((1u << (fp & 31)) - 1u));
            if (next + rank < F.max_flows) id = next + rank;
            if (pkt == fp) {
                const uint4 k = F.miss_key[e];
                F.slots[slot] = make_uint4(k.x, k.y, k.z, k.w | ((id != FCGPU_FLOW_FULL ? id + 1u : kTagFull) << 8));
                F.claim[slot] = 0;
                F.first[slot] = 0xffffffffu;
            }
        }
        if (F.flowid) F.flowid[pkt] = id;
    }
    __syncthreads();
    for (uint32_t w = t; w < nwords; w += kFinishBlock) F.bitmap[w] = 0;
    if (t == 0) {
        const uint32_t room = next < F.max_flows ? F.max_flows - next : 0u;
        F.state[kFsNext] = next + (total < room ? total : room);
        F.state[kFsMiss] = 0;
    }
}

}  // namespace fcgpu
