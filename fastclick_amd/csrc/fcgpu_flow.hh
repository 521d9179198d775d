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
//   the finish: the first packet of each new flow gets rank = the number of
//     first appearances before it; ID = next + rank. The first packet commits
//     the slot (key + tag) and frees the claim; every miss gets its flow's ID;
//     the counter advances. The last k_rx workgroup to finish runs it
//     (flow_epilogue, fcgpu_device.hh): up to kInlineFinish misses by an LDS
//     compare, more with a bitmap over packet indices and an exclusive popcount
//     prefix over its words -- unless the host expects a large batch of new
//     flows (the previous batch's miss count, read from a mapped word) and
//     queued k_flow_finish, the same bitmap pass on 1024 threads.
//
// With no new flows (steady state) nothing but the ticket runs.
#pragma once
#include "fcgpu_device.hh"

namespace fcgpu {

constexpr int kFinishBlock = 1024;

// nwords = ceil(n / 32) of this batch. One block of kFinishBlock threads.
__global__ __launch_bounds__(kFinishBlock) void k_flow_finish(FlowArgs F, uint32_t nwords) {
    __shared__ uint32_t s_w[kFinishBlock / 64];
    const uint32_t m = F.state[kFsMiss];
    if (m == 0) return;          // no new flows, or the last k_rx workgroup took them
    flow_finish_block<kFinishBlock>(F, nwords, m, s_w);
}

}  // namespace fcgpu
