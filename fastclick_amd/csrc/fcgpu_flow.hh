// fcgpu_flow.hh -- the new-flow pass of the device flow table (gfx950).
//
// FlowIPManagerHMP's find_create + `_current.fetch_and_add(1)` walked over a
// batch on one thread (elements/research/flowipmanagerhmp.cc:96-126) gives
// every flow, at its first packet, the next ID: IDs are the order of first
// appearance. On the device that is split in two:
//
//   k_rx (flow_issue / flow_resolve, fcgpu_device.hh): every checked packet
//     looks its IPFlow5ID up in the table -- reads only. A miss keeps its
//     record (key, the empty slot its probe stopped at) at its packet index;
//     each wave writes its 64-bit miss word; a wave with a miss stamps the
//     batch's epoch.
//   the new-flow pass (this file, after k_rx, in batch order): every miss
//     looks its key up again from where its probe stopped -- a flow an earlier
//     batch (or an earlier chunk of this one) added since is a hit now -- and
//     otherwise claims a slot: the first miss of a key to reach an empty slot
//     claims it (CAS on `claim`), later misses of the same key find the claim
//     and compare keys, so all misses of one key end on one slot; atomicMin
//     leaves the flow's first packet index in `first`. The first packet of
//     each new flow gets rank = the number of first appearances before it;
//     ID = next + rank. The first packet commits the slot (key + tag) and frees
//     the claim; every miss gets its flow's ID; the counter advances.
//   Because k_rx never writes the table, a batch's lookups need not wait for
//   the previous batch's new-flow pass: a flow that pass adds is a miss the
//   batch's own pass resolves.
//
// Two shapes of pass, chosen by the host from a hint the previous pass
// published in mapped host memory (the size class of its batch's misses):
//
//   k_flow_finish (one block): batch without misses (epoch not stamped) ->
//     returns at its first load; otherwise the misses in packet order, 1024
//     at a time (one chunk when the hint is right): compacted from the miss
//     words into LDS, one per thread, placed, the first packets ranked by a
//     block scan, every other miss finding its flow's first packet by binary
//     search.
//   k_flow_claim / k_flow_mark / k_flow_scan / k_flow_assign (grid-wide, for
//     batches with many misses): every miss placed; each wave marks the first
//     packets among its 64 packets as a 64-bit word; an exclusive popcount
//     prefix over those words (one block, coalesced loads transposed through
//     LDS) ranks them; every miss takes its ID. Nothing needs clearing: every
//     word is rewritten each batch.
#pragma once
#include "fcgpu_device.hh"

namespace fcgpu {

constexpr int kFinishBlock = 1024;
// misses per k_flow_finish chunk, one per thread (four per thread made the
// commit stage of a 4000-miss chunk take 35 us: one CU's stores to random
// slots; the grid-wide pass does such batches in ~24 us)
constexpr uint32_t kSmallFinish = kFinishBlock;
// hint classes (FlowArgs::host_hint)
constexpr uint32_t kHintNone = 0, kHintSmall = 1, kHintBig = 2;

__device__ __forceinline__ uint32_t hint_class(uint32_t m) {
    return m == 0 ? kHintNone : m <= kSmallFinish ? kHintSmall : kHintBig;
}
// Written only when the class changes: a store over the host link costs its
// latency at the end of the launch.
__device__ __forceinline__ void publish_hint(const FlowArgs &F, uint32_t m) {
    const uint32_t h = hint_class(m);
    if (h != F.state[kFsHint]) {
        F.state[kFsHint] = h;
        __hip_atomic_store(F.host_hint, h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// The flow's ID (FULL past max_flows or without a slot); its first packet
// commits the slot (key + tag) and frees the claim. A flow the table had no
// ID left for is committed as FULL too, so later lookups of keys that probe
// past this slot still find their own.
//   HMP: ID = base + rank. IMP: the (base + rank)-th pop of the free-ID stack
//   (virtualflowmanager.hh:264), and with timeouts the first packet stamps the
//   flow and schedules it TE epochs ahead (:293-296): appended, in rank order,
//   to the wheel bucket `wb` whose length was `wbase` when the batch began.
__device__ __forceinline__ void flow_commit(const FlowArgs &F, uint32_t i, uint32_t slot, uint32_t fp,
                                            uint32_t base, uint32_t rank, uint32_t wb, uint32_t wbase) {
    uint32_t id = FCGPU_FLOW_FULL;
    if (slot != kSlotNone) {
        if (base + rank < F.max_flows) id = F.stack ? F.stack[F.max_flows - 1u - (base + rank)] : base + rank;
        if (i == fp) {
            const uint4 k = F.miss_key[i];
            F.slots[slot] = make_uint4(k.x, k.y, k.z, k.w | ((id != FCGPU_FLOW_FULL ? id + 1u : kTagFull) << 8));
            F.claim[slot] = 0;
            F.first[slot] = 0xffffffffu;
            if (F.lastseen && id != FCGPU_FLOW_FULL) {
                F.lastseen[id] = F.now;
                F.wheel[(size_t)wb * F.wstride + wbase + rank] = id;
            }
        }
    }
    if (F.flowid) F.flowid[i] = id;
}

// IMP with timeouts: the bucket new flows go to (schedule_after(fcb, TE),
// timerwheel.hh: index + TE) and its length when the batch began.
__device__ __forceinline__ uint2 flow_new_bucket(const FlowArgs &F) {
    if (!F.lastseen) return make_uint2(0, 0);
    const uint32_t wb = (F.state[kFsIndex] + F.te) & F.wmask;
    return make_uint2(wb, F.wheel_len[wb]);
}

__device__ __forceinline__ uint32_t flow_next_after(const FlowArgs &F, uint32_t next, uint32_t total) {
    const uint32_t room = next < F.max_flows ? F.max_flows - next : 0u;
    return next + (total < room ? total : room);
}

// Miss i of the batch placed in the table: its key looked up again from the
// slot its k_rx probe stopped at (slots only fill between maintainer runs, so
// the key cannot lie before it) -- found: kSlotHit, its ID stored; else the
// empty slot it claims or shares with an earlier miss of the same key (the
// claimant's key, written by k_rx, is compared), its first packet index
// atomicMin'd into `first`. kSlotNone: no IDs left (FCGPU_FLOW_FULL).
constexpr uint32_t kSlotHit = 0xfffffffeu;
__device__ __forceinline__ uint32_t flow_place(const FlowArgs &F, uint32_t i, uint32_t &hid) {
    const uint4 k = F.miss_key[i];
    uint32_t pos = F.miss_slot[i];
    const bool full = __hip_atomic_load(&F.state[kFsNext], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= F.max_flows;
    for (uint32_t p = 0; p <= F.mask; ++p) {
        // agent scope: an earlier chunk of this pass may have committed it
        const uint32_t *sp = reinterpret_cast<const uint32_t *>(&F.slots[pos]);
        const uint32_t tag = __hip_atomic_load(sp + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (tag != 0) {
            if ((tag & 0xffu) == k.w && __hip_atomic_load(sp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == k.x &&
                __hip_atomic_load(sp + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == k.y &&
                __hip_atomic_load(sp + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == k.z) {
                const uint32_t id = flow_tag_id(tag);
                if (F.lastseen && id < kTagFull) F.lastseen[id] = F.now;
                if (F.flowid) F.flowid[i] = id;
                hid = id;
                return kSlotHit;
            }
        } else {
            if (full) return kSlotNone;
            const uint32_t old = atomicCAS(&F.claim[pos], 0u, i + 1);
            if (old == 0) {
                atomicMin(&F.first[pos], i);
                return pos;
            }
            const uint4 o = F.miss_key[old - 1];
            if (o.x == k.x && o.y == k.y && o.z == k.z && o.w == k.w) {
                atomicMin(&F.first[pos], i);
                return pos;
            }
        }
        pos = (pos + 1) & F.mask;
    }
    return kSlotNone;
}

// flow_place for the misses of a wave (`live` lanes; every lane of the wave
// calls it). Misses of one key stop their k_rx probe at the same slot, so the
// lanes sharing a stop slot and the key of the lowest such lane follow that
// lane: it alone places the key (its index is the lowest, so its atomicMin on
// `first` is theirs too) and they take its result. A batch whose misses are
// mostly one new flow (an elephant's first batch) then costs one CAS + one
// atomicMin per wave on the flow's slot, not per packet (1M packets of one new
// flow: 17 ms of contended atomics on one address without this).
__device__ __forceinline__ uint32_t flow_place_wave(const FlowArgs &F, uint32_t i, bool live) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t stop = live ? F.miss_slot[i] : 0u;
    const uint4 k = live ? F.miss_key[i] : make_uint4(0, 0, 0, 0);
    const uint64_t grp = match_any(stop, 32u - __clz(F.mask | 1u), __ballot(live));
    const uint32_t lead = grp ? (uint32_t)__builtin_ctzll(grp) : lane;
    const bool same = __shfl(k.x, (int)lead) == k.x && __shfl(k.y, (int)lead) == k.y &&
                      __shfl(k.z, (int)lead) == k.z && __shfl(k.w, (int)lead) == k.w;
    const bool follow = live && lead != lane && same;
    uint32_t slot = kSlotNone, hid = 0;
    if (live && !follow) slot = flow_place(F, i, hid);
    const uint32_t ls = (uint32_t)__shfl((int)slot, (int)lead), lh = (uint32_t)__shfl((int)hid, (int)lead);
    if (follow) {
        slot = ls;
        if (slot == kSlotHit && F.flowid) F.flowid[i] = lh;
    }
    return slot;
}

// The wave's 64 packets from i0 (a multiple of 64): the first packet of each
// new flow sets its bit in the wave's first-packet word (written even when 0).
__device__ __forceinline__ void flow_mark_wave(const FlowArgs &F, uint32_t i0) {
    const uint32_t lane = threadIdx.x & 63, i = i0 + lane;
    const uint64_t mw = F.missmask[i0 >> 6];
    bool isfirst = false;
    if ((mw >> lane) & 1u) {
        const uint32_t slot = F.miss_slot[i];
        uint32_t fp = kSlotNone;
        if (slot != kSlotNone && slot != kSlotHit) {
            fp = F.first[slot];
            isfirst = fp == i;
        }
        F.miss_first[i] = fp;
    }
    const uint64_t fm = __ballot(isfirst);
    if (lane == 0) F.firstmask[i0 >> 6] = fm;
}

__device__ __forceinline__ void flow_assign_wave(const FlowArgs &F, uint32_t i0, uint32_t base, uint2 wb) {
    const uint32_t lane = threadIdx.x & 63, i = i0 + lane;
    const uint64_t mw = F.missmask[i0 >> 6];
    if ((mw >> lane) & 1u && F.miss_slot[i] != kSlotHit) {
        const uint32_t slot = F.miss_slot[i], fp = F.miss_first[i];
        uint32_t rank = 0;
        if (slot != kSlotNone) {
            const uint32_t w = fp >> 6;
            rank = F.wordpre[w] + (uint32_t)__popcll(F.firstmask[w] & ((1ull << (fp & 63)) - 1ull));
        }
        flow_commit(F, i, slot, fp, base, rank, wb.x, wb.y);
    }
}

// Block-wide exclusive scan of one value per thread; total to every thread.
template <int BS>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t *s_w, uint32_t &total) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t incl = wave_incl_scan(v);
    if (lane == 63) s_w[wave] = incl;
    __syncthreads();
    uint32_t carry = 0;
    total = 0;
    for (uint32_t w = 0; w < BS / 64; ++w) {
        carry += w < wave ? s_w[w] : 0u;
        total += s_w[w];
    }
    __syncthreads();                  // s_w free again
    return carry + incl - v;
}

// The mask words are read coalesced (a word per lane, 16 loads in flight per
// thread) and their popcounts transposed through LDS to the thread-contiguous
// order a block scan needs. (Reading 16 contiguous words per thread instead
// touched 64 lines per load instruction: 25 us for two 128-KB masks.)
constexpr uint32_t kLdsWords = (1u << 14) + 64;   // batches up to 1M + 4096 packets
// s_pre is padded by one word per 16, so a thread walking 16 consecutive words
// hits distinct banks (unpadded, the 64 lanes of a wave shared two banks: 8 us
// of the 13.5 us a 100-miss finish took)
constexpr uint32_t kLdsPadded = kLdsWords + kLdsWords / 16 + 2;
__device__ __forceinline__ uint32_t lw(uint32_t w) { return w + (w >> 4); }

// s_pre[w] = popcount(mask[w]) for w < nw (nw <= kLdsWords); returns this
// thread's share of the total, and of mask2's in `other`. Fixed trip count,
// predicated loads: all of a thread's loads are in flight together (a loop
// with a bound check per step waited for each load in turn: ~16 us).
template <int BS, bool TWO>
__device__ __forceinline__ uint32_t popc_to_lds(const uint64_t *mask, uint32_t nw, uint32_t *s_pre,
                                                const uint64_t *mask2, uint32_t &other) {
    constexpr uint32_t kIt = (kLdsWords + BS - 1) / BS;
    uint64_t a[kIt], b[kIt];
#pragma unroll
    for (uint32_t k = 0; k < kIt; ++k) {
        const uint32_t w = threadIdx.x + k * BS, wc = w < nw ? w : nw - 1;   // clamped: no branch
        a[k] = mask[wc];
        b[k] = TWO ? mask2[wc] : 0ull;
    }
    uint32_t c = 0, c2 = 0;
#pragma unroll
    for (uint32_t k = 0; k < kIt; ++k) {
        const uint32_t w = threadIdx.x + k * BS;
        const uint32_t v = w < nw ? (uint32_t)__popcll(a[k]) : 0u;
        if (w < nw) s_pre[lw(w)] = v;
        c += v;
        c2 += w < nw ? (uint32_t)__popcll(b[k]) : 0u;
    }
    other = c2;
    return c;
}

// One block over the nw 64-bit words: exclusive popcount prefix of the
// first-packet words into wordpre; returns {new flows, misses}.
template <int BS>
__device__ uint2 mask_prefix(const FlowArgs &F, uint32_t nw, uint32_t *s_w, uint32_t *s_pre) {
    uint32_t cm;
    popc_to_lds<BS, true>(F.firstmask, nw, s_pre, F.missmask, cm);
    __syncthreads();
    const uint32_t per = (nw + BS - 1) / BS, w0 = threadIdx.x * per;
    uint32_t sum = 0;
    for (uint32_t k = 0; k < per; ++k)
        if (w0 + k < nw) sum += s_pre[lw(w0 + k)];
    uint32_t tf, tm;
    uint32_t off = block_excl_scan<BS>(sum, s_w, tf);
    block_excl_scan<BS>(cm, s_w, tm);
    for (uint32_t k = 0; k < per; ++k) {
        if (w0 + k < nw) {
            const uint32_t c = s_pre[lw(w0 + k)];
            s_pre[lw(w0 + k)] = off;
            off += c;
        }
    }
    __syncthreads();
    for (uint32_t w = threadIdx.x; w < nw; w += BS) F.wordpre[w] = s_pre[lw(w)];
    return make_uint2(tf, tm);
}

// nw = ceil(n / 64) of this batch (<= kLdsWords). One block of kFinishBlock
// threads. The misses are taken in packet order, kSmallFinish at a time: a
// chunk's misses are compacted into LDS, their slots and first packets loaded
// together, the first packets ranked by a block scan (plus the first packets
// of earlier chunks), and every other miss finds its flow's first packet in
// the chunk by binary search -- or, when it lay in an earlier chunk, takes
// the ID from the slot that chunk committed. Cost grows with the misses, not the
// batch: one chunk for <= 1024 misses.
struct FinishLds {
    uint32_t idx[kSmallFinish], f[kSmallFinish], pre[kLdsPadded];
    uint32_t w[kFinishBlock / 64];
    uint32_t bc[3];
};

// One batch's single-block pass (k_flow_finish, k_flow_finish_multi).
__device__ __forceinline__ void flow_finish_body(const FlowArgs &F, uint32_t nw, FinishLds &L) {
    constexpr uint32_t kQ = kSmallFinish / kFinishBlock;     // misses per thread per chunk
    constexpr uint32_t kIt = (kLdsWords + kFinishBlock - 1) / kFinishBlock;
    uint32_t *s_idx = L.idx, *s_f = L.f, *s_pre = L.pre, *s_w = L.w;
    const uint32_t t = threadIdx.x;
    if (*F.missed != F.epoch) {      // no misses in this batch
        if (t == 0) publish_hint(F, 0);
        return;
    }
    // the table state as the previous pass left it (agent scope: in
    // k_flow_finish_multi that pass ran in this block, its stores by thread 0)
    if (t == 0) {
        L.bc[0] = __hip_atomic_load(&F.state[kFsNext], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        uint2 b = make_uint2(0, 0);
        if (F.lastseen) {
            b.x = (__hip_atomic_load(&F.state[kFsIndex], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + F.te) & F.wmask;
            b.y = __hip_atomic_load(&F.wheel_len[b.x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        L.bc[1] = b.x;
        L.bc[2] = b.y;
    }
    __syncthreads();
    const uint32_t next = L.bc[0];
    const uint2 wb = make_uint2(L.bc[1], L.bc[2]);
    // miss words: word w = t + k * kFinishBlock stays in registers; its
    // popcount goes to LDS, becomes the word's first miss index (exclusive
    // prefix in word order, via thread-contiguous chunks of LDS)
    {
        uint64_t a[kIt];
#pragma unroll
        for (uint32_t k = 0; k < kIt; ++k) {
            const uint32_t w = t + k * kFinishBlock;
            a[k] = F.missmask[w < nw ? w : nw - 1];
        }
#pragma unroll
        for (uint32_t k = 0; k < kIt; ++k) {
            const uint32_t w = t + k * kFinishBlock;
            if (w < nw) s_pre[lw(w)] = (uint32_t)__popcll(a[k]);
        }
    }
    __syncthreads();
    const uint32_t per = (nw + kFinishBlock - 1) / kFinishBlock, w0 = t * per;
    uint32_t c = 0;
    for (uint32_t k = 0; k < per; ++k)
        if (w0 + k < nw) c += s_pre[lw(w0 + k)];
    uint32_t m;
    uint32_t off = block_excl_scan<kFinishBlock>(c, s_w, m);
    for (uint32_t k = 0; k < per; ++k) {
        if (w0 + k < nw) {
            const uint32_t v = s_pre[lw(w0 + k)];
            s_pre[lw(w0 + k)] = off;
            off += v;
        }
    }
    if (t == 0) s_pre[lw(nw)] = m;
    __syncthreads();
    uint32_t nfirst_before = 0;
    for (uint32_t c0 = 0; c0 < m; c0 += kSmallFinish) {
        const uint32_t cn = m - c0 < kSmallFinish ? m - c0 : kSmallFinish;
        // (the words are re-read where they hold misses: keeping all 17 per
        // thread in registers spilled to scratch)
        for (uint32_t k = 0; k < kIt; ++k) {
            const uint32_t w = t + k * kFinishBlock;
            if (w >= nw) break;
            uint32_t e = s_pre[lw(w)];
            const uint32_t e1 = s_pre[lw(w + 1)];
            if (e == e1 || e >= c0 + cn || e1 <= c0) continue;
            uint64_t x = F.missmask[w];
            while (x) {
                if (e >= c0 && e < c0 + cn) s_idx[e - c0] = w * 64 + (uint32_t)__builtin_ctzll(x);
                ++e;
                x &= x - 1;
            }
        }
        __syncthreads();
        // kQ consecutive entries per thread, each placed (found again, or a
        // slot claimed / shared); then every claim and first[] update is in
        const uint32_t e0 = t * kQ;
        uint32_t pkt[kQ], slot[kQ], fp[kQ];
#pragma unroll
        for (uint32_t q = 0; q < kQ; ++q) {
            pkt[q] = e0 + q < cn ? s_idx[e0 + q] : 0u;
            slot[q] = flow_place_wave(F, pkt[q], e0 + q < cn);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        uint32_t nfirst = 0;
#pragma unroll
        for (uint32_t q = 0; q < kQ; ++q) {
            const bool placed = slot[q] != kSlotNone && slot[q] != kSlotHit;
            // agent scope: other waves' atomicMin
            const uint32_t f = __hip_atomic_load(&F.first[placed ? slot[q] : 0u], __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
            fp[q] = placed ? f : kSlotNone;
            nfirst += placed && fp[q] == pkt[q];
        }
        uint32_t nf;
        uint32_t r = nfirst_before + block_excl_scan<kFinishBlock>(nfirst, s_w, nf);
#pragma unroll
        for (uint32_t q = 0; q < kQ; ++q) {
            if (e0 + q < cn) s_f[e0 + q] = r;
            r += slot[q] != kSlotNone && slot[q] != kSlotHit && fp[q] == pkt[q];
        }
        __syncthreads();
#pragma unroll
        for (uint32_t q = 0; q < kQ; ++q) {
            if (e0 + q >= cn || slot[q] == kSlotHit) continue;   // a hit has its ID
            uint32_t rank = 0;
            if (slot[q] != kSlotNone) {
                uint32_t lo = 0, hi = cn;         // the entry of fp in this chunk
                while (lo < hi) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (s_idx[mid] < fp[q]) lo = mid + 1;
                    else hi = mid;
                }
                rank = s_f[lo];
            }
            flow_commit(F, pkt[q], slot[q], fp[q], next, rank, wb.x, wb.y);
        }
        nfirst_before += nf;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // commits done before the next chunk looks
        __syncthreads();                      // s_idx / s_f reused by the next chunk
    }
    if (t == 0) {
        const uint32_t nx = flow_next_after(F, next, nfirst_before);
        F.state[kFsNext] = nx;
        if (F.lastseen) F.wheel_len[wb.x] = wb.y + (nx - next);
        publish_hint(F, m);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
}

__global__ __launch_bounds__(kFinishBlock) void k_flow_finish(FlowArgs F, uint32_t nw) {
    __shared__ FinishLds L;
    flow_finish_body(F, nw, L);
}

// The passes of the batches one fused k_rx launch looked up, in batch order,
// in one block (batch j's miss records at j x stride packets / words past F's,
// its epoch F.epoch + j): a queue of batches without new flows costs one
// launch, not one per batch.
constexpr uint32_t kMaxFusePass = 8;
struct FinishMulti {
    uint32_t g, stride, words;
    uint32_t n[kMaxFusePass];
    uint32_t *flowid[kMaxFusePass];
};
__global__ __launch_bounds__(kFinishBlock) void k_flow_finish_multi(FlowArgs F, FinishMulti M) {
    __shared__ FinishLds L;
    for (uint32_t j = 0; j < M.g; ++j) {
        FlowArgs Fj = F;
        Fj.miss_key += (size_t)j * M.stride;
        Fj.miss_slot += (size_t)j * M.stride;
        Fj.missmask += (size_t)j * M.words;
        Fj.missed += j;
        Fj.epoch += j;
        Fj.flowid = M.flowid[j];
        flow_finish_body(Fj, (M.n[j] + 63) / 64, L);
    }
}

// ---- grid-wide finish (the hint says many misses) ---------------------------
constexpr int kFlowGridBlock = 256;

// Every miss placed (flow_place); hits take their ID here.
__global__ __launch_bounds__(kFlowGridBlock) void k_flow_claim(FlowArgs F, uint32_t nw) {
    if (*F.missed != F.epoch) return;
    for (uint32_t i0 = blockIdx.x * kFlowGridBlock + (threadIdx.x & ~63u); i0 < nw * 64;
         i0 += gridDim.x * kFlowGridBlock) {
        const uint32_t lane = threadIdx.x & 63, i = i0 + lane;
        const bool live = (F.missmask[i0 >> 6] >> lane) & 1u;
        const uint32_t slot = flow_place_wave(F, i, live);
        if (live) F.miss_slot[i] = slot;
    }
}

__global__ __launch_bounds__(kFlowGridBlock) void k_flow_mark(FlowArgs F, uint32_t nw) {
    if (*F.missed != F.epoch) return;
    for (uint32_t i0 = blockIdx.x * kFlowGridBlock + (threadIdx.x & ~63u); i0 < nw * 64;
         i0 += gridDim.x * kFlowGridBlock)
        flow_mark_wave(F, i0);
}

__global__ __launch_bounds__(kFinishBlock) void k_flow_scan(FlowArgs F, uint32_t nw) {
    __shared__ uint32_t s_w[kFinishBlock / 64], s_pre[kLdsPadded];
    if (*F.missed != F.epoch) {
        if (threadIdx.x == 0) publish_hint(F, 0);
        return;
    }
    const uint2 tot = mask_prefix<kFinishBlock>(F, nw, s_w, s_pre);
    if (threadIdx.x == 0) {
        const uint32_t next = F.state[kFsNext], nx = flow_next_after(F, next, tot.x);
        F.state[kFsBase] = next;
        F.state[kFsNext] = nx;
        if (F.lastseen) {
            const uint2 wb = flow_new_bucket(F);
            F.state[kFsWBase] = wb.y;
            F.wheel_len[wb.x] = wb.y + (nx - next);
        }
        publish_hint(F, tot.y);
    }
}

__global__ __launch_bounds__(kFlowGridBlock) void k_flow_assign(FlowArgs F, uint32_t nw) {
    if (*F.missed != F.epoch) return;
    const uint32_t base = F.state[kFsBase];
    const uint2 wb = F.lastseen ? make_uint2((F.state[kFsIndex] + F.te) & F.wmask, F.state[kFsWBase]) : make_uint2(0, 0);
    for (uint32_t i0 = blockIdx.x * kFlowGridBlock + (threadIdx.x & ~63u); i0 < nw * 64;
         i0 += gridDim.x * kFlowGridBlock)
        flow_assign_wave(F, i0, base, wb);
}

// ---- IMP maintainer run (VirtualFlowManagerIMP::maintainer,
// include/click/flow/virtualflowmanager.hh:151-223) ---------------------------
// The reference keeps each wheel bucket as a singly linked list through the
// FCBs (prepend on schedule, walk from the head), and the IDs a run releases
// as another such list pushed back onto the stack at the start of the next
// run. Here a bucket is an array in scheduling order (so the walk is the array
// backwards) and the released IDs an array in release order (pushed back last
// first), which keeps the same order with coalesced accesses.
//
// An entry of the walked bucket goes to the released list (r = 0) or to the
// bucket r epochs ahead (1 <= r <= TE), keeping its walk order within its
// destination: a stable partition of the walk into TE + 1 destinations, done
// grid-wide in 1024-entry chunks of the walk:
//   k_maint_count   (grid) each entry's r (kept in rbuf); per chunk, the count
//                   per destination; also pushes the previous run's releases
//   k_maint_scan    (a block per destination) exclusive scan of its counts
//                   over the chunks, from the destination's current length
//   k_maint_scatter (grid) each entry to its place: the chunk's offset plus
//                   its rank among the chunk's earlier entries of the same r
//   k_maint_finish  the walked bucket emptied, the wheel index advanced
// (One block walking the bucket took 4.1 ms for a 1M-flow bucket, one
// memory latency per 1024 entries.)
constexpr uint32_t kMaxWheel = 1u << 14;     // wheel buckets (LDS counters)
constexpr uint32_t kMaintChunk = 1024;       // walk entries per chunk (= block)
// (the maintainer runs' arguments, MaintArgs, are in fcgpu_device.hh)

// lastseen -> destination: 0 = release, else reschedule r epochs ahead
__device__ __forceinline__ uint32_t maint_dest(const FlowArgs &F, const MaintArgs &M, uint32_t ls) {
    const int32_t old = (int32_t)(M.now - ls);
    if (old <= 0) return F.te;                                   // lastseen not in the past (:174-180)
    if ((uint32_t)old + M.ri_ms >= M.to_ms) return 0;            // expire (:185-205)
    // time left (:209-211); a flow with under one epoch left (eps floored,
    // e.g. RECYCLE_INTERVAL 300 ms) goes one epoch ahead: r = 0 is the
    // reference's "likely a bug" (timerwheel.hh:25 asserts timeout > 0)
    const uint32_t r = ((M.to_ms - (uint32_t)old) * M.eps) / 1000u;
    return r ? r : 1u;
}

// Stable rank of each valid lane among the chunk's earlier lanes with the
// same destination, from the per-destination bases in s_off (advanced past the
// chunk): the waves take turns; inside a wave each distinct r (few: r is the
// flow's remaining idle time in epochs) is one group.
__device__ __forceinline__ uint32_t maint_rank(uint32_t *s_off, bool valid, uint32_t r) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t pos = 0;
    for (uint32_t w = 0; w < kMaintChunk / 64; ++w) {
        if (wave == w) {
            uint64_t rem = __ballot(valid);
            while (rem) {
                const uint32_t leader = (uint32_t)__builtin_ctzll(rem);
                const uint32_t k = __shfl(r, leader);
                const uint64_t m = __ballot(valid && r == k);
                uint32_t b = 0;
                if (lane == leader) {
                    b = s_off[k];
                    s_off[k] = b + (uint32_t)__popcll(m);
                }
                b = __shfl(b, leader);
                if (valid && r == k) pos = b + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
                rem &= ~m;
            }
        }
        __syncthreads();
    }
    return pos;
}

__global__ __launch_bounds__(kMaintChunk) void k_maint_count(FlowArgs F, MaintArgs M) {
    __shared__ uint32_t s_cnt[kMaxWheel];
    const uint32_t t = threadIdx.x;
    const uint32_t idx = F.state[kFsIndex], q = F.state[kFsQlen];
    // the previous run's releases back onto the stack, the list's head (the
    // last released) first (:155-161); k_maint_scatter rewrites qbsr later
    const uint32_t S = F.max_flows - F.state[kFsNext];
    for (uint32_t j = blockIdx.x * kMaintChunk + t; j < q; j += gridDim.x * kMaintChunk)
        F.stack[S + j] = M.qbsr[q - 1u - j];
    const uint32_t cur = idx & F.wmask, n = F.wheel_len[cur], D = F.te + 1u;
    const uint32_t *list = F.wheel + (size_t)cur * F.wstride;
    for (uint32_t c = blockIdx.x; c * kMaintChunk < n; c += gridDim.x) {
        for (uint32_t r = t; r < D; r += kMaintChunk) s_cnt[r] = 0;
        __syncthreads();
        const uint32_t j = c * kMaintChunk + t;
        const bool valid = j < n;
        uint32_t r = 0;
        if (valid) {
            r = maint_dest(F, M, F.lastseen[list[n - 1u - j]]);
            M.rbuf[j] = (uint16_t)r;
        }
        // one LDS add per (wave, destination)
        uint64_t rem = __ballot(valid);
        while (rem) {
            const uint32_t leader = (uint32_t)__builtin_ctzll(rem);
            const uint32_t k = __shfl(r, leader);
            const uint64_t m = __ballot(valid && r == k);
            if ((t & 63) == leader) atomicAdd(&s_cnt[k], (uint32_t)__popcll(m));
            rem &= ~m;
        }
        __syncthreads();
        for (uint32_t d = t; d < D; d += kMaintChunk) M.counts[(size_t)c * D + d] = s_cnt[d];
        __syncthreads();
    }
}

// One block per destination r: its counts over the chunks become offsets
// (its current length + the earlier chunks' counts); its new length written.
__global__ __launch_bounds__(kMaintChunk) void k_maint_scan(FlowArgs F, MaintArgs M) {
    __shared__ uint32_t s_w[kMaintChunk / 64];
    const uint32_t t = threadIdx.x, r = blockIdx.x, D = F.te + 1u;
    const uint32_t idx = F.state[kFsIndex], cur = idx & F.wmask;
    const uint32_t n = F.wheel_len[cur], nch = (n + kMaintChunk - 1) / kMaintChunk;
    const uint32_t dest = (idx + r) & F.wmask;
    const uint32_t base = r ? F.wheel_len[dest] : 0u;
    const uint32_t per = (nch + kMaintChunk - 1) / kMaintChunk, c0 = t * per;
    uint32_t sum = 0;
    for (uint32_t k = 0; k < per; ++k)
        if (c0 + k < nch) sum += M.counts[(size_t)(c0 + k) * D + r];
    uint32_t total;
    uint32_t off = base + block_excl_scan<kMaintChunk>(sum, s_w, total);
    for (uint32_t k = 0; k < per; ++k) {
        if (c0 + k < nch) {
            uint32_t *p = &M.counts[(size_t)(c0 + k) * D + r];
            const uint32_t v = *p;
            *p = off;
            off += v;
        }
    }
    if (t == 0) {
        if (r) {
            F.wheel_len[dest] = base + total;
        } else {
            F.state[kFsNext] -= F.state[kFsQlen];    // the releases pushed by k_maint_count
            F.state[kFsQlen] = total;
        }
    }
}

__global__ __launch_bounds__(kMaintChunk) void k_maint_scatter(FlowArgs F, MaintArgs M) {
    __shared__ uint32_t s_off[kMaxWheel];
    const uint32_t t = threadIdx.x, D = F.te + 1u;
    const uint32_t idx = F.state[kFsIndex], cur = idx & F.wmask, n = F.wheel_len[cur];
    const uint32_t *list = F.wheel + (size_t)cur * F.wstride;
    for (uint32_t c = blockIdx.x; c * kMaintChunk < n; c += gridDim.x) {
        for (uint32_t d = t; d < D; d += kMaintChunk) s_off[d] = M.counts[(size_t)c * D + d];
        __syncthreads();
        const uint32_t j = c * kMaintChunk + t;
        const bool valid = j < n;
        const uint32_t r = valid ? M.rbuf[j] : 0u;
        const uint32_t id = valid ? list[n - 1u - j] : 0u;
        const uint32_t pos = maint_rank(s_off, valid, r);
        if (valid) {
            if (r == 0) {
                M.qbsr[pos] = id;
                M.dead[id] = M.seq;
            } else {
                F.wheel[(size_t)((idx + r) & F.wmask) * F.wstride + pos] = id;
            }
        }
    }
}

__global__ void k_maint_finish(FlowArgs F) {
    if (threadIdx.x == 0) {
        const uint32_t idx = F.state[kFsIndex];
        F.wheel_len[idx & F.wmask] = 0;
        F.state[kFsIndex] = idx + 1u;
    }
}

// The table without the flows this run expired (and without FULL markers:
// the flows they stood for retry when they next arrive, as IDs may be back):
// every other entry re-inserted into the cleared spare slot array. Placement
// differs from the old array's; IDs do not depend on it.
__global__ __launch_bounds__(kFlowGridBlock) void k_flow_rebuild(const uint4 *old, uint4 *slots, uint32_t *claim,
                                                                 uint32_t mask, const uint32_t *dead, uint32_t seq) {
    for (uint32_t s = blockIdx.x * kFlowGridBlock + threadIdx.x; s <= mask; s += gridDim.x * kFlowGridBlock) {
        const uint4 e = old[s];
        const uint32_t tag = e.w >> 8;
        if (e.w == 0 || tag == kTagFull || dead[tag - 1u] == seq) continue;
        uint32_t pos = flow_slot_hash(make_uint4(e.x, e.y, e.z, e.w & 0xffu)) & mask;
        for (uint32_t p = 0; p <= mask; ++p) {
            if (atomicCAS(&claim[pos], 0u, 1u) == 0u) {
                slots[pos] = e;
                break;
            }
            pos = (pos + 1) & mask;
        }
    }
}

}  // namespace fcgpu
