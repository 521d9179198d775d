// fcgpu_flow_api.hip -- the device flow table:
// FlowIPManagerHMP and the VirtualFlowManager IMP managers with timeouts
// (fcgpu_flow_configure ... fcgpu_flow_count), the new-flow passes that follow
// each k_rx launch (flow_pass, flow_pass_fused) and the maintainer runs
// (fcgpu_flow_maintain). The kernels are fcgpu_flow.hh's; k_rx's lookups
// are in fcgpu_device.hh.
#include "fcgpu_internal.hh"
#include "fcgpu_flow.hh"

using namespace fcgpu;
using namespace fcgpu_rt;

namespace fcgpu_rt {

void flow_free(fcgpu_ctx *c) {
    FlowArgs &F = c->fl;
    for (void *p : {(void *)F.slots, (void *)F.claim, (void *)F.first, (void *)F.miss_key, (void *)F.miss_slot,
                    (void *)F.miss_first, (void *)F.missmask, (void *)F.firstmask, (void *)F.wordpre,
                    (void *)F.state, (void *)F.stack, (void *)F.lastseen, (void *)F.wheel, (void *)F.wheel_len,
                    (void *)c->flow_spare, (void *)c->maint.qbsr, (void *)c->maint.dead, (void *)c->maint.rbuf,
                    (void *)c->maint.counts, (void *)c->fuse_key, (void *)c->fuse_slot, (void *)c->fuse_missed,
                    (void *)c->fuse_mask})
        if (p) hipFree(p);
    if (c->flow_hint) hipHostFree(c->flow_hint);
    c->flow_hint = nullptr;
    c->flow_spare = nullptr;
    c->fuse_key = nullptr;
    c->fuse_slot = c->fuse_missed = nullptr;
    c->fuse_mask = nullptr;
    F = FlowArgs{};
    c->maint = MaintArgs{};
    c->flow_conf = fcgpu_flow_config{};
    c->max_flows = c->flow_slots = c->flow_words = 0;
}

// Empty table, IDs from the start (synchronous).
static int flow_clear(fcgpu_ctx *c) {
    FlowArgs &F = c->fl;
    HIPCHK(c, memset_sync(F.slots, 0, sizeof(uint4) * c->flow_slots));
    HIPCHK(c, memset_sync(F.claim, 0, sizeof(uint32_t) * c->flow_slots));
    HIPCHK(c, memset_sync(F.first, 0xff, sizeof(uint32_t) * c->flow_slots));
    HIPCHK(c, memset_sync(F.missmask, 0, sizeof(uint64_t) * c->flow_words));
    HIPCHK(c, memset_sync(F.firstmask, 0, sizeof(uint64_t) * c->flow_words));
    c->flow_epoch = 0;
    HIPCHK(c, memset_sync(F.state, 0, sizeof(uint32_t) * 16));
    if (F.stack) {
        // FlowManagerIMPState: 0 .. cap-1 pushed in order (virtualflowmanager.hh:113-115);
        // the device stack holds 1 .. cap-1 (ID 0 is the reference's "full")
        std::vector<uint32_t> ids(c->max_flows);
        for (uint32_t i = 0; i < c->max_flows; ++i) ids[i] = i + 1;
        HIPCHK(c, hipMemcpy(F.stack, ids.data(), sizeof(uint32_t) * ids.size(), hipMemcpyHostToDevice));
    }
    if (F.lastseen) {
        HIPCHK(c, memset_sync(F.lastseen, 0, sizeof(uint32_t) * F.wstride));
        HIPCHK(c, memset_sync(F.wheel_len, 0, sizeof(uint32_t) * (F.wmask + 1)));
        HIPCHK(c, memset_sync(c->maint.dead, 0, sizeof(uint32_t) * F.wstride));
        c->maint.seq = 0;
    }
    // an empty table expects many new flows: the grid-wide finish first
    const uint32_t big = kHintBig;
    HIPCHK(c, hipMemcpy(F.state + kFsHint, &big, sizeof big, hipMemcpyHostToDevice));
    *(volatile uint32_t *)c->flow_hint = kHintBig;
    return FCGPU_OK;
}

static uint32_t pow2_at_least(uint32_t x) {
    uint32_t p = 1;
    while (p < x) p <<= 1;
    return p;
}

// The new-flow pass of one batch of n packets (fcgpu_flow.hh), its shape
// predicted by the last pass's class of misses (no sync: maybe older).
hipError_t flow_pass(fcgpu_ctx *c, const FlowArgs &F, uint32_t n, hipStream_t s) {
    const uint32_t nw = (n + 63) / 64;
    if (*(volatile uint32_t *)c->flow_hint == kHintBig) {
        const uint32_t g = std::max(1u, std::min((n + kFlowGridBlock - 1) / kFlowGridBlock, 2048u));
        hipLaunchKernelGGL(k_flow_claim, dim3(g), dim3(kFlowGridBlock), 0, s, F, nw);
        hipLaunchKernelGGL(k_flow_mark, dim3(g), dim3(kFlowGridBlock), 0, s, F, nw);
        hipLaunchKernelGGL(k_flow_scan, dim3(1), dim3(kFinishBlock), 0, s, F, nw);
        hipLaunchKernelGGL(k_flow_assign, dim3(g), dim3(kFlowGridBlock), 0, s, F, nw);
    } else {
        hipLaunchKernelGGL(k_flow_finish, dim3(1), dim3(kFinishBlock), 0, s, F, nw);
    }
    return hipGetLastError();
}

// The new-flow passes of a fused launch's batches, in batch order: one
// block for all of them while the last pass saw few misses, else each
// batch's grid-wide pass.
hipError_t flow_pass_fused(fcgpu_ctx *c, const FlowArgs &F, uint32_t g, const uint32_t *n,
                           uint32_t *const *flowid, uint32_t stride, uint32_t words, uint32_t epoch0, hipStream_t s) {
    if (*(volatile uint32_t *)c->flow_hint != kHintBig) {
        if (g > kMaxFusePass) return hipErrorInvalidValue;
        FinishMulti M{};
        M.g = g;
        M.stride = stride;
        M.words = words;
        for (uint32_t k = 0; k < g; ++k) {
            M.n[k] = n[k];
            M.flowid[k] = flowid[k];
        }
        hipLaunchKernelGGL(k_flow_finish_multi, dim3(1), dim3(kFinishBlock), 0, s, F, M);
        return hipGetLastError();
    }
    for (uint32_t k = 0; k < g; ++k) {
        FlowArgs B = F;
        B.miss_key += (size_t)k * stride;
        B.miss_slot += (size_t)k * stride;
        B.missmask += (size_t)k * words;
        B.missed += k;
        B.epoch = epoch0 + k;
        B.flowid = flowid[k];
        const hipError_t e = flow_pass(c, B, n[k], s);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace fcgpu_rt

extern "C" {

int fcgpu_flow_configure(fcgpu_ctx *c, const fcgpu_flow_config *fc) {
    if (!c || !fc) return FCGPU_EINVAL;
    if (fc->manager != FCGPU_FLOW_MGR_HMP && fc->manager != FCGPU_FLOW_MGR_IMP)
        return fail(c, FCGPU_EINVAL, "flow manager: FCGPU_FLOW_MGR_HMP or FCGPU_FLOW_MGR_IMP");
    const bool imp = fc->manager == FCGPU_FLOW_MGR_IMP;
    if (!imp && fc->timeout_s) return fail(c, FCGPU_EINVAL, "flow timeouts need FCGPU_FLOW_MGR_IMP");
    if (fc->capacity > FCGPU_MAX_FLOWS) return fail(c, FCGPU_EINVAL, "flow capacity above FCGPU_MAX_FLOWS");
    // IMP: CAPACITY rounded up to a power of two (virtualflowmanager.hh:85), IDs 1 .. cap-1
    const uint32_t cap = imp && fc->capacity ? pow2_at_least(std::max(fc->capacity, 2u)) : fc->capacity;
    const uint32_t max_flows = imp && cap ? cap - 1u : cap;
    if (cap > FCGPU_MAX_FLOWS) return fail(c, FCGPU_EINVAL, "flow capacity above FCGPU_MAX_FLOWS");
    uint32_t eps = 0, te = 0, nb = 0;
    if (imp && fc->timeout_s) {
        if (fc->recycle_ms < 1 || fc->recycle_ms > 65535)
            return fail(c, FCGPU_EINVAL, "flow recycle interval must be 1 .. 65535 ms");
        // parse (:58-79): epochs per second, timeout in epochs; TimerWheel::initialize
        eps = std::max(1u, 1000u / fc->recycle_ms);
        if ((uint64_t)fc->timeout_s * eps + 2u > kMaxWheel)
            return fail(c, FCGPU_EINVAL, "flow timeout too long for the recycle interval (timer wheel above 16384 epochs)");
        te = fc->timeout_s * eps;
        nb = pow2_at_least(te + 2u);
        // the maintainer's per-chunk counts: (cap / 1024) x (TE + 1) words
        if ((uint64_t)((cap + kMaintChunk - 1) / kMaintChunk) * (te + 1u) > (1ull << 26))
            return fail(c, FCGPU_EINVAL, "flow timeout in epochs x capacity too large for the maintainer (timer wheel)");
    }
    static_assert(FCGPU_FLOW_MAX_BATCH == 64u * kLdsWords, "fcgpu_flow.hh kLdsWords");
    if (cap && c->max_batch > FCGPU_FLOW_MAX_BATCH)
        return fail(c, FCGPU_EINVAL, "flow table: the context's max_batch is above FCGPU_FLOW_MAX_BATCH");
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipDeviceSynchronize());
    flow_free(c);
    if (cap == 0) return FCGPU_OK;
    // a failure part way leaves no table: never a partial one that the next
    // launch would use (the pointers k_rx reads are all set or all null)
    const int rc = [&]() -> int {
        // at most max_flows IDs plus one batch of FULL markers (the batch that
        // fills the table): keep the load at or under 1/2
        uint32_t slots = 1024;
        while (slots < 2 * (max_flows + c->max_batch)) slots <<= 1;
        const uint32_t words = (c->max_batch + 63) / 64 + 1;
        FlowArgs &F = c->fl;
        HIPCHK(c, dev_malloc(&F.slots, sizeof(uint4) * slots));
        HIPCHK(c, dev_malloc(&F.claim, sizeof(uint32_t) * slots));
        HIPCHK(c, dev_malloc(&F.first, sizeof(uint32_t) * slots));
        HIPCHK(c, dev_malloc(&F.miss_key, sizeof(uint4) * c->max_batch));
        HIPCHK(c, dev_malloc(&F.miss_slot, sizeof(uint32_t) * c->max_batch));
        HIPCHK(c, dev_malloc(&F.miss_first, sizeof(uint32_t) * c->max_batch));
        HIPCHK(c, dev_malloc(&F.missmask, sizeof(uint64_t) * words));
        HIPCHK(c, dev_malloc(&F.firstmask, sizeof(uint64_t) * words));
        HIPCHK(c, dev_malloc(&F.wordpre, sizeof(uint32_t) * words));
        HIPCHK(c, dev_malloc(&F.state, sizeof(uint32_t) * 16));
        F.missed = F.state + kFsMissed;
        if (imp) HIPCHK(c, dev_malloc(&F.stack, sizeof(uint32_t) * max_flows));
        if (te) {
            F.wstride = cap;
            F.wmask = nb - 1;
            F.te = te;
            // lastseen stamps once per run of a flow's packets, read before they
            // write (at 1 / 10k / 1M flows no slower than storing, 2.7 % faster at
            // 10k, 2 % at 1M: profiles/r06_imp/summary.txt). FCGPU_LASTSEEN=
            // run|check|packet forces one way (same-box A/B runs)
            F.ls_mode = kLsCheck;
            if (const char *e = getenv("FCGPU_LASTSEEN")) {
                if (!strcmp(e, "run")) F.ls_mode = kLsRun;
                else if (!strcmp(e, "check")) F.ls_mode = kLsCheck;
                else if (!strcmp(e, "packet")) F.ls_mode = kLsPacket;
            }
            HIPCHK(c, dev_malloc(&F.lastseen, sizeof(uint32_t) * cap));
            HIPCHK(c, dev_malloc(&F.wheel, sizeof(uint32_t) * (size_t)nb * cap));
            HIPCHK(c, dev_malloc(&F.wheel_len, sizeof(uint32_t) * nb));
            HIPCHK(c, dev_malloc(&c->flow_spare, sizeof(uint4) * slots));
            HIPCHK(c, dev_malloc(&c->maint.qbsr, sizeof(uint32_t) * cap));
            HIPCHK(c, dev_malloc(&c->maint.dead, sizeof(uint32_t) * cap));
            HIPCHK(c, dev_malloc(&c->maint.rbuf, sizeof(uint16_t) * cap));
            HIPCHK(c, dev_malloc(&c->maint.counts, sizeof(uint32_t) * (size_t)((cap + kMaintChunk - 1) / kMaintChunk) *
                                                      (te + 1)));
            c->maint.to_ms = fc->timeout_s * 1000u;
            c->maint.ri_ms = fc->recycle_ms;
            c->maint.eps = eps;
        }
        HIPCHK(c, hipHostMalloc((void **)&c->flow_hint, sizeof(uint32_t), hipHostMallocMapped));
        for (auto &e : c->flow_order)
            if (!e) HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
        HIPCHK(c, hipHostGetDevicePointer((void **)&F.host_hint, c->flow_hint, 0));
        F.mask = slots - 1;
        F.max_flows = max_flows;
        c->max_flows = max_flows;
        c->flow_slots = slots;
        c->flow_words = words;
        c->flow_conf = *fc;
        c->flow_conf.capacity = cap;
        return flow_clear(c);
    }();
    if (rc != FCGPU_OK) {
        (void)hipGetLastError();
        flow_free(c);
    }
    return rc;
}

int fcgpu_flow_enable(fcgpu_ctx *c, uint32_t max_flows) {
    if (!c) return FCGPU_EINVAL;
    if (max_flows > FCGPU_MAX_FLOWS) return fail(c, FCGPU_EINVAL, "max_flows above FCGPU_MAX_FLOWS");
    fcgpu_flow_config fc{};
    fc.manager = FCGPU_FLOW_MGR_HMP;
    fc.capacity = max_flows;
    return fcgpu_flow_configure(c, &fc);
}

int fcgpu_flow_set_time(fcgpu_ctx *c, uint32_t now_ms) {
    if (!c) return FCGPU_EINVAL;
    c->flow_now = now_ms;
    return FCGPU_OK;
}

int fcgpu_flow_maintain(fcgpu_ctx *c, uint32_t now_ms, void *stream) {
    if (!c) return FCGPU_EINVAL;
    if (!c->fl.lastseen) return FCGPU_OK;           // no timeouts: nothing expires
    HIPCHK(c, hipSetDevice(c->device));
    // the stream the flow batches are ordered on
    hipStream_t s = c->stream ? c->stream : (hipStream_t)stream;
    if (++c->maint.seq == 0) {                        // run numbers mark released IDs; never 0
        HIPCHK(c, hipMemsetAsync(c->maint.dead, 0, sizeof(uint32_t) * c->fl.wstride, s));
        c->maint.seq = 1;
    }
    MaintArgs M = c->maint;
    M.now = now_ms;
    const uint32_t nch = (c->fl.wstride + kMaintChunk - 1) / kMaintChunk;
    const uint32_t g = std::min(nch, 1024u);
    hipLaunchKernelGGL(k_maint_count, dim3(g), dim3(kMaintChunk), 0, s, c->fl, M);
    hipLaunchKernelGGL(k_maint_scan, dim3(c->fl.te + 1), dim3(kMaintChunk), 0, s, c->fl, M);
    hipLaunchKernelGGL(k_maint_scatter, dim3(g), dim3(kMaintChunk), 0, s, c->fl, M);
    hipLaunchKernelGGL(k_maint_finish, dim3(1), dim3(64), 0, s, c->fl);
    HIPCHK(c, hipGetLastError());
    const size_t bytes = sizeof(uint4) * c->flow_slots;
    HIPCHK(c, hipMemsetAsync(c->flow_spare, 0, bytes, s));
    const uint32_t gr = std::min((c->flow_slots + kFlowGridBlock - 1) / kFlowGridBlock, 4096u);
    hipLaunchKernelGGL(k_flow_rebuild, dim3(gr), dim3(kFlowGridBlock), 0, s, c->fl.slots, c->flow_spare,
                       c->fl.claim, c->fl.mask, c->maint.dead, c->maint.seq);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemsetAsync(c->fl.claim, 0, sizeof(uint32_t) * c->flow_slots, s));
    std::swap(c->fl.slots, c->flow_spare);
    return FCGPU_OK;
}

int fcgpu_flow_stats(fcgpu_ctx *c, fcgpu_flow_stat *st) {
    if (!c || !st) return FCGPU_EINVAL;
    *st = fcgpu_flow_stat{};
    if (!c->fl.slots) return FCGPU_OK;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipDeviceSynchronize());
    uint32_t w[16];
    HIPCHK(c, hipMemcpy(w, c->fl.state, sizeof w, hipMemcpyDeviceToHost));
    st->manager = c->flow_conf.manager;
    st->capacity = c->flow_conf.capacity;
    const uint32_t q = c->fl.lastseen ? w[kFsQlen] : 0u;
    st->count = w[kFsNext] - q;
    st->free_ids = c->max_flows - w[kFsNext];
    st->pending = q;
    st->epochs = c->fl.lastseen ? w[kFsIndex] : 0u;
    return FCGPU_OK;
}

int fcgpu_flow_reset(fcgpu_ctx *c) {
    if (!c) return FCGPU_EINVAL;
    if (!c->fl.slots) return FCGPU_OK;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipDeviceSynchronize());
    return flow_clear(c);
}

int fcgpu_flow_count(fcgpu_ctx *c, uint32_t *count) {
    if (!c || !count) return FCGPU_EINVAL;
    *count = 0;
    if (!c->fl.slots) return FCGPU_OK;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipDeviceSynchronize());
    uint32_t w[16];
    HIPCHK(c, hipMemcpy(w, c->fl.state, sizeof w, hipMemcpyDeviceToHost));
    *count = w[kFsNext] - (c->fl.lastseen ? w[kFsQlen] : 0u);
    return FCGPU_OK;
}

}  // extern "C"
