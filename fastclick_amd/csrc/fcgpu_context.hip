// fcgpu_context.hip -- the context of include/fastclick_gpu.h: open,
// configure, close; counters and sampled timing; errors (fcgpu_last_error)
// and fault injection (fcgpu_inject_fault); page-locked host memory.
//
// A context owns: the uploaded configuration (DevCfg), the partition
// workspace (per-tile histograms + bin totals), the device counter vector,
// pinned/device staging for host-resident batches (fcgpu_process.hip), the
// span slots (fcgpu_span.hip), the flow table (fcgpu_flow_api.hip), the
// exchange scratch (fcgpu_exchange_api.hip) and optional per-stage timing
// events. Launch sequence per batch (all on one stream, fcgpu_process.hip):
//   k_rx   fused check/hash/classify, per-tile histograms, sharded counters,
//          and (FCGPU_PART_TILE) each tile's stable partition  (grid = tiles)
//   FCGPU_PART_GLOBAL only:
//   k_scan per-output exclusive scan over tiles                 (grid = outputs)
//   k_part_multi dense stable partition scatter  (grid = batches' tiles / 8)
//   flow table only: the new-flow pass (fcgpu_flow.hh)
// Queued batches of one stream share one k_rx launch (process_fused).
#include "fcgpu_internal.hh"

using namespace fcgpu;
using namespace fcgpu_rt;

namespace fcgpu_rt {

std::string g_open_err;

// Bytes of each frame the host paths stage (capture.hh): the reach of the
// configured chain, at least 128 B, or whole frames (L4 checksum, PROCESS_EH).
uint32_t host_capture(const fcgpu_ctx *c) {
    const bool autom = c->cfg.check_mode == FCGPU_CHECK_AUTO;
    const uint32_t l3 = (uint32_t)c->cfg.offset + (autom ? 18u : 0u);
    const uint32_t reach = c->cfg.classify == FCGPU_CLS_PROGRAM && !c->prog_host.empty()
                               ? program_reach(c->prog_kind, c->prog_host.data(), (uint32_t)c->prog_host.size(),
                                               l3, l3 + 60)
                               : 0u;
    return capture_bytes(c->cfg, reach);
}

// hipMemset can complete after work already queued on non-blocking streams
// (it is ordered on the null stream only): every setup-time fill waits for
// itself before the buffer is handed to a stream.
hipError_t memset_sync(void *p, int v, size_t bytes) {
    hipError_t e = hipMemsetAsync(p, v, bytes, nullptr);
    if (e != hipSuccess) return e;
    return hipStreamSynchronize(nullptr);
}

int fail(fcgpu_ctx *c, int code, const std::string &msg) {
    if (c) c->err = msg;
    else g_open_err = msg;
    return code;
}


hipEvent_t take_event(fcgpu_ctx *c) {
    if (!c->free_ev.empty()) {
        hipEvent_t e = c->free_ev.back();
        c->free_ev.pop_back();
        return e;
    }
    // timing-only events: no system-scope fence, so recording one does not
    // write back the launch's dirty L2 lines (which would bill the kernel for
    // a cache flush the pipeline never asks for; hip_runtime_api.h notes this
    // flag for timing accuracy)
    hipEvent_t e = nullptr;
    (void)hipEventCreateWithFlags(&e, hipEventDisableSystemFence);
    return e;
}

static std::atomic<uint32_t> g_fault_armed{0};     // bit k: kind k has events to skip or fail
static std::mutex g_fault_mu;
static uint32_t g_fault_skip[4], g_fault_count[4];
bool fault_take(uint32_t where) {
    if (!(g_fault_armed.load(std::memory_order_relaxed) & (1u << where))) return false;
    std::lock_guard<std::mutex> g(g_fault_mu);
    bool hit = false;
    if (g_fault_skip[where]) --g_fault_skip[where];
    else if (g_fault_count[where]) {
        --g_fault_count[where];
        hit = true;
    }
    if (!g_fault_count[where]) g_fault_armed.fetch_and(~(1u << where), std::memory_order_relaxed);
    return hit;
}

hipError_t dev_malloc(void **p, size_t bytes) {
    if (fault_take(FCGPU_FAULT_ALLOC)) return hipErrorOutOfMemory;
    return hipMalloc(p, bytes);
}

hipError_t alloc_group(std::initializer_list<Scratch> g) {
    hipError_t e = hipSuccess;
    for (const Scratch &b : g) {
        if (b.kind == 2) e = fault_take(FCGPU_FAULT_ALLOC) ? hipErrorOutOfMemory
                                                           : hipHostMalloc(b.p, b.bytes, hipHostMallocDefault);
        else e = dev_malloc(b.p, b.bytes);
        if (e == hipSuccess && b.kind == 1) e = memset_sync(*b.p, 0, b.bytes);
        if (e != hipSuccess) break;
    }
    if (e != hipSuccess) {
        (void)hipGetLastError();
        for (const Scratch &b : g) {
            if (*b.p) (void)(b.kind == 2 ? hipHostFree(*b.p) : hipFree(*b.p));
            *b.p = nullptr;
        }
    }
    return e;
}

int alloc_or_fail(fcgpu_ctx *c, const char *what, std::initializer_list<Scratch> g) {
    const hipError_t e = alloc_group(g);
    if (e == hipSuccess) return FCGPU_OK;
    return fail(c, e == hipErrorOutOfMemory ? FCGPU_ENOMEM : FCGPU_ERUNTIME,
                std::string(what) + ": " + hipGetErrorString(e));
}

}  // namespace fcgpu_rt

extern "C" {

int fcgpu_abi_version(void) { return FCGPU_ABI_VERSION; }

int fcgpu_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

void fcgpu_default_cfg(fcgpu_cfg *c) {
    memset(c, 0, sizeof(*c));
    c->size = sizeof(fcgpu_cfg);
    c->check_mode = FCGPU_CHECK_IP4;
    c->offset = 0;
    c->checksum = 0;                   // CheckIPHeader::configure read_or_set(..., 0)
    c->hash_mode = FCGPU_HASH_FLOWID;
    c->classify = FCGPU_CLS_NONE;
    c->nports = 1;
    c->hs_length = 1;
    c->native_vlan = 0;                // StripEtherVLANHeader default NATIVE_VLAN 0
    c->nbad6 = 1;                      // CheckIP6Header default bad source ff..ff
    c->l4_checksum = 1;                // CheckUDPHeader/CheckTCPHeader default CHECKSUM true
    c->ttl_multicast = 1;              // DecIPTTL default MULTICAST true (decipttl.cc:31)
    memset(c->bad6[0], 0xff, 16);
}

const char *fcgpu_last_error(fcgpu_ctx *ctx) { return ctx ? ctx->err.c_str() : g_open_err.c_str(); }

void fcgpu_close(fcgpu_ctx *c) {
    if (!c) return;
    for (uint32_t k = 0; k < FCGPU_SPAN_SLOTS; ++k)      // submissions in the shared queue
        if (c->span[k].agg) fcgpu_span_wait(c, k);
    span_auto_count(c, FCGPU_SPAN_COPY);
    if (c->device >= 0) {
        hipSetDevice(c->device);
        if (c->stream) hipStreamSynchronize(c->stream);
        hipDeviceSynchronize();
        c->jit.unload();
        for (auto &p : c->pending) { hipEventDestroy(p.a); hipEventDestroy(p.b); }
        for (auto e : c->free_ev) hipEventDestroy(e);
        hipFree(c->d_tilecnt);
        hipFree(c->d_totals);
        hipFree(c->fuse_tilecnt);
        hipFree(c->fuse_totals);
        hipFree(c->d_ctr_own);
        hipFree(c->d_prog);
        hipFree(c->d_crc);
        hipFree(c->d_lbtab);
        hipFree(c->d_verdict);
        hipFree(c->d_arena);
        hipFree(c->d_desc);
        hipFree(c->d_hv);
        hipFree(c->d_hh);
        hipFree(c->d_hperm);
        hipFree(c->d_hstart);
        hipFree(c->d_hanno);
        hipFree(c->d_htc);
        hipFree(c->d_htp);
        hipFree(c->d_hflow);
        hipFree(c->d_hrw);
        for (auto &sp : c->span) {
            if (sp.s) hipStreamSynchronize(sp.s);
            for (void *p : {(void *)sp.d_span, (void *)sp.d_desc, (void *)sp.d_v, (void *)sp.d_tc, (void *)sp.d_h,
                            (void *)sp.d_perm, (void *)sp.d_start, (void *)sp.d_fl, (void *)sp.d_rw, (void *)sp.d_an,
                            (void *)sp.d_tp, (void *)sp.d_in, (void *)sp.d_res})
                hipFree(p);
            if (sp.own) hipStreamDestroy(sp.own);
            if (sp.done) hipEventDestroy(sp.done);
        }
        flow_free(c);
        hipFree(c->d_mptr);
        hipFree(c->d_mdesc);
        hipFree(c->x_bsum);
        hipFree(c->x_base);
        hipFree(c->x_part);
        hipFree(c->x_src);
        hipFree(c->x_tcnt);
        hipFree(c->x_tbyt);
        hipFree(c->x_segn);
        hipFree(c->x_segb);
        pool_release(c);
        for (auto e : c->flow_order)
            if (e) hipEventDestroy(e);
        hipHostFree(c->h_arena);
        hipHostFree(c->h_desc);
        if (c->stream) hipStreamDestroy(c->stream);
        for (auto &sl : c->slot) {
            if (sl.s) hipStreamSynchronize(sl.s);
            for (void *p : {(void *)sl.d_arena, (void *)sl.d_desc, (void *)sl.d_v, (void *)sl.d_h, (void *)sl.d_an,
                            (void *)sl.d_perm, (void *)sl.d_tp, (void *)sl.d_tc})
                hipFree(p);
            for (void *p : {(void *)sl.h_arena, (void *)sl.h_desc, (void *)sl.h_v, (void *)sl.h_h, (void *)sl.h_an,
                            (void *)sl.h_perm, (void *)sl.h_tp, (void *)sl.h_tc})
                hipHostFree(p);
            if (sl.done) hipEventDestroy(sl.done);
            if (sl.s) hipStreamDestroy(sl.s);
        }
    }
    delete c;
}

int fcgpu_open(int device, uint32_t max_batch, fcgpu_ctx **out) {
    if (!out || max_batch == 0) return fail(nullptr, FCGPU_EINVAL, "fcgpu_open: bad arguments");
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return fail(nullptr, FCGPU_ENODEV, "fcgpu_open: no HIP device");
    if (device < 0 || device >= ndev) return fail(nullptr, FCGPU_ENODEV, "fcgpu_open: bad device index");
    fcgpu_ctx *c = new fcgpu_ctx();
    c->device = device;
    c->max_batch = max_batch;
    c->max_tiles = (max_batch + kTile - 1) / kTile;
    int rc = FCGPU_OK;
    auto chk = [&](hipError_t e, const char *what) {
        if (e != hipSuccess && rc == FCGPU_OK) rc = fail(c, FCGPU_ENOMEM, std::string(what) + ": " + hipGetErrorString(e));
    };
    chk(hipSetDevice(device), "hipSetDevice");
    chk(hipMalloc(&c->d_tilecnt, sizeof(uint32_t) * (size_t)(FCGPU_MAX_PORTS + 1) * c->max_tiles), "hipMalloc tilecnt");
    chk(hipMalloc(&c->d_totals, sizeof(uint32_t) * kMaxBins), "hipMalloc totals");
    chk(hipMalloc(&c->d_ctr_own, sizeof(unsigned long long) * kCtrWords), "hipMalloc counters");
    c->d_ctr = c->d_ctr_own;
    if (rc == FCGPU_OK) chk(memset_sync(c->d_ctr, 0, sizeof(unsigned long long) * kCtrWords), "hipMemset");
    if (rc != FCGPU_OK) {
        g_open_err = c->err;
        fcgpu_close(c);
        return rc;
    }
    fcgpu_cfg def;
    fcgpu_default_cfg(&def);
    fcgpu_configure(c, &def);
    *out = c;
    return FCGPU_OK;
}

int fcgpu_configure(fcgpu_ctx *c, const fcgpu_cfg *cfg) {
    if (!c || !cfg) return FCGPU_EINVAL;
    if (agg_queued(c)) return fail(c, FCGPU_EINVAL, "fcgpu_configure: a queued span submission is not waited for");
    if (cfg->size != sizeof(fcgpu_cfg)) return fail(c, FCGPU_EINVAL, "fcgpu_cfg size mismatch (ABI)");
    if (cfg->check_mode > FCGPU_MARK_IP6) return fail(c, FCGPU_EINVAL, "bad check_mode");
    const bool ip4mode = cfg->check_mode == FCGPU_CHECK_IP4 || cfg->check_mode == FCGPU_MARK_IP4;
    if (cfg->vlan_ethertype > 0xffff) return fail(c, FCGPU_EINVAL, "bad vlan_ethertype");
    if (cfg->hash_mode > FCGPU_HASH_FLOW5ID) return fail(c, FCGPU_EINVAL, "bad hash_mode");
    if (cfg->classify > FCGPU_CLS_LB_TABLE) return fail(c, FCGPU_EINVAL, "bad classify mode");
    if (cfg->classify == FCGPU_CLS_LB_CRC && !(cfg->check_mode == FCGPU_CHECK_IP4 || cfg->check_mode == FCGPU_MARK_IP4))
        return fail(c, FCGPU_EINVAL, "LB_MODE hash_crc hashes IPFlow5ID: IPv4 check modes only");
    if (cfg->l4_mode > FCGPU_L4_TCP) return fail(c, FCGPU_EINVAL, "bad l4_mode");
    if (cfg->l4_mode != FCGPU_L4_NONE && !ip4mode)
        return fail(c, FCGPU_EINVAL, "l4_mode needs an IPv4 check mode (CHECK_IP4 or MARK_IP4)");
    if (cfg->nports < 1 || cfg->nports > FCGPU_MAX_PORTS) return fail(c, FCGPU_EINVAL, "nports out of range");
    if (cfg->offset < 0 || cfg->offset > 255) return fail(c, FCGPU_EINVAL, "OFFSET out of range [0,255]");
    if (cfg->nbadsrc > FCGPU_MAX_ADDRS || cfg->ngooddst > FCGPU_MAX_ADDRS || cfg->nbad6 > FCGPU_MAX_ADDRS)
        return fail(c, FCGPU_EINVAL, "too many addresses");
    if (cfg->classify == FCGPU_CLS_HASHSWITCH && (cfg->hs_length <= 0 || cfg->hs_offset < 0))
        return fail(c, FCGPU_EINVAL, "length must be > 0");   // hashswitch.cc:40-41
    if (cfg->native_vlan > 0xFFF) return fail(c, FCGPU_EINVAL, "bad NATIVE_VLAN");
    if (cfg->rewrite & ~(FCGPU_RW_DECTTL | FCGPU_RW_SETCKSUM | FCGPU_RW_INPLACE))
        return fail(c, FCGPU_EINVAL, "bad rewrite flags");
    if ((cfg->rewrite & (FCGPU_RW_DECTTL | FCGPU_RW_SETCKSUM)) && !ip4mode)
        return fail(c, FCGPU_EINVAL, "rewrite needs an IPv4 check mode (CHECK_IP4 or MARK_IP4)");
    // the one allocation comes first: a failed reconfiguration leaves the
    // previous configuration (c->cfg and the device config) as it was
    if (cfg->classify == FCGPU_CLS_LB_CRC && !c->d_crc) {
        // U_k[b] = 16 shift steps of b << 8k: rte_hash_crc_4byte's 32 steps
        // are linear, so a word is two rounds of two lookups (fcgpu_device.hh)
        std::vector<uint32_t> t(512);
        for (uint32_t k = 0; k < 2; ++k)
            for (uint32_t b = 0; b < 256; ++b) {
                uint32_t x = b << (8 * k);
                for (int j = 0; j < 16; ++j) x = (x >> 1) ^ (0x82F63B78u & (0u - (x & 1u)));
                t[256 * k + b] = x;
            }
        HIPCHK(c, hipSetDevice(c->device));
        uint4 *tab = nullptr;
        if (int rc = alloc_or_fail(c, "CRC table", {dev_buf(tab, sizeof(uint32_t) * 512)})) return rc;
        if (hipError_t e = hipMemcpy(tab, t.data(), sizeof(uint32_t) * 512, hipMemcpyHostToDevice)) {
            (void)hipFree(tab);
            return fail(c, FCGPU_ERUNTIME, std::string("CRC table upload: ") + hipGetErrorString(e));
        }
        c->d_crc = tab;
    }
    c->cfg = *cfg;
    DevCfg &d = c->dcfg;
    memset(&d, 0, sizeof(d));
    d.offset = cfg->offset;
    d.nports = cfg->nports;
    d.lb_magic = cfg->nports > 1 ? (uint32_t)((((uint64_t)1 << 32) + cfg->nports - 1) / cfg->nports) : 0u;
    d.hash_mode = cfg->hash_mode;
    d.classify = cfg->classify;
    d.hs_offset = cfg->hs_offset;
    d.hs_length = cfg->hs_length;
    d.native_vlan = cfg->native_vlan;
    {
        const uint32_t tpid = cfg->vlan_ethertype ? cfg->vlan_ethertype : 0x8100u;
        d.vlan_tpid = ((tpid & 0xff) << 8) | (tpid >> 8);
    }
    d.nbadsrc = cfg->nbadsrc;
    d.ngooddst = cfg->ngooddst;
    d.nbad6 = cfg->nbad6;
    d.process_eh = cfg->process_eh ? 1u : 0u;
    d.l4_mode = cfg->l4_mode;
    d.l4_checksum = cfg->l4_checksum ? 1u : 0u;
    d.rewrite = (cfg->rewrite & (FCGPU_RW_DECTTL | FCGPU_RW_SETCKSUM)) ? cfg->rewrite : 0u;
    d.ttl_multicast = cfg->ttl_multicast ? 1u : 0u;
    memcpy(d.badsrc, cfg->badsrc, sizeof(d.badsrc));
    memcpy(d.gooddst, cfg->gooddst, sizeof(d.gooddst));
    memcpy(d.bad6, cfg->bad6, sizeof(d.bad6));
    d.crc_tab = cfg->classify == FCGPU_CLS_LB_CRC ? c->d_crc : nullptr;
    d.lb_tab = cfg->classify == FCGPU_CLS_LB_TABLE ? c->d_lbtab : nullptr;
    d.lb_tab_n = c->lbtab_n;
    d.lb_tab_magic = c->lbtab_n > 1 ? (uint32_t)((((uint64_t)1 << 32) + c->lbtab_n - 1) / c->lbtab_n) : 0u;
    d.prog = c->d_prog;
    d.prog_n = c->prog_n;
    d.prog_q = c->prog_q;
    d.prog_tab = c->prog_tab;
    d.prog_kind = c->prog_kind;
    d.prog_all = c->prog_all;
    c->configured = true;
    return FCGPU_OK;
}

int fcgpu_inject_fault(uint32_t where, uint32_t skip, uint32_t count) {
    if (where > FCGPU_FAULT_ALLOC) return FCGPU_EINVAL;
    std::lock_guard<std::mutex> g(g_fault_mu);
    g_fault_skip[where] = count ? skip : 0;
    g_fault_count[where] = count;
    if (count) g_fault_armed.fetch_or(1u << where, std::memory_order_relaxed);
    else g_fault_armed.fetch_and(~(1u << where), std::memory_order_relaxed);
    return FCGPU_OK;
}

int fcgpu_host_register(void *p, size_t bytes, int read_only) {
    if (!p || !bytes) return FCGPU_EINVAL;
    hipError_t e = hipHostRegister(p, bytes, read_only ? hipHostRegisterReadOnly : hipHostRegisterDefault);
    if (e != hipSuccess) {
        g_open_err = std::string("hipHostRegister: ") + hipGetErrorString(e);
        (void)hipGetLastError();
        return FCGPU_ERUNTIME;
    }
    return FCGPU_OK;
}

int fcgpu_host_unregister(void *p) {
    if (!p) return FCGPU_EINVAL;
    return hipHostUnregister(p) == hipSuccess ? FCGPU_OK : FCGPU_ERUNTIME;
}

int fcgpu_set_host_threads(fcgpu_ctx *c, uint32_t nthreads) {
    if (!c || nthreads == 0 || nthreads > 64) return FCGPU_EINVAL;
    c->pool.resize(nthreads);
    return FCGPU_OK;
}

void *fcgpu_host_alloc(size_t bytes) {
    void *p = nullptr;
    if (hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess) return nullptr;
    return p;
}

void fcgpu_host_free(void *p) {
    if (p) hipHostFree(p);
}

void fcgpu_counters_derive(uint64_t *v) {
    if (!v) return;
    uint64_t drops = 0, total = 0;
    for (uint32_t s = 0; s < reason_slot(FCGPU_R_NO_MATCH); ++s) drops += v[FCGPU_CTR_REASON + s];
    for (uint32_t b = 0; b <= FCGPU_MAX_PORTS; ++b) total += v[FCGPU_CTR_PORT + b];
    v[FCGPU_CTR_DROPS] = drops;
    v[FCGPU_CTR_COUNT] = total - drops;
}

int fcgpu_read_counters(fcgpu_ctx *c, uint64_t *out, int n) {
    if (!c || !out || n < 0) return FCGPU_EINVAL;
    if (n > FCGPU_NCOUNTERS) n = FCGPU_NCOUNTERS;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipDeviceSynchronize());
    std::vector<uint64_t> all(kCtrWords), sum(FCGPU_NCOUNTERS, 0);
    HIPCHK(c, hipMemcpy(all.data(), c->d_ctr, sizeof(uint64_t) * kCtrWords, hipMemcpyDeviceToHost));
    for (int k = 0; k < FCGPU_NCOUNTERS; ++k)
        for (int r = 0; r < FCGPU_CTR_SHARDS; ++r) sum[k] += all[(size_t)r * FCGPU_NCOUNTERS + k];
    fcgpu_counters_derive(sum.data());
    for (int k = 0; k < n; ++k) out[k] = sum[k];
    return FCGPU_OK;
}

int fcgpu_reset_counters(fcgpu_ctx *c) {
    if (!c) return FCGPU_EINVAL;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipDeviceSynchronize());
    HIPCHK(c, memset_sync(c->d_ctr, 0, sizeof(unsigned long long) * kCtrWords));
    return FCGPU_OK;
}

int fcgpu_counters_device(fcgpu_ctx *c, uint64_t **d) {
    if (!c || !d) return FCGPU_EINVAL;
    *d = reinterpret_cast<uint64_t *>(c->d_ctr);
    return FCGPU_OK;
}

int fcgpu_use_counters(fcgpu_ctx *c, uint64_t *d) {
    if (!c) return FCGPU_EINVAL;
    c->d_ctr = d ? reinterpret_cast<unsigned long long *>(d) : c->d_ctr_own;
    return FCGPU_OK;
}

int fcgpu_set_timing(fcgpu_ctx *c, int every) {
    if (!c || every < 0) return FCGPU_EINVAL;
    c->timing_every = (uint32_t)every;
    c->timing_seq = 0;
    if (every) {
        // create the events now, not inside a timed region: a sampled launch
        // takes 6 (three stages x start/stop)
        HIPCHK(c, hipSetDevice(c->device));
        while (c->free_ev.size() < kTimingEvents) {
            hipEvent_t e = nullptr;
            HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
            c->free_ev.push_back(e);
        }
    }
    return FCGPU_OK;
}

int fcgpu_read_timing(fcgpu_ctx *c, double *ms, uint32_t *launches, int nstages) {
    if (!c || nstages < 0) return FCGPU_EINVAL;
    HIPCHK(c, hipSetDevice(c->device));
    double acc[3] = {0, 0, 0};
    uint32_t cnt[3] = {0, 0, 0};
    for (auto &p : c->pending) {
        HIPCHK(c, hipEventSynchronize(p.b));
        float t = 0.f;
        HIPCHK(c, hipEventElapsedTime(&t, p.a, p.b));
        acc[p.stage] += t;
        cnt[p.stage] += p.batches;
        c->free_ev.push_back(p.a);
        c->free_ev.push_back(p.b);
    }
    c->pending.clear();
    for (int k = 0; k < nstages && k < 3; ++k) {
        if (ms) ms[k] = acc[k];
        if (launches) launches[k] = cnt[k];
    }
    return FCGPU_OK;
}

}  // extern "C"
