// fcgpu_process.hip -- batches through the context: device-resident
// (fcgpu_process: k_rx, then the whole-batch partition passes; queued jobs
// of one stream fused into one k_rx launch, fcgpu_process_jobs),
// host-resident (fcgpu_process_host: pipelined chunks over kSlots streams,
// or one whole batch for a flow table / whole-batch partition), and DPDK-style
// mbufs from a registered pool (fcgpu_pool_register / fcgpu_process_mbufs).
#include "fcgpu_internal.hh"
#include "fcgpu_part.hh"

using namespace fcgpu;
using namespace fcgpu_rt;

namespace fcgpu_rt {

// Tiles per k_part_multi workgroup: up to kPartTiles, while the grid keeps
// ~2048 workgroups (8 per CU) to fill the machine.
static uint32_t part_tiles_per_wg(uint32_t tiles) {
    return std::max(1u, std::min(kPartTiles, tiles / 2048u));
}

// Argument checks shared by fcgpu_process and fcgpu_process_jobs.
int check_process(fcgpu_ctx *c, const uint8_t *d_arena, const uint32_t *d_desc, uint32_t n,
                         const fcgpu_out *o) {
    if (!c->configured) return fail(c, FCGPU_EINVAL, "not configured");
    if (c->cfg.classify == FCGPU_CLS_PROGRAM && !c->d_prog && c->prog_all < 0)
        return fail(c, FCGPU_EINVAL, "FCGPU_CLS_PROGRAM without fcgpu_set_program");
    if (c->cfg.classify == FCGPU_CLS_LB_TABLE && (!c->d_lbtab || c->lbtab_max >= c->cfg.nports))
        return fail(c, FCGPU_EINVAL, "FCGPU_CLS_LB_TABLE without fcgpu_set_lb_table of outputs < nports");
    if (n > c->max_batch) return fail(c, FCGPU_ENOMEM, "batch larger than max_batch");
    if (n && (!d_arena || !d_desc)) return fail(c, FCGPU_EINVAL, "null arena/desc");
    if (o->partition > FCGPU_PART_TILE) return fail(c, FCGPU_EINVAL, "bad partition mode");
    if (o->partition == FCGPU_PART_TILE && ((o->perm || o->tile_perm) != (o->tile_count != nullptr)))
        return fail(c, FCGPU_EINVAL, "FCGPU_PART_TILE needs tile_count and perm and/or tile_perm");
    if (c->fl.slots && c->cfg.check_mode != FCGPU_CHECK_IP4 && c->cfg.check_mode != FCGPU_MARK_IP4)
        return fail(c, FCGPU_EINVAL, "the flow table needs an IPv4 check mode (CHECK_IP4 or MARK_IP4)");
    return FCGPU_OK;
}

// One batch's launches on stream s (arguments checked, device current).
// layout: kLay* bits of the batch's descriptors and annotations (0 through
// the public entry points: {off, len} descriptors, fcgpu_anno).
int process_one(fcgpu_ctx *c, const uint8_t *d_arena, const uint32_t *d_desc, uint32_t n,
                       const fcgpu_out *o, hipStream_t s, uint32_t layout, const uint32_t *n_dev, uint32_t n_base) {
    if (n == 0) return FCGPU_OK;
    const uint32_t ntiles = (n + kTile - 1) / kTile;
    const uint32_t nports = c->cfg.nports;
    uint16_t *verdict = o->verdict;
    if (!verdict && o->partition == FCGPU_PART_GLOBAL && o->perm) {
        if (!c->d_verdict) {
            const int rc = alloc_or_fail(c, "verdict scratch", {dev_buf(c->d_verdict, sizeof(uint16_t) * c->max_batch)});
            if (rc != FCGPU_OK) return rc;
        }
        verdict = c->d_verdict;
    }
    const bool tile = o->partition == FCGPU_PART_TILE;
    const bool tperm = o->perm || o->tile_perm;
    const bool want_global = !tile && (o->perm || o->port_start);
    const int part = tile && tperm ? kPartTile : (want_global ? kPartGlobal : kPartNone);
    RxArgs a;
    a.arena = d_arena;
    a.desc = reinterpret_cast<const uint2 *>(d_desc);
    a.n = n;
    a.ntiles = ntiles;
    a.verdict = verdict;
    a.hash = o->hash;
    a.anno = o->anno;
    a.tilecnt = c->d_tilecnt;
    a.perm = o->perm;
    a.tile_count = o->tile_count;
    a.tile_perm = tile ? o->tile_perm : nullptr;
    if (tile) a.perm = o->perm;
    a.ctr = c->d_ctr;
    a.cfg = c->dcfg;
    a.fl = c->fl;
    a.fl.flowid = o->flowid;
    a.fl.now = c->flow_now;
    if (a.fl.slots) {
        if (++c->flow_epoch == 0) ++c->flow_epoch;   // never 0 (the cleared state)
        a.fl.epoch = c->flow_epoch;
    }
    a.ip_rw = o->ip_rw;
    a.layout = layout;
    a.n_dev = n_dev;
    a.n_base = n_base;

    // sampled timing: the timing_every-th, 2*timing_every-th, ... launch since
    // fcgpu_set_timing (not the first: a start event ahead of an idle queue's
    // first launch would delay it)
    const bool timed = c->timing_every && (++c->timing_seq % c->timing_every) == 0;
    EvPair ev[3];
    if (timed)
        for (int k = 0; k < 3; ++k) { ev[k].a = take_event(c); ev[k].b = take_event(c); ev[k].stage = k; }

    // the flow table's per-batch scratch is shared by every stream the
    // context launches on: a batch on another stream than the one the span
    // submissions use waits for that stream, and that stream for it
    const bool cross = a.fl.slots && c->stream && s != c->stream;
    if (cross) {
        HIPCHK(c, hipEventRecord(c->flow_order[0], c->stream));
        HIPCHK(c, hipStreamWaitEvent(s, c->flow_order[0], 0));
    }
    HIPCHK(c, launch_rx_one(part, c->cfg.check_mode, c->cfg.checksum != 0, a, s, timed ? ev[0].a : nullptr,
                            timed ? ev[0].b : nullptr, c->jit_src.empty() ? nullptr : c));
    HIPCHK(c, hipGetLastError());
    if (a.fl.slots) {   // the batch's new flows get their IDs (fcgpu_flow.hh)
        HIPCHK(c, flow_pass(c, a.fl, n, s));
        if (cross) {
            HIPCHK(c, hipEventRecord(c->flow_order[1], s));
            HIPCHK(c, hipStreamWaitEvent(c->stream, c->flow_order[1], 0));
        }
    }
    if (want_global) {
        if (timed) hipEventRecord(ev[1].a, s);
        hipLaunchKernelGGL(k_scan, dim3(nports + 1), dim3(1024), 0, s, c->d_tilecnt, ntiles, c->d_totals);
        HIPCHK(c, hipGetLastError());
        if (timed) { hipEventRecord(ev[1].b, s); hipEventRecord(ev[2].a, s); }
        PartMulti P{};   // the scatter pass of one batch (k_part_multi with one job)
        P.verdict[0] = verdict;
        P.tileoff[0] = c->d_tilecnt;
        P.totals[0] = c->d_totals;
        P.perm[0] = o->perm;
        P.port_start[0] = o->port_start;
        P.n[0] = o->perm ? n : 0u;
        P.ntiles[0] = ntiles;
        P.wg0[0] = 0;
        P.g = 1;
        P.nports = nports;
        P.tpw = part_tiles_per_wg(ntiles);
        hipLaunchKernelGGL(k_part_multi, dim3(o->perm ? (ntiles + P.tpw - 1) / P.tpw : 1u), dim3(kTile), 0, s, P);
        HIPCHK(c, hipGetLastError());
        if (timed) hipEventRecord(ev[2].b, s);
    }
    if (timed) {
        c->pending.push_back(ev[0]);
        if (want_global) {
            c->pending.push_back(ev[1]);
            c->pending.push_back(ev[2]);
        } else {
            for (int k = 1; k < 3; ++k) { c->free_ev.push_back(ev[k].a); c->free_ev.push_back(ev[k].b); }
        }
    }
    return FCGPU_OK;
}

// The partition shape process_one launches k_rx with for these outputs.
int out_part(const fcgpu_out *o) {
    const bool tile = o->partition == FCGPU_PART_TILE;
    const bool want_global = !tile && (o->perm || o->port_start);
    return tile && (o->perm || o->tile_perm) ? kPartTile : (want_global ? kPartGlobal : kPartNone);
}

// A job that may share a k_rx launch with others: no whole-batch partition
// (context scratch), no in-place header rewrite (jobs may share an arena).
// With a flow table the lookups of the launch's batches only read the table
// and each batch keeps its miss records apart (up to kMaxFuseFlow batches);
// their new-flow passes then run in batch order after the launch.
constexpr uint32_t kMaxFuseFlow = 8;
constexpr uint32_t kFuseCntStride = FCGPU_MAX_PORTS + 2;   // per-batch rows of fuse_tilecnt / fuse_totals
static bool fusable(const fcgpu_ctx *c, const fcgpu_job &j) {
    // a whole-batch partition fuses with its per-batch counts in fuse_tilecnt
    // (not with the flow table, and only with the caller's verdicts, which
    // its scatter pass reads)
    const bool global_ok = out_part(&j.out) != kPartGlobal || (!c->fl.slots && j.out.verdict);
    // header rewrites into the arena do not fuse (jobs may share an arena);
    // rewrites reported through ip_rw do
    return j.n && !(c->cfg.rewrite & FCGPU_RW_INPLACE) && global_ok;
}

static bool outputs_overlap(const fcgpu_out &x, const fcgpu_out &y) {
    const void *a[] = {x.verdict, x.hash, x.anno, x.perm, x.tile_count, x.tile_perm, x.port_start, x.flowid,
                       x.ip_rw};
    const void *b[] = {y.verdict, y.hash, y.anno, y.perm, y.tile_count, y.tile_perm, y.port_start, y.flowid,
                       y.ip_rw};
    for (const void *p : a)
        for (const void *q : b)
            if (p && p == q) return true;
    return false;
}

// Jobs grp[0..g) (fusable, one stream, one partition shape, disjoint outputs)
// as one k_rx launch.
// lay: each job's kLay* bits (nullptr: all 0, the public layouts).
static int process_fused(fcgpu_ctx *c, const fcgpu_job *const *grp, uint32_t g, hipStream_t s,
                         const uint32_t *lay = nullptr) {
    RxLaunch L;
    const fcgpu_out &o0 = grp[0]->out;
    const int part = out_part(&o0);
    RxArgs &a = L.A;
    a = RxArgs{};
    a.tilecnt = c->d_tilecnt;
    a.ctr = c->d_ctr;
    a.cfg = c->dcfg;
    a.fl = c->fl;
    L.njobs = g;
    L.flow_stride = L.flow_words = 0;
    const bool flow = c->fl.slots != nullptr;
    uint32_t epoch0 = 0;
    if (flow) {
        // each batch's miss records apart; one epoch per batch, none 0
        const size_t words = c->flow_words;
        if (!c->fuse_key) {
            const int rc = alloc_or_fail(c, "fused flow scratch",
                                         {dev_buf(c->fuse_key, sizeof(uint4) * (size_t)kMaxFuseFlow * c->max_batch),
                                          dev_buf(c->fuse_slot, sizeof(uint32_t) * (size_t)kMaxFuseFlow * c->max_batch),
                                          dev_buf(c->fuse_mask, sizeof(uint64_t) * kMaxFuseFlow * words, true),
                                          dev_buf(c->fuse_missed, sizeof(uint32_t) * kMaxFuseFlow, true)});
            if (rc != FCGPU_OK) return rc;
        }
        if (c->flow_epoch > 0xffffffffu - 2 * kMaxFuse) c->flow_epoch = 0;
        epoch0 = c->flow_epoch + 1;
        c->flow_epoch += g;
        a.fl.miss_key = c->fuse_key;
        a.fl.miss_slot = c->fuse_slot;
        a.fl.missmask = c->fuse_mask;
        a.fl.missed = c->fuse_missed;
        a.fl.epoch = epoch0;
        a.fl.now = c->flow_now;
        L.flow_stride = c->max_batch;
        L.flow_words = (uint32_t)words;
    }
    if (part == kPartGlobal && !c->fuse_tilecnt) {
        const int rc = alloc_or_fail(
            c, "fused partition scratch",
            {dev_buf(c->fuse_tilecnt, sizeof(uint32_t) * (size_t)kMaxFuse * kFuseCntStride * c->max_tiles),
             dev_buf(c->fuse_totals, sizeof(uint32_t) * (size_t)kMaxFuse * kFuseCntStride)});
        if (rc != FCGPU_OK) return rc;
    }
    uint32_t tiles = 0;
    for (uint32_t k = 0; k < g; ++k) {
        const fcgpu_job &j = *grp[k];
        const bool tile = j.out.partition == FCGPU_PART_TILE;
        RxJob &J = L.job[k];
        J.flowid = j.out.flowid;
        J.arena = j.arena;
        J.desc = reinterpret_cast<const uint2 *>(j.desc);
        J.verdict = j.out.verdict;
        J.hash = j.out.hash;
        J.anno = j.out.anno;
        J.perm = j.out.perm;
        J.tile_count = j.out.tile_count;
        J.tile_perm = tile ? j.out.tile_perm : nullptr;
        J.tilecnt = part == kPartGlobal ? c->fuse_tilecnt + (size_t)k * kFuseCntStride * c->max_tiles : nullptr;
        J.ip_rw = j.out.ip_rw;
        J.ctr = c->d_ctr;
        J.n = j.n;
        J.tile0 = tiles;
        J.layout = lay ? lay[k] : 0u;
        tiles += (j.n + kTile - 1) / kTile;
    }
    L.job_tiles = L.job[0].n ? (L.job[0].n + kTile - 1) / kTile : 0u;
    for (uint32_t k = 1; k < g; ++k)
        if (L.job[k].tile0 != k * L.job_tiles) L.job_tiles = 0;
    if (tiles > g * L.job_tiles) L.job_tiles = 0;    // a last batch larger than the others
    // the first job's pointers also fill A (a workgroup of a fused launch
    // replaces them with its own job's)
    a.arena = L.job[0].arena;
    a.desc = L.job[0].desc;
    a.n = L.job[0].n;
    a.ntiles = (a.n + kTile - 1) / kTile;
    a.layout = L.job[0].layout;
    if (part == kPartGlobal) a.tilecnt = L.job[0].tilecnt;
    // sampled timing counts batches: a fused launch is timed when it covers
    // a multiple of timing_every
    const uint64_t before = c->timing_seq;
    bool timed = false;
    if (c->timing_every) {
        c->timing_seq += g;
        timed = before / c->timing_every != c->timing_seq / c->timing_every;
    }
    EvPair ev;
    if (timed) { ev.a = take_event(c); ev.b = take_event(c); ev.stage = 0; ev.batches = g; }
    // the flow table's scratch is shared with the context's span stream (see process_one)
    const bool cross = flow && c->stream && s != c->stream;
    if (cross) {
        HIPCHK(c, hipEventRecord(c->flow_order[0], c->stream));
        HIPCHK(c, hipStreamWaitEvent(s, c->flow_order[0], 0));
    }
    // a sampled launch is bracketed by two stream markers (hipEventRecord),
    // not by hipExtLaunchKernelGGL's event pair: the pair cost ~4 us more of
    // host enqueue and 5-10 us more per timed region on an idle queue
    // (profiles/r02_s9/evt_ab.txt); the markers' interval adds only the
    // launch's dispatch latency, shared by its batches
    if (timed) HIPCHK(c, hipEventRecord(ev.a, s));
    HIPCHK(c, launch_rx_any(part, c->cfg.check_mode, c->cfg.checksum != 0, L, tiles, s, nullptr, nullptr,
                            c->jit_src.empty() ? nullptr : c));
    if (timed) HIPCHK(c, hipEventRecord(ev.b, s));
    HIPCHK(c, hipGetLastError());
    if (timed) c->pending.push_back(ev);
    if (part == kPartGlobal) {
        // the batches' whole-batch partitions: one scan launch (block (b, j):
        // output b of batch j) and one scatter launch over all their tiles
        const uint32_t nb = c->cfg.nports + 1;
        ScanMulti S{};
        PartMulti P{};
        uint32_t wg = 0, all_tiles = 0;
        for (uint32_t k = 0; k < g; ++k) all_tiles += (grp[k]->n + kTile - 1) / kTile;
        P.tpw = part_tiles_per_wg(all_tiles);
        for (uint32_t k = 0; k < g; ++k) {
            const fcgpu_job &j = *grp[k];
            const uint32_t nt = (j.n + kTile - 1) / kTile;
            S.tilecnt[k] = L.job[k].tilecnt;
            S.totals[k] = c->fuse_totals + (size_t)k * kFuseCntStride;
            S.ntiles[k] = nt;
            P.verdict[k] = j.out.verdict;
            P.tileoff[k] = S.tilecnt[k];
            P.totals[k] = S.totals[k];
            P.perm[k] = j.out.perm;
            P.port_start[k] = j.out.port_start;
            P.n[k] = j.out.perm ? j.n : 0u;
            P.ntiles[k] = nt;
            P.wg0[k] = wg;
            wg += j.out.perm ? (nt + P.tpw - 1) / P.tpw : 1u;
        }
        P.g = g;
        P.nports = c->cfg.nports;
        EvPair e1, e2;
        if (timed) {
            e1.a = take_event(c); e1.b = take_event(c); e1.stage = 1; e1.batches = g;
            e2.a = take_event(c); e2.b = take_event(c); e2.stage = 2; e2.batches = g;
            HIPCHK(c, hipEventRecord(e1.a, s));
        }
        hipLaunchKernelGGL(k_scan_multi, dim3(nb, g), dim3(1024), 0, s, S);
        HIPCHK(c, hipGetLastError());
        if (timed) { HIPCHK(c, hipEventRecord(e1.b, s)); HIPCHK(c, hipEventRecord(e2.a, s)); }
        hipLaunchKernelGGL(k_part_multi, dim3(wg), dim3(kTile), 0, s, P);
        HIPCHK(c, hipGetLastError());
        if (timed) {
            HIPCHK(c, hipEventRecord(e2.b, s));
            c->pending.push_back(e1);
            c->pending.push_back(e2);
        }
    }
    if (flow) {   // the batches' new-flow passes, in batch order
        uint32_t nb[kMaxFuse];
        uint32_t *fid[kMaxFuse];
        for (uint32_t k = 0; k < g; ++k) {
            nb[k] = grp[k]->n;
            fid[k] = grp[k]->out.flowid;
        }
        HIPCHK(c, flow_pass_fused(c, a.fl, g, nb, fid, L.flow_stride, L.flow_words, epoch0, s));
    }
    if (flow) {
        if (cross) {
            HIPCHK(c, hipEventRecord(c->flow_order[1], s));
            HIPCHK(c, hipStreamWaitEvent(c->stream, c->flow_order[1], 0));
        }
    }
    return FCGPU_OK;
}

// Whole batch in one shot (FCGPU_PART_GLOBAL: the partition spans the batch).
static int process_host_whole(fcgpu_ctx *c, const uint8_t *const *frames, const uint32_t *lens, uint32_t n,
                              const fcgpu_out *h) {
    const size_t arena_cap = (size_t)c->max_batch * kHostCap + kArenaPad;
    // the context's own stream exists only for the host-resident path and a
    // flow table's span slots (a stream per context maps onto one of the few
    // hardware queues)
    if (!c->stream) HIPCHK(c, hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    if (!c->d_desc) {
        const int rc = alloc_or_fail(c, "host-resident staging",
                                     {pinned_buf(c->h_desc, sizeof(uint32_t) * 2 * c->max_batch),
                                      dev_buf(c->d_desc, sizeof(uint32_t) * 2 * c->max_batch),
                                      dev_buf(c->d_hv, sizeof(uint16_t) * c->max_batch),
                                      dev_buf(c->d_hh, sizeof(uint32_t) * c->max_batch),
                                      dev_buf(c->d_hperm, sizeof(uint32_t) * c->max_batch),
                                      dev_buf(c->d_hstart, sizeof(uint32_t) * (FCGPU_MAX_PORTS + 2)),
                                      dev_buf(c->d_hanno, sizeof(fcgpu_anno) * c->max_batch),
                                      dev_buf(c->d_htc, sizeof(uint16_t) * (FCGPU_MAX_PORTS + 1) * c->max_tiles),
                                      dev_buf(c->d_htp, (size_t)c->max_batch + kTile)});
        if (rc != FCGPU_OK) return rc;
    }
    // gather: first min(len, 128) bytes of each frame (whole frames for the L4
    // checksum) at 64-B aligned offsets. The device sees the real frame
    // length; bytes past the capture are never needed for a verdict.
    const uint32_t hcap = host_capture(c);
    size_t need = kArenaPad;
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t cap = lens[i] < hcap ? lens[i] : hcap;
        need += cap ? (cap + 63) & ~(size_t)63 : 64;
    }
    if (need > c->h_arena_cap) {          // first use (max_batch * kHostCap), or whole frames past it
        if (c->h_arena) {
            HIPCHK(c, hipStreamSynchronize(c->stream));
            hipHostFree(c->h_arena);
            hipFree(c->d_arena);
        }
        c->h_arena = nullptr;
        c->d_arena = nullptr;
        c->h_arena_cap = 0;
        const size_t want = std::max(need, arena_cap);
        const int rc = alloc_or_fail(c, "host-resident arena", {pinned_buf(c->h_arena, want), dev_buf(c->d_arena, want, true)});
        if (rc != FCGPU_OK) return rc;
        c->h_arena_cap = want;
    }
    size_t off = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t cap = lens[i] < hcap ? lens[i] : hcap;
        memcpy(c->h_arena + off, frames[i], cap);
        c->h_desc[2 * i] = (uint32_t)off;
        c->h_desc[2 * i + 1] = lens[i];
        off += (cap + 63) & ~(size_t)63;
        if (cap == 0) off += 64;
    }
    hipStream_t s = c->stream;
    HIPCHK(c, hipMemcpyAsync(c->d_arena, c->h_arena, off, hipMemcpyHostToDevice, s));
    HIPCHK(c, hipMemcpyAsync(c->d_desc, c->h_desc, sizeof(uint32_t) * 2 * n, hipMemcpyHostToDevice, s));
    fcgpu_out d;
    d.verdict = c->d_hv;
    d.hash = h->hash ? c->d_hh : nullptr;
    d.anno = h->anno ? c->d_hanno : nullptr;
    d.perm = h->perm ? c->d_hperm : nullptr;
    d.port_start = h->port_start ? c->d_hstart : nullptr;
    d.tile_count = h->tile_count ? c->d_htc : nullptr;
    d.partition = h->partition;
    d.reserved = 0;
    d.tile_perm = h->tile_perm ? c->d_htp : nullptr;
    if (h->flowid && !c->d_hflow) {
        const int rc = alloc_or_fail(c, "host-resident flow IDs", {dev_buf(c->d_hflow, sizeof(uint32_t) * c->max_batch)});
        if (rc != FCGPU_OK) return rc;
    }
    d.flowid = h->flowid ? c->d_hflow : nullptr;
    if (h->ip_rw && !c->d_hrw) {
        const int rc = alloc_or_fail(c, "host-resident ip_rw", {dev_buf(c->d_hrw, sizeof(uint32_t) * c->max_batch)});
        if (rc != FCGPU_OK) return rc;
    }
    d.ip_rw = h->ip_rw ? c->d_hrw : nullptr;
    int rc = fcgpu_process(c, c->d_arena, c->d_desc, n, &d, s);
    if (rc != FCGPU_OK) return rc;
    if (h->verdict) HIPCHK(c, hipMemcpyAsync(h->verdict, d.verdict, sizeof(uint16_t) * n, hipMemcpyDeviceToHost, s));
    if (h->hash) HIPCHK(c, hipMemcpyAsync(h->hash, d.hash, sizeof(uint32_t) * n, hipMemcpyDeviceToHost, s));
    if (h->flowid) HIPCHK(c, hipMemcpyAsync(h->flowid, d.flowid, sizeof(uint32_t) * n, hipMemcpyDeviceToHost, s));
    if (h->ip_rw) HIPCHK(c, hipMemcpyAsync(h->ip_rw, d.ip_rw, sizeof(uint32_t) * n, hipMemcpyDeviceToHost, s));
    if (h->anno) HIPCHK(c, hipMemcpyAsync(h->anno, d.anno, sizeof(fcgpu_anno) * n, hipMemcpyDeviceToHost, s));
    if (h->perm) HIPCHK(c, hipMemcpyAsync(h->perm, d.perm, sizeof(uint32_t) * n, hipMemcpyDeviceToHost, s));
    if (h->tile_perm) HIPCHK(c, hipMemcpyAsync(h->tile_perm, d.tile_perm, n, hipMemcpyDeviceToHost, s));
    if (h->tile_count)
        HIPCHK(c, hipMemcpyAsync(h->tile_count, d.tile_count,
                                 sizeof(uint16_t) * (c->cfg.nports + 1) * ((n + kTile - 1) / kTile),
                                 hipMemcpyDeviceToHost, s));
    if (h->port_start)
        HIPCHK(c, hipMemcpyAsync(h->port_start, d.port_start, sizeof(uint32_t) * (c->cfg.nports + 2),
                                 hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    return FCGPU_OK;
}

static int slot_alloc(fcgpu_ctx *c, HostSlot &sl, uint32_t cap) {
    const size_t tiles = (cap + kTile - 1) / kTile;
    if (!sl.s) HIPCHK(c, hipStreamCreateWithFlags(&sl.s, hipStreamNonBlocking));
    if (!sl.done) HIPCHK(c, hipEventCreateWithFlags(&sl.done, hipEventDisableTiming));
    if (sl.d_desc) return FCGPU_OK;       // made by an earlier call (the group is all or nothing)
    const size_t arena = (size_t)cap * kHostCap + kArenaPad;
    const int rc = alloc_or_fail(c, "host-resident slot",
                                 {pinned_buf(sl.h_arena, arena), pinned_buf(sl.h_desc, sizeof(uint32_t) * 2 * cap),
                                  dev_buf(sl.d_arena, arena, true), dev_buf(sl.d_desc, sizeof(uint32_t) * 2 * cap),
                                  dev_buf(sl.d_v, sizeof(uint16_t) * cap), dev_buf(sl.d_h, sizeof(uint32_t) * cap),
                                  dev_buf(sl.d_an, sizeof(fcgpu_anno) * cap), dev_buf(sl.d_perm, sizeof(uint32_t) * cap),
                                  dev_buf(sl.d_tp, (size_t)cap + kTile),
                                  dev_buf(sl.d_tc, sizeof(uint16_t) * (FCGPU_MAX_PORTS + 1) * tiles),
                                  pinned_buf(sl.h_v, sizeof(uint16_t) * cap), pinned_buf(sl.h_h, sizeof(uint32_t) * cap),
                                  pinned_buf(sl.h_an, sizeof(fcgpu_anno) * cap),
                                  pinned_buf(sl.h_perm, sizeof(uint32_t) * cap), pinned_buf(sl.h_tp, (size_t)cap + kTile),
                                  pinned_buf(sl.h_tc, sizeof(uint16_t) * (FCGPU_MAX_PORTS + 1) * tiles)});
    if (rc != FCGPU_OK) return rc;
    sl.arena_cap = arena;
    return FCGPU_OK;
}

struct PinnedOut {           // which caller arrays the DMA engine can write directly
    bool v, h, an, perm, tp, tc;
};

// Copy a finished chunk's outputs from pinned staging into the caller's
// (pageable) arrays; `perm` entries become batch indices.
static void slot_drain(fcgpu_ctx *c, HostSlot &sl, const fcgpu_out *h, const PinnedOut &pin) {
    const uint32_t nb = c->cfg.nports + 1, n = sl.n, base = sl.base;
    const uint32_t ntile = (n + kTile - 1) / kTile, tbase = base / kTile;
    c->pool.run([&](uint32_t part, uint32_t np) {
        const uint32_t lo = span(n, part, np), hi = span(n, part + 1, np);
        if (hi <= lo) return;
        if (h->verdict && !pin.v) memcpy(h->verdict + base + lo, sl.h_v + lo, sizeof(uint16_t) * (hi - lo));
        if (h->hash && !pin.h) memcpy(h->hash + base + lo, sl.h_h + lo, sizeof(uint32_t) * (hi - lo));
        if (h->anno && !pin.an) memcpy(h->anno + base + lo, sl.h_an + lo, sizeof(fcgpu_anno) * (hi - lo));
        if (h->tile_perm && !pin.tp) memcpy(h->tile_perm + base + lo, sl.h_tp + lo, hi - lo);
        if (h->perm) {
            uint32_t *dst = h->perm + base;
            const uint32_t *src = pin.perm ? dst : sl.h_perm;
            for (uint32_t k = lo; k < hi; ++k) dst[k] = src[k] + base;
        }
        if (h->tile_count && !pin.tc && part == 0)
            memcpy(h->tile_count + (size_t)tbase * nb, sl.h_tc, sizeof(uint16_t) * nb * ntile);
    });
    sl.busy = false;
}

// Host-resident batches, pipelined in chunks of kChunk packets over kSlots
// streams: while chunk k is copied in, classified and copied out on its own
// stream, the host gathers chunk k+1 (and drains chunk k-2). Every chunk is a
// whole number of 256-packet tiles, so per-tile outputs are those of the
// whole batch.
static int process_host_pipelined(fcgpu_ctx *c, const uint8_t *const *frames, const uint32_t *lens, uint32_t n,
                                  const fcgpu_out *h) {
    if (!c->slot_cap) {
        uint32_t chunk = kChunk;
        if (const char *e = getenv("FCGPU_HOST_CHUNK")) {      // tuning knob (packets, whole tiles)
            const long v = atol(e);
            if (v >= kTile && v <= (1L << 24)) chunk = (uint32_t)v;
        }
        uint32_t cap = c->max_batch < chunk ? c->max_batch : chunk;
        cap = (cap + kTile - 1) / kTile * kTile;
        for (auto &sl : c->slot) {
            int rc = slot_alloc(c, sl, cap);
            if (rc != FCGPU_OK) return rc;
        }
        c->slot_cap = cap;
    }
    const uint32_t cap = c->slot_cap, nb = c->cfg.nports + 1;
    PinnedOut pin{host_pinned(h->verdict), host_pinned(h->hash), host_pinned(h->anno), host_pinned(h->perm),
                  host_pinned(h->tile_perm), host_pinned(h->tile_count)};
    const uint32_t nchunks = (n + cap - 1) / cap;
    for (uint32_t k = 0; k < nchunks; ++k) {
        HostSlot &sl = c->slot[k % kSlots];
        if (sl.busy) {
            HIPCHK(c, hipEventSynchronize(sl.done));
            slot_drain(c, sl, h, pin);
        }
        const uint32_t base = k * cap, cn = n - base < cap ? n - base : cap;
        // gather the first min(len, 128) B of every frame (whole frames when
        // the L4 checksum needs them) at 64-B aligned offsets: sizes per
        // part, then parts copy in parallel
        const uint32_t np = c->pool.size();
        const uint32_t hcap = host_capture(c);
        std::vector<size_t> part_off(np + 1, 0);
        c->pool.run([&](uint32_t part, uint32_t nparts) {
            size_t sz = 0;
            for (uint32_t i = span(cn, part, nparts); i < span(cn, part + 1, nparts); ++i) {
                const uint32_t L = lens[base + i], cp = L < hcap ? L : hcap;
                sz += cp ? (cp + 63) & ~63u : 64;
            }
            part_off[part + 1] = sz;
        });
        for (uint32_t p = 0; p < np; ++p) part_off[p + 1] += part_off[p];
        if (part_off[np] + kArenaPad > sl.arena_cap) {      // whole frames: grow the slot's arena
            const size_t want = (part_off[np] + kArenaPad) * 5 / 4;
            hipHostFree(sl.h_arena);
            hipFree(sl.d_arena);
            sl.h_arena = nullptr;
            sl.d_arena = nullptr;
            sl.arena_cap = 0;
            const int rc = alloc_or_fail(c, "host-resident slot arena",
                                         {pinned_buf(sl.h_arena, want), dev_buf(sl.d_arena, want, true)});
            if (rc != FCGPU_OK) return rc;
            sl.arena_cap = want;
        }
        c->pool.run([&](uint32_t part, uint32_t nparts) {
            size_t off = part_off[part];
            for (uint32_t i = span(cn, part, nparts); i < span(cn, part + 1, nparts); ++i) {
                const uint32_t L = lens[base + i], cp = L < hcap ? L : hcap;
                const uint8_t *src = frames[base + i];
                uint8_t *dst = sl.h_arena + off;
                if (cp >= 64) {
                    memcpy(dst, src, 64);
                    if (cp > 64) memcpy(dst + 64, src + 64, cp - 64);
                } else {
                    memcpy(dst, src, cp);
                }
                sl.h_desc[2 * i] = (uint32_t)off;
                sl.h_desc[2 * i + 1] = L;
                off += cp ? (cp + 63) & ~63u : 64;
            }
        });
        hipStream_t s = sl.s;
        HIPCHK(c, hipMemcpyAsync(sl.d_arena, sl.h_arena, part_off[np], hipMemcpyHostToDevice, s));
        HIPCHK(c, hipMemcpyAsync(sl.d_desc, sl.h_desc, sizeof(uint32_t) * 2 * cn, hipMemcpyHostToDevice, s));
        fcgpu_out d;
        d.verdict = sl.d_v;
        d.hash = h->hash ? sl.d_h : nullptr;
        d.anno = h->anno ? sl.d_an : nullptr;
        d.perm = h->perm ? sl.d_perm : nullptr;
        d.port_start = nullptr;
        d.tile_count = h->tile_count ? sl.d_tc : nullptr;
        d.partition = h->partition;
        d.reserved = 0;
        d.tile_perm = h->tile_perm ? sl.d_tp : nullptr;
        d.flowid = nullptr;   // flow tables run the whole batch in order (process_host_whole)
        d.ip_rw = nullptr;    // so do header rewrites the caller wants back
        int rc = fcgpu_process(c, sl.d_arena, sl.d_desc, cn, &d, s);
        if (rc != FCGPU_OK) return rc;
        const uint32_t tb = base / kTile, nt = (cn + kTile - 1) / kTile;
        auto d2h = [&](void *user, bool pinned, void *stage, const void *dev, size_t bytes, size_t uoff) {
            return hipMemcpyAsync(pinned ? (uint8_t *)user + uoff : stage, dev, bytes, hipMemcpyDeviceToHost, s);
        };
        if (h->verdict) HIPCHK(c, d2h(h->verdict, pin.v, sl.h_v, sl.d_v, 2ull * cn, 2ull * base));
        if (h->hash) HIPCHK(c, d2h(h->hash, pin.h, sl.h_h, sl.d_h, 4ull * cn, 4ull * base));
        if (h->anno) HIPCHK(c, d2h(h->anno, pin.an, sl.h_an, sl.d_an, sizeof(fcgpu_anno) * cn, sizeof(fcgpu_anno) * base));
        if (h->perm) HIPCHK(c, d2h(h->perm, pin.perm, sl.h_perm, sl.d_perm, 4ull * cn, 4ull * base));
        if (h->tile_perm) HIPCHK(c, d2h(h->tile_perm, pin.tp, sl.h_tp, sl.d_tp, cn, base));
        if (h->tile_count)
            HIPCHK(c, d2h(h->tile_count, pin.tc, sl.h_tc, sl.d_tc, 2ull * nb * nt, 2ull * nb * tb));
        HIPCHK(c, hipEventRecord(sl.done, s));
        sl.busy = true;
        sl.base = base;
        sl.n = cn;
    }
    for (uint32_t k = nchunks > kSlots ? nchunks - kSlots : 0; k < nchunks; ++k) {
        HostSlot &sl = c->slot[k % kSlots];
        if (!sl.busy) continue;
        HIPCHK(c, hipEventSynchronize(sl.done));
        slot_drain(c, sl, h, pin);
    }
    return FCGPU_OK;
}

// Pools registered by fcgpu_pool_register, with the number of contexts using each.
static std::mutex g_pool_mu;
static std::map<std::pair<uint64_t, uint64_t>, uint32_t> g_pools;

void pool_release(fcgpu_ctx *c) {
    if (!c->pool_host || !c->pool_owned) return;
    std::lock_guard<std::mutex> lk(g_pool_mu);
    auto it = g_pools.find({c->pool_host, c->pool_bytes});
    if (it != g_pools.end() && --it->second == 0) {
        hipHostUnregister((void *)c->pool_host);
        (void)hipGetLastError();
        g_pools.erase(it);
    }
    c->pool_owned = false;
}

}  // namespace fcgpu_rt

extern "C" {

int fcgpu_process(fcgpu_ctx *c, const uint8_t *d_arena, const uint32_t *d_desc, uint32_t n,
                  const fcgpu_out *o, void *stream) {
    if (!c || !o) return FCGPU_EINVAL;
    int rc = check_process(c, d_arena, d_desc, n, o);
    if (rc != FCGPU_OK || n == 0) return rc;
    HIPCHK(c, hipSetDevice(c->device));
    return process_one(c, d_arena, d_desc, n, o, (hipStream_t)stream);   // NULL = the null stream
}

int fcgpu_process_counted(fcgpu_ctx *c, const uint8_t *d_arena, const uint32_t *d_desc, uint32_t n_max,
                          const uint32_t *d_count, uint32_t base, const fcgpu_out *o, void *stream) {
    if (!c || !o) return FCGPU_EINVAL;
    if (!d_count) return fail(c, FCGPU_EINVAL, "fcgpu_process_counted: null count");
    // the whole-batch partition's scan and scatter take the host's n
    if (o->partition == FCGPU_PART_GLOBAL && (o->perm || o->port_start))
        return fail(c, FCGPU_EINVAL, "fcgpu_process_counted: no whole-batch partition (FCGPU_PART_GLOBAL)");
    int rc = check_process(c, d_arena, d_desc, n_max, o);
    if (rc != FCGPU_OK || n_max == 0) return rc;
    HIPCHK(c, hipSetDevice(c->device));
    return process_one(c, d_arena, d_desc, n_max, o, (hipStream_t)stream, 0, d_count, base);
}

int fcgpu_process_jobs(fcgpu_ctx *c, const fcgpu_job *jobs, uint32_t njobs, void *stream) {
    if (!c || (njobs && !jobs)) return FCGPU_EINVAL;
    // every job is checked before any is launched: a bad job launches nothing
    bool split = false;
    for (uint32_t k = 0; k < njobs; ++k) {
        const fcgpu_job &j = jobs[k];
        int rc = check_process(c, j.arena, j.desc, j.n, &j.out);
        if (rc != FCGPU_OK) return rc;
        const bool shared = c->fl.slots || (j.out.partition == FCGPU_PART_GLOBAL && (j.out.perm || j.out.port_start));
        if ((j.stream ? j.stream : stream) != (jobs[0].stream ? jobs[0].stream : stream)) split = true;
        if (split && shared)
            return fail(c, FCGPU_EINVAL, "jobs on several streams: the flow table and the whole-batch "
                                         "partition use context scratch (one stream only)");
    }
    HIPCHK(c, hipSetDevice(c->device));
    auto eff = [&](const fcgpu_job &j) { return (hipStream_t)(j.stream ? j.stream : stream); };
    // Per stream, in order: a fusable job and the stream's next fusable jobs
    // (up to kMaxFuse, disjoint outputs, same partition shape, stopping at the
    // stream's next non-fusable job) share one launch. Jobs on other streams
    // are independent of them, so they are taken up in their own turn.
    std::vector<uint8_t> done(njobs, 0);
    std::vector<const fcgpu_job *> grp;
    grp.reserve(kMaxFuse);
    for (uint32_t k = 0; k < njobs; ++k) {
        if (done[k]) continue;
        const fcgpu_job &j = jobs[k];
        done[k] = 1;
        if (!fusable(c, j)) {
            int rc = process_one(c, j.arena, j.desc, j.n, &j.out, eff(j));
            if (rc != FCGPU_OK) return rc;
            continue;
        }
        const hipStream_t s = eff(j);
        grp.assign(1, &j);
        const size_t gmax = c->fl.slots ? kMaxFuseFlow : kMaxFuse;
        for (uint32_t m = k + 1; m < njobs && grp.size() < gmax; ++m) {
            if (done[m] || eff(jobs[m]) != s) continue;
            const fcgpu_job &x = jobs[m];
            if (!fusable(c, x)) break;                  // the stream's order barrier
            if (out_part(&x.out) != out_part(&j.out) || x.out.partition != j.out.partition) break;
            bool clash = false;
            for (const fcgpu_job *y : grp) clash = clash || outputs_overlap(x.out, y->out);
            if (clash) break;
            grp.push_back(&x);
            done[m] = 1;
        }
        int rc = grp.size() == 1 ? process_one(c, j.arena, j.desc, j.n, &j.out, s)
                                 : process_fused(c, grp.data(), (uint32_t)grp.size(), s);
        if (rc != FCGPU_OK) return rc;
    }
    return FCGPU_OK;
}

int fcgpu_process_host(fcgpu_ctx *c, const uint8_t *const *frames, const uint32_t *lens, uint32_t n,
                       const fcgpu_out *h) {
    if (!c || !h || (n && (!frames || !lens))) return FCGPU_EINVAL;
    if (n > c->max_batch) return fail(c, FCGPU_ENOMEM, "batch larger than max_batch");
    if (n == 0) return FCGPU_OK;
    if (h->partition > FCGPU_PART_TILE) return fail(c, FCGPU_EINVAL, "bad partition mode");
    HIPCHK(c, hipSetDevice(c->device));
    // a flow table assigns IDs in packet order: one pass on one stream
    if ((h->partition == FCGPU_PART_GLOBAL && (h->perm || h->port_start)) || c->fl.slots || h->ip_rw)
        return process_host_whole(c, frames, lens, n, h);
    if (h->partition == FCGPU_PART_TILE && ((h->perm || h->tile_perm) != (h->tile_count != nullptr)))
        return fail(c, FCGPU_EINVAL, "FCGPU_PART_TILE needs tile_count and perm and/or tile_perm");
    return process_host_pipelined(c, frames, lens, n, h);
}

int fcgpu_pool_register(fcgpu_ctx *c, void *base, size_t bytes) {
    if (!c || !base || bytes < 4096) return fail(c, FCGPU_EINVAL, "fcgpu_pool_register: bad pool");
    if (bytes > 0xffffffffull - kArenaPad) return fail(c, FCGPU_EINVAL, "pool larger than 4 GiB (u32 frame offsets)");
    HIPCHK(c, hipSetDevice(c->device));
    if (c->pool_host) {
        HIPCHK(c, hipDeviceSynchronize());
        pool_release(c);
        c->pool_host = c->pool_bytes = 0;
        c->pool_dev = nullptr;
    }
    // the descriptor scratch first: a failure leaves no pool registered
    if (!c->d_mptr) {
        const int rc = alloc_or_fail(c, "fcgpu_pool_register scratch",
                                     {dev_buf(c->d_mptr, sizeof(uint64_t) * c->max_batch),
                                      dev_buf(c->d_mdesc, sizeof(uint2) * c->max_batch)});
        if (rc != FCGPU_OK) return rc;
    }
    // several contexts (one per rx queue / thread) may share one pool: the
    // library pins it once and unpins it when the last of them lets go
    {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        auto it = g_pools.find({(uint64_t)base, bytes});
        if (it != g_pools.end()) {
            ++it->second;
        } else {
            hipError_t e = hipHostRegister(base, bytes, hipHostRegisterMapped);
            if (e != hipSuccess) {
                (void)hipGetLastError();
                return fail(c, FCGPU_ERUNTIME, std::string("hipHostRegister(pool): ") + hipGetErrorString(e));
            }
            g_pools[{(uint64_t)base, bytes}] = 1;
        }
    }
    c->pool_owned = true;
    c->pool_host = (uint64_t)base;
    c->pool_bytes = bytes;
    void *dev = nullptr;
    if (hipError_t e = hipHostGetDevicePointer(&dev, base, 0)) {
        (void)hipGetLastError();
        pool_release(c);                  // the registration's reference goes back
        c->pool_host = c->pool_bytes = 0;
        return fail(c, FCGPU_ERUNTIME, std::string("hipHostGetDevicePointer(pool): ") + hipGetErrorString(e));
    }
    c->pool_dev = static_cast<uint8_t *>(dev);
    return FCGPU_OK;
}

int fcgpu_process_mbufs(fcgpu_ctx *c, void *const *mbufs, uint32_t n, const fcgpu_mbuf_layout *L,
                        const fcgpu_out *o, void *stream) {
    if (!c || !o || !L || (n && !mbufs)) return FCGPU_EINVAL;
    if (!c->pool_host) return fail(c, FCGPU_EINVAL, "fcgpu_process_mbufs: no pool registered (fcgpu_pool_register)");
    if (L->header_bytes > 64 || L->buf_addr + 8 > L->header_bytes || L->data_off + 2 > L->header_bytes ||
        L->data_len + 2 > L->header_bytes || (L->buf_addr & 7) || (L->data_off & 1) || (L->data_len & 1))
        return fail(c, FCGPU_EINVAL, "bad mbuf layout (fields aligned, inside header_bytes <= 64)");
    int rc = check_process(c, c->pool_dev, reinterpret_cast<const uint32_t *>(c->d_mdesc), n, o);
    if (rc != FCGPU_OK || n == 0) return rc;
    HIPCHK(c, hipSetDevice(c->device));
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(c, hipMemcpyAsync(c->d_mptr, mbufs, sizeof(uint64_t) * n, hipMemcpyHostToDevice, s));
    MbufArgs a;
    a.ptrs = c->d_mptr;
    a.n = n;
    a.pool_host = c->pool_host;
    a.pool_bytes = c->pool_bytes;
    a.pool_dev = c->pool_dev;
    a.f_buf = L->buf_addr;
    a.f_off = L->data_off;
    a.f_len = L->data_len;
    a.hdr = L->header_bytes;
    a.desc = c->d_mdesc;
    hipLaunchKernelGGL(k_mbuf_desc, dim3((n + 255) / 256), dim3(256), 0, s, a);
    HIPCHK(c, hipGetLastError());
    return process_one(c, c->pool_dev, reinterpret_cast<const uint32_t *>(c->d_mdesc), n, o, s);
}

}  // extern "C"
