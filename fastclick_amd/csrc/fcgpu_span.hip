// fcgpu_span.hip -- host-resident batches a caller stages itself, handed
// over asynchronously: spans (fcgpu_span_submit) and blocks
// (fcgpu_span_submit_block, the GPUIPCheckClassify element's path) in
// FCGPU_SPAN_SLOTS slots per context, copied or read in place (zero-copy), and
// in FCGPU_SPAN_AUTO mode with many contexts on one device, the device's
// shared zero-copy queue that carries several contexts' blocks in one k_rx
// launch.
#include "fcgpu_internal.hh"

using namespace fcgpu;
using namespace fcgpu_rt;

namespace fcgpu_rt {

static void agg_release(int device);
// FCGPU_SPAN_AUTO: contexts per device in that mode; block submissions go
// zero-copy while at least kZeroCopyAuto of them exist (one or two threads
// submit few enough copies for the copy engine, and copies are faster there:
// profiles/r03_s8/el_zc.log)
constexpr uint32_t kZeroCopyAuto = 4;
constexpr int kMaxDevices = 64;
static std::atomic<uint32_t> g_auto_n[kMaxDevices];   // AUTO contexts per device (read on every submission)
void span_auto_count(fcgpu_ctx *c, uint32_t new_mode) {
    const bool was = c->span_mode == FCGPU_SPAN_AUTO, now = new_mode == FCGPU_SPAN_AUTO;
    if (was == now || c->device < 0 || c->device >= kMaxDevices) return;
    if (now) {
        g_auto_n[c->device].fetch_add(1, std::memory_order_relaxed);
    } else if (g_auto_n[c->device].fetch_sub(1, std::memory_order_acq_rel) == 1) {
        agg_release(c->device);
    }
}
bool span_zerocopy(const fcgpu_ctx *c) {
    if (c->span_mode != FCGPU_SPAN_AUTO) return c->span_mode == FCGPU_SPAN_ZEROCOPY;
    return c->device >= 0 && c->device < kMaxDevices &&
           g_auto_n[c->device].load(std::memory_order_relaxed) >= kZeroCopyAuto;
}

// ---- the shared zero-copy queue of FCGPU_SPAN_AUTO --------------------------
// With many element contexts on one device, each zero-copy batch is a small
// kernel (16-64 workgroups, latency-bound over PCIe) that waits behind other
// contexts' kernels in the few HW queues their streams map to (4 on the box:
// the HW queues ran ~2 kernels at a time, profiles/r03_s10/kt_el16). So in
// AUTO mode, once kZeroCopyAuto contexts share the device, block submissions
// go to one queue per device, and a submitter that finds kAggLaunch of them
// pending -- or a context waiting for one of its own still pending --
// launches them together: one k_rx launch carries the batches of several
// contexts with one configuration (RxJob::ctr keeps each context's counters),
// on one of kAggStreams streams. Flow tables (batch order), whole-batch
// partitions and in-place rewrites (context scratch) keep their own launches.
struct AggItem {
    fcgpu_ctx *c;
    uint32_t slot;
    fcgpu_job job;            // device (mapped) addresses
    uint32_t layout;          // kLay* bits of job's descriptors and annotations
    // the launch inputs, taken on the owner's thread at submit time: the
    // launch may happen on another context's thread, later
    DevCfg dcfg;
    uint32_t cm;              // k_rx check mode / checksum as launch_rx_part normalises them
    bool ck;
    unsigned long long *ctr;  // the counter vector in use at submit
    hipFunction_t fn;         // the compiled program's k_rx (nullptr: the built-in kernel)
    uint64_t prog_key;        // the program's contents (dcfg.prog is this context's copy of it)
};
// the queue's launch streams: HIP maps a process's streams onto
// GPU_MAX_HW_QUEUES hardware queues (4 by default). FCGPU_AGG_STREAMS=1..8
// changes the count (same-box A/B with GPU_MAX_HW_QUEUES)
constexpr uint32_t kAggStreams = 4, kAggStreamsMax = 8;
struct AggQueue {
    std::mutex mu;
    int device = -1;
    std::vector<AggItem> pending;
    hipStream_t st[kAggStreamsMax] = {};   // created by agg_issue (st_mu), never under mu
    uint32_t nst = kAggStreams;
    uint32_t take_at = 4;     // pending submissions that trigger a launch (kAggLaunch, FCGPU_AGG_LAUNCH)
    std::mutex st_mu;
    uint32_t rr = 0;
    std::vector<AggLaunch *> spare;
    // owners whose launch is still being issued by another thread sleep
    // here (agg_finish); agg_issue wakes them
    std::condition_variable cv;
};
constexpr uint32_t kAggLaunch = 4;    // default of AggQueue::take_at
static std::mutex g_agg_mu;
static std::map<int, AggQueue *> g_agg;
static AggQueue &agg_queue(fcgpu_ctx *c) {
    if (c->aq) return *c->aq;
    std::lock_guard<std::mutex> g(g_agg_mu);
    AggQueue *&q = g_agg[c->device];
    if (!q) {
        q = new AggQueue();
        q->device = c->device;
        if (const char *e = getenv("FCGPU_AGG_STREAMS")) {
            const int v = atoi(e);
            if (v >= 1 && v <= (int)kAggStreamsMax) q->nst = (uint32_t)v;
        }
        q->take_at = kAggLaunch;
        if (const char *e = getenv("FCGPU_AGG_LAUNCH")) {     // same-box A/B
            const int v = atoi(e);
            if (v >= 1 && v <= (int)kMaxFuse) q->take_at = (uint32_t)v;
        }
    }
    c->aq = q;
    return *q;
}
static bool agg_eligible(const fcgpu_ctx *c, const fcgpu_out &o) {
    return c->span_mode == FCGPU_SPAN_AUTO && !c->fl.slots && out_part(&o) != kPartGlobal &&
           !(c->cfg.rewrite & FCGPU_RW_INPLACE) && !c->timing_every;
}
// One launch takes its configuration from its first item: the others must
// have the same one (everything agg_take_locked reads from it).
// Device copies of equal contents (the program, the CRC tables) do not
// matter: the launch reads the first item's, which its owner keeps until
// its own wait (and fcgpu_set_program synchronises before freeing one).
static bool agg_compatible(const AggItem &a, const AggItem &b) {
    DevCfg x = a.dcfg, y = b.dcfg;
    x.prog = y.prog = nullptr;
    x.crc_tab = y.crc_tab = nullptr;
    x.lb_tab = y.lb_tab = nullptr;
    return memcmp(&x, &y, sizeof(DevCfg)) == 0 && a.prog_key == b.prog_key &&
           (a.dcfg.crc_tab != nullptr) == (b.dcfg.crc_tab != nullptr) && a.cm == b.cm && a.ck == b.ck &&
           (a.fn != nullptr) == (b.fn != nullptr) && out_part(&a.job.out) == out_part(&b.job.out) &&
           a.job.out.partition == b.job.out.partition;
}
// A context with a queued submission keeps the configuration, program and
// compiled module that submission was taken with (fcgpu_configure,
// fcgpu_set_program and fcgpu_program_jit refuse until it is waited for).
bool agg_queued(const fcgpu_ctx *c) {
    for (const SpanSlot &sp : c->span)
        if (sp.busy && sp.agg) return true;
    return false;
}
// A group of pending submissions taken from the queue, to be issued by the
// thread that took it, outside the queue's lock (a kernel launch from 16
// threads contending for the lock serialised their submissions).
struct AggIssue {
    RxLaunch L;
    int part;
    uint32_t cm, tiles;
    bool ck;
    hipFunction_t fn;
    uint32_t si;              // the queue stream it goes on
    AggLaunch *al;
};
// Take every pending submission (q.mu held) as launches: the first one with
// the next ones of its configuration, up to kMaxFuse per launch, until none
// is left. Each taken submission's slot points at its launch (state
// kAggIssuing) before the lock is released.
static void agg_take_locked(AggQueue &q, std::vector<AggIssue> &out) {
    while (!q.pending.empty()) {
        std::vector<size_t> grp{0};
        for (size_t m = 1; m < q.pending.size() && grp.size() < kMaxFuse; ++m)
            if (agg_compatible(q.pending[0], q.pending[m])) grp.push_back(m);
        const AggItem &i0 = q.pending[0];
        out.emplace_back();
        AggIssue &is = out.back();
        is.part = out_part(&i0.job.out);
        is.cm = i0.cm;
        is.ck = i0.ck;
        is.fn = i0.fn;
        RxLaunch &L = is.L;
        RxArgs &a = L.A;
        a = RxArgs{};    // no whole-batch partition or flow table here (agg_eligible)
        a.cfg = i0.dcfg;
        L.njobs = (uint32_t)grp.size();
        L.flow_stride = L.flow_words = 0;
        uint32_t tiles = 0;
        for (size_t k = 0; k < grp.size(); ++k) {
            const AggItem &it = q.pending[grp[k]];
            const fcgpu_job &j = it.job;
            RxJob &J = L.job[k];
            J = RxJob{};
            J.arena = j.arena;
            J.desc = reinterpret_cast<const uint2 *>(j.desc);
            J.verdict = j.out.verdict;
            J.hash = j.out.hash;
            J.anno = j.out.anno;
            J.perm = j.out.perm;
            J.tile_count = j.out.tile_count;
            J.tile_perm = j.out.partition == FCGPU_PART_TILE ? j.out.tile_perm : nullptr;
            J.flowid = nullptr;
            J.ip_rw = j.out.ip_rw;
            J.ctr = it.ctr;
            J.n = j.n;
            J.tile0 = tiles;
            J.layout = it.layout;
            tiles += (j.n + kTile - 1) / kTile;
        }
        is.tiles = tiles;
        L.job_tiles = (L.job[0].n + kTile - 1) / kTile;
        for (uint32_t k = 1; k < L.njobs; ++k)
            if (L.job[k].tile0 != k * L.job_tiles) L.job_tiles = 0;
        if (tiles > L.njobs * L.job_tiles) L.job_tiles = 0;
        // the first batch also fills A: a launch of one batch reads A alone
        const RxJob &J0 = L.job[0];
        a.arena = J0.arena;
        a.desc = J0.desc;
        a.n = J0.n;
        a.ntiles = (a.n + kTile - 1) / kTile;
        a.verdict = J0.verdict;
        a.hash = J0.hash;
        a.anno = J0.anno;
        a.perm = J0.perm;
        a.tile_count = J0.tile_count;
        a.tile_perm = J0.tile_perm;
        a.ip_rw = J0.ip_rw;
        a.ctr = J0.ctr;
        a.layout = J0.layout;
        // no HIP call under the queue's lock: the stream and a new launch's
        // event are created by the issuing thread (agg_issue)
        is.si = q.rr++ % q.nst;
        AggLaunch *al = nullptr;
        if (!q.spare.empty()) {
            al = q.spare.back();
            q.spare.pop_back();
        } else {
            al = new AggLaunch();
        }
        al->state.store(kAggIssuing, std::memory_order_relaxed);
        al->phase.store(kAggPhaseTaken, std::memory_order_relaxed);
        al->refs = (uint32_t)grp.size();
        is.al = al;
        for (size_t k : grp) {
            AggItem &it = q.pending[k];
            it.c->span[it.slot].al = al;
        }
        // the taken submissions leave the queue, the rest keep their order
        std::vector<AggItem> rest;
        rest.reserve(q.pending.size() - grp.size());
        size_t g = 0;
        for (size_t m = 0; m < q.pending.size(); ++m) {
            if (g < grp.size() && grp[g] == m) { ++g; continue; }
            rest.push_back(q.pending[m]);
        }
        q.pending.swap(rest);
    }
}
// Issue taken launches (no lock held); their owners' waits see the outcome.
// Nothing here waits for anything: a launch, one event record per group.
static void agg_issue(AggQueue &q, std::vector<AggIssue> &iss) {
    if (iss.empty()) return;
    const bool dev_ok = hipSetDevice(q.device) == hipSuccess;
    for (AggIssue &is : iss) {
        hipStream_t st = nullptr;
        if (dev_ok) {
            std::lock_guard<std::mutex> g(q.st_mu);
            if (!q.st[is.si] && hipStreamCreateWithFlags(&q.st[is.si], hipStreamNonBlocking) != hipSuccess) {
                (void)hipGetLastError();
                q.st[is.si] = nullptr;
            }
            st = q.st[is.si];
        }
        if (dev_ok && !is.al->ev && hipEventCreateWithFlags(&is.al->ev, hipEventDisableTiming) != hipSuccess) {
            (void)hipGetLastError();
            is.al->ev = nullptr;
        }
        hipError_t e = dev_ok && st && is.al->ev ? hipSuccess : hipErrorInvalidValue;
        if (e == hipSuccess && fault_take(FCGPU_FAULT_LAUNCH)) e = hipErrorLaunchFailure;
        is.al->phase.store(kAggPhaseLaunch, std::memory_order_relaxed);
        if (e == hipSuccess) {
            if (is.fn) {
                e = launch_rx_fn(is.fn, is.part, is.L, is.tiles, st);
            } else {
                e = launch_rx_any(is.part, is.cm, is.ck, is.L, is.tiles, st, nullptr, nullptr, nullptr);
                if (e == hipSuccess) e = hipGetLastError();
            }
        }
        is.al->phase.store(kAggPhaseRecord, std::memory_order_relaxed);
        if (e == hipSuccess) e = hipEventRecord(is.al->ev, st);
        if (e != hipSuccess) (void)hipGetLastError();
        is.al->state.store(e == hipSuccess ? kAggIssued : kAggFailed, std::memory_order_release);
    }
    iss.clear();
    {   // an owner that found its launch still being issued is asleep in
        // agg_finish: taking the lock orders this wake-up after its check
        std::lock_guard<std::mutex> g(q.mu);
    }
    q.cv.notify_all();
}
// The last AUTO context of a device is gone: every submission it queued was
// waited for (fcgpu_close / fcgpu_span_mode wait or refuse busy slots), so
// the queue's streams and events are idle and go.
static void agg_release(int device) {
    AggQueue *q = nullptr;
    {
        std::lock_guard<std::mutex> g(g_agg_mu);
        auto it = g_agg.find(device);
        if (it == g_agg.end()) return;
        q = it->second;
    }
    std::lock_guard<std::mutex> g(q->mu);
    std::lock_guard<std::mutex> g2(q->st_mu);
    if (!q->pending.empty()) return;
    for (AggLaunch *al : q->spare) {
        if (al->ev) hipEventDestroy(al->ev);
        delete al;
    }
    q->spare.clear();
    for (hipStream_t &st : q->st)
        if (st) {
            hipStreamDestroy(st);
            st = nullptr;
        }
}

// Queue one zero-copy block submission (device addresses in j). Once queued
// the submission is the owner's to wait for: a failed launch (of its group or
// another) is reported by that wait (AggLaunch::state), never by this call.
static int agg_submit(fcgpu_ctx *c, uint32_t slot, const fcgpu_job &j, uint32_t layout) {
    AggItem it{};
    it.c = c;
    it.slot = slot;
    it.job = j;
    it.layout = layout;
    it.dcfg = c->dcfg;
    it.cm = c->cfg.check_mode;
    it.ck = c->cfg.checksum != 0;
    if (it.cm == FCGPU_MARK_IP4 || it.cm == FCGPU_MARK_IP6) it.ck = false;
    it.ctr = c->d_ctr;
    it.fn = nullptr;
    it.prog_key = c->cfg.classify == FCGPU_CLS_PROGRAM ? c->prog_key
                : c->cfg.classify == FCGPU_CLS_LB_TABLE ? c->lbtab_key : 0;
    if (c->cfg.classify == FCGPU_CLS_PROGRAM && !c->jit_src.empty()) {
        const bool ip4 = it.cm == FCGPU_CHECK_IP4 || it.cm == FCGPU_MARK_IP4;
        it.fn = jit_function(c, jit_key((int)it.cm, it.ck, out_part(&j.out), ip4 && c->cfg.l4_mode != FCGPU_L4_NONE,
                                        false));
    }
    AggQueue &q = agg_queue(c);
    SpanSlot &sp = c->span[slot];
    std::vector<AggIssue> iss;
    {
        std::lock_guard<std::mutex> g(q.mu);
        q.pending.push_back(it);
        sp.agg = true;
        sp.al = nullptr;
        sp.busy = true;
        if (q.pending.size() >= q.take_at) agg_take_locked(q, iss);
    }
    agg_issue(q, iss);
    return FCGPU_OK;
}
// Wait for (block = true) or poll a queued submission: launched first if
// still pending. Returns 1 done, 0 running, < 0 error.
static int agg_finish(fcgpu_ctx *c, uint32_t slot, bool block) {
    AggQueue &q = agg_queue(c);
    SpanSlot &sp = c->span[slot];
    AggLaunch *al = nullptr;
    std::vector<AggIssue> iss;
    {
        std::lock_guard<std::mutex> g(q.mu);
        if (!sp.al) agg_take_locked(q, iss);     // still pending: it (and every other) goes now
        al = sp.al;
    }
    agg_issue(q, iss);
    // the thread that took its group issues it outside the lock: sleep until
    // it has (a yield loop here kept up to 15 owner threads spinning on the
    // CPUs the issuing thread needed). Issuing never waits for anything, so
    // a launch still not issued after seconds means a stall inside the HIP
    // runtime on that thread: reported (stderr) every 5 s, with where it is
    int st = al->state.load(std::memory_order_acquire);
    if (st == kAggIssuing) {
        if (!block) return 0;
        std::unique_lock<std::mutex> lk(q.mu);
        uint32_t waited_s = 0;
        while ((st = al->state.load(std::memory_order_acquire)) == kAggIssuing) {
            if (q.cv.wait_for(lk, std::chrono::seconds(5)) == std::cv_status::timeout &&
                al->state.load(std::memory_order_acquire) == kAggIssuing) {
                waited_s += 5;
                static const char *const where[] = {"taken, not yet launched", "in its k_rx launch",
                                                    "recording its completion event"};
                fprintf(stderr, "fcgpu: shared-queue launch not issued after %u s: the issuing thread is %s\n",
                        waited_s, where[al->phase.load(std::memory_order_relaxed) % 3]);
            }
        }
    }
    hipError_t e = hipSuccess;
    if (st == kAggIssued) {
        e = block ? hipEventSynchronize(al->ev) : hipEventQuery(al->ev);
        if (!block && e == hipErrorNotReady) return 0;
    }
    {
        std::lock_guard<std::mutex> g(q.mu);
        if (--al->refs == 0) q.spare.push_back(al);
        sp.al = nullptr;
        sp.agg = false;
        sp.busy = false;
    }
    if (st == kAggFailed) return fail(c, FCGPU_ERUNTIME, "shared zero-copy launch failed");
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return fail(c, FCGPU_ERUNTIME, std::string("shared zero-copy batch: ") + hipGetErrorString(e));
    }
    return 1;
}

}  // namespace fcgpu_rt

extern "C" {

int fcgpu_span_submit(fcgpu_ctx *c, uint32_t slot, const uint8_t *h_span, size_t bytes, const uint32_t *h_desc,
                      uint32_t n, const fcgpu_out *h) {
    if (!c || !h || slot >= FCGPU_SPAN_SLOTS || (n && (!h_span || !h_desc))) return FCGPU_EINVAL;
    if (n > c->max_batch) return fail(c, FCGPU_ENOMEM, "batch larger than max_batch");
    if (bytes > 0xffffffffull - kArenaPad) return fail(c, FCGPU_EINVAL, "span larger than 4 GiB");
    SpanSlot &sp = c->span[slot];
    if (sp.busy) return fail(c, FCGPU_EINVAL, "span slot busy: fcgpu_span_wait it first");
    if (fault_take(FCGPU_FAULT_SUBMIT)) return fail(c, FCGPU_ERUNTIME, "injected fault: submission failed");
    if (fault_take(FCGPU_FAULT_WAIT)) {
        sp.doomed = sp.busy = true;
        return FCGPU_OK;
    }
    HIPCHK(c, hipSetDevice(c->device));
    if (!sp.d_desc) {                     // all or nothing
        const size_t m = c->max_batch, tiles = (m + kTile - 1) / kTile;
        const int rc = alloc_or_fail(c, "span slot outputs",
                                     {dev_buf(sp.d_desc, sizeof(uint32_t) * 2 * m), dev_buf(sp.d_v, sizeof(uint16_t) * m),
                                      dev_buf(sp.d_h, sizeof(uint32_t) * m), dev_buf(sp.d_an, sizeof(fcgpu_anno) * m),
                                      dev_buf(sp.d_perm, sizeof(uint32_t) * m),
                                      dev_buf(sp.d_start, sizeof(uint32_t) * (FCGPU_MAX_PORTS + 2)),
                                      dev_buf(sp.d_tp, m + kTile),
                                      dev_buf(sp.d_tc, sizeof(uint16_t) * (FCGPU_MAX_PORTS + 1) * tiles),
                                      dev_buf(sp.d_fl, sizeof(uint32_t) * m), dev_buf(sp.d_rw, sizeof(uint32_t) * m)});
        if (rc != FCGPU_OK) return rc;
    }
    if (!sp.own) HIPCHK(c, hipStreamCreateWithFlags(&sp.own, hipStreamNonBlocking));
    const bool zc = span_zerocopy(c);
    if (!zc && bytes + kArenaPad > sp.span_cap) {
        HIPCHK(c, hipStreamSynchronize(sp.own));
        hipFree(sp.d_span);
        sp.d_span = nullptr;
        sp.span_cap = 0;
        const size_t cap = (bytes + kArenaPad + (1u << 20) - 1) & ~(size_t)((1u << 20) - 1);
        const int rc = alloc_or_fail(c, "span block", {dev_buf(sp.d_span, cap, true)});
        if (rc != FCGPU_OK) return rc;
        sp.span_cap = cap;
    }
    // a flow table assigns IDs in batch order: every slot then runs on the
    // context's stream
    if (c->fl.slots && !c->stream) HIPCHK(c, hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    sp.s = c->fl.slots ? c->stream : sp.own;
    hipStream_t s = sp.s;
    if (n == 0) return FCGPU_OK;
    if (zc) {
        // in place: the kernels read the caller's page-locked span and
        // descriptors and write its page-locked output arrays over PCIe
        int k = 0;
        auto dev = [&](const void *p, const char *what, void **out) -> int {
            const int slot_k = k++;
            *out = nullptr;
            if (!p) return FCGPU_OK;
            if (p == sp.zc_key[slot_k]) {        // the caller's buffers are usually reused
                *out = sp.zc_val[slot_k];
                return FCGPU_OK;
            }
            sp.zc_key[slot_k] = nullptr;
            if (hipHostGetDevicePointer(out, const_cast<void *>(p), 0) != hipSuccess || !*out) {
                (void)hipGetLastError();
                return fail(c, FCGPU_EINVAL, std::string("zero-copy span: ") + what +
                                                 " is not page-locked host memory (fcgpu_host_alloc / fcgpu_host_register)");
            }
            sp.zc_key[slot_k] = p;
            sp.zc_val[slot_k] = *out;
            return FCGPU_OK;
        };
        void *dspan, *ddesc;
        fcgpu_out d{};
        d.partition = h->partition;
        int rc;
        if ((rc = dev(h_span, "h_span", &dspan)) || (rc = dev(h_desc, "h_desc", &ddesc)) ||
            (rc = dev(h->verdict, "verdict", (void **)&d.verdict)) || (rc = dev(h->hash, "hash", (void **)&d.hash)) ||
            (rc = dev(h->anno, "anno", (void **)&d.anno)) || (rc = dev(h->perm, "perm", (void **)&d.perm)) ||
            (rc = dev(h->port_start, "port_start", (void **)&d.port_start)) ||
            (rc = dev(h->tile_count, "tile_count", (void **)&d.tile_count)) ||
            (rc = dev(h->tile_perm, "tile_perm", (void **)&d.tile_perm)) ||
            (rc = dev(h->flowid, "flowid", (void **)&d.flowid)) || (rc = dev(h->ip_rw, "ip_rw", (void **)&d.ip_rw)))
            return rc;
        rc = fcgpu_process(c, static_cast<const uint8_t *>(dspan), static_cast<const uint32_t *>(ddesc), n, &d, s);
        if (rc != FCGPU_OK) return rc;
        sp.evt = false;
        sp.busy = true;
        return FCGPU_OK;
    }
    HIPCHK(c, hipMemcpyAsync(sp.d_span, h_span, bytes, hipMemcpyHostToDevice, s));
    HIPCHK(c, hipMemcpyAsync(sp.d_desc, h_desc, sizeof(uint32_t) * 2 * n, hipMemcpyHostToDevice, s));
    fcgpu_out d{};
    d.verdict = h->verdict ? sp.d_v : nullptr;
    d.hash = h->hash ? sp.d_h : nullptr;
    d.anno = h->anno ? sp.d_an : nullptr;
    d.perm = h->perm ? sp.d_perm : nullptr;
    d.port_start = h->port_start ? sp.d_start : nullptr;
    d.tile_count = h->tile_count ? sp.d_tc : nullptr;
    d.partition = h->partition;
    d.tile_perm = h->tile_perm ? sp.d_tp : nullptr;
    d.flowid = h->flowid ? sp.d_fl : nullptr;
    d.ip_rw = h->ip_rw ? sp.d_rw : nullptr;
    int rc = fcgpu_process(c, sp.d_span, sp.d_desc, n, &d, s);
    if (rc != FCGPU_OK) return rc;
    auto back = [&](void *dst, const void *src, size_t b) -> int {
        if (dst) HIPCHK(c, hipMemcpyAsync(dst, src, b, hipMemcpyDeviceToHost, s));
        return FCGPU_OK;
    };
    const size_t tiles = (n + kTile - 1) / kTile;
    if ((rc = back(h->verdict, sp.d_v, sizeof(uint16_t) * n)) || (rc = back(h->hash, sp.d_h, sizeof(uint32_t) * n)) ||
        (rc = back(h->anno, sp.d_an, sizeof(fcgpu_anno) * n)) || (rc = back(h->perm, sp.d_perm, sizeof(uint32_t) * n)) ||
        (rc = back(h->port_start, sp.d_start, sizeof(uint32_t) * (c->cfg.nports + 2))) ||
        (rc = back(h->tile_count, sp.d_tc, sizeof(uint16_t) * (c->cfg.nports + 1) * tiles)) ||
        (rc = back(h->tile_perm, sp.d_tp, n)) || (rc = back(h->flowid, sp.d_fl, sizeof(uint32_t) * n)) ||
        (rc = back(h->ip_rw, sp.d_rw, sizeof(uint32_t) * n)))
        return rc;
    sp.evt = false;
    sp.busy = true;
    return FCGPU_OK;
}

int fcgpu_span_zerocopy_active(const fcgpu_ctx *c) { return c && span_zerocopy(c) ? 1 : 0; }

int fcgpu_span_mode(fcgpu_ctx *c, uint32_t mode) {
    if (!c || mode > FCGPU_SPAN_AUTO) return FCGPU_EINVAL;
    for (const SpanSlot &sp : c->span)
        if (sp.busy) return fail(c, FCGPU_EINVAL, "fcgpu_span_mode: a span slot is in flight");
    span_auto_count(c, mode);
    c->span_mode = mode;
    for (SpanSlot &sp : c->span) {      // forget the zero-copy address translations
        sp.zc_hin = sp.zc_hout = nullptr;
        for (auto &k : sp.zc_key) k = nullptr;
    }
    return FCGPU_OK;
}

int fcgpu_span_poll(fcgpu_ctx *c, uint32_t slot) {
    if (!c || slot >= FCGPU_SPAN_SLOTS) return FCGPU_EINVAL;
    SpanSlot &sp = c->span[slot];
    if (!sp.busy) return 1;
    if (sp.doomed) {
        sp.doomed = sp.busy = false;
        return fail(c, FCGPU_ERUNTIME, "injected fault: batch failed on the device");
    }
    if (sp.agg) return agg_finish(c, slot, false);
    const hipError_t e = sp.evt ? hipEventQuery(sp.done) : hipStreamQuery(sp.s);
    if (e == hipSuccess) return 1;
    if (e == hipErrorNotReady) return 0;
    return fail(c, FCGPU_ERUNTIME, std::string("hipStreamQuery: ") + hipGetErrorString(e));
}

int fcgpu_block_layout_for(const fcgpu_ctx *c, uint32_t n, uint32_t outputs, uint32_t partition, fcgpu_block_layout *L) {
    if (!c || !L || partition > FCGPU_PART_TILE) return FCGPU_EINVAL;
    const size_t nb = c->cfg.nports + 1, tiles = (n + kTile - 1) / kTile;
    size_t off = 0;
    auto put = [&](size_t &field, uint32_t bit, size_t bytes) {
        field = FCGPU_OUT_ABSENT;
        if (!(outputs & bit)) return;
        off = (off + 255) & ~(size_t)255;
        field = off;
        off += bytes;
    };
    put(L->verdict, FCGPU_OUT_VERDICT, 2ull * n);
    put(L->hash, FCGPU_OUT_HASH, 4ull * n);
    if (outputs & FCGPU_OUT_ANNO8) put(L->anno, FCGPU_OUT_ANNO8, sizeof(fcgpu_anno8) * n);
    else put(L->anno, FCGPU_OUT_ANNO, sizeof(fcgpu_anno) * n);
    put(L->perm, FCGPU_OUT_PERM, 4ull * n);
    put(L->port_start, FCGPU_OUT_PORT_START, 4ull * (FCGPU_MAX_PORTS + 2));
    put(L->tile_count, FCGPU_OUT_TILE_COUNT, 2ull * nb * tiles);
    put(L->tile_perm, FCGPU_OUT_TILE_PERM, (size_t)n);
    put(L->flowid, FCGPU_OUT_FLOWID, 4ull * n);
    put(L->ip_rw, FCGPU_OUT_IP_RW, 4ull * n);
    L->bytes = (off + 255) & ~(size_t)255;
    return FCGPU_OK;
}

// The stream a span slot's copies and kernels go on. FCGPU_SPAN_STREAMS
// (read once): "slot" (default) -- a stream per slot; "ctx" -- one per
// context (its slots share it); "shared:N" -- N streams per device shared by
// every context of the process, slot k of the i-th context on stream
// (2i + k) mod N. Fewer streams are fewer hardware (compute and SDMA) queues
// for the runtime to map; the context's own work still completes in order.
static std::mutex g_span_mu;
static std::map<int, std::vector<hipStream_t>> g_span_shared;
static uint32_t g_span_ctx_seq = 0;
static int span_stream_mode(uint32_t &nshared) {
    struct Mode {
        int mode = 0;
        uint32_t ns = 0;
    };
    static const Mode m = [] {      // initialised once, thread-safe
        Mode r;
        const char *e = getenv("FCGPU_SPAN_STREAMS");
        if (e && !strcmp(e, "ctx")) r.mode = 1;
        else if (e && !strncmp(e, "shared:", 7)) {
            const long v = atol(e + 7);
            if (v >= 1 && v <= 64) { r.mode = 2; r.ns = (uint32_t)v; }
        }
        return r;
    }();
    nshared = m.ns;
    return m.mode;
}
static hipError_t span_stream(fcgpu_ctx *c, uint32_t slot, hipStream_t *out) {
    uint32_t ns = 0;
    const int mode = span_stream_mode(ns);
    SpanSlot &sp = c->span[slot];
    if (mode == 0 || (mode == 1 && slot == 0)) {
        if (!sp.own) {
            hipError_t e = hipStreamCreateWithFlags(&sp.own, hipStreamNonBlocking);
            if (e != hipSuccess) return e;
        }
        *out = sp.own;
        return hipSuccess;
    }
    if (mode == 1) return span_stream(c, 0, out);
    std::lock_guard<std::mutex> g(g_span_mu);
    if (c->span_index < 0) c->span_index = (int)g_span_ctx_seq++;
    auto &pool = g_span_shared[c->device];
    while (pool.size() < ns) {
        hipStream_t st = nullptr;
        hipError_t e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
        if (e != hipSuccess) return e;
        pool.push_back(st);
    }
    *out = pool[((uint32_t)c->span_index * FCGPU_SPAN_SLOTS + slot) % ns];
    return hipSuccess;
}

// Slot `slot`'s device blocks for block submissions through copies: an
// input block of in_bytes (padded for the header-window over-read, zeroed)
// and a result block for a full batch with these outputs. Replacing smaller
// ones waits for the slot's stream first. Setup work: fcgpu_span_reserve runs
// it for every slot; a submission only when no reservation was made.
static int span_blocks(fcgpu_ctx *c, uint32_t slot, hipStream_t ss, size_t in_bytes, uint32_t outputs,
                       uint32_t partition) {
    SpanSlot &sp = c->span[slot];
    fcgpu_block_layout M;    // room for a full batch with these outputs
    if (fcgpu_block_layout_for(c, c->max_batch, outputs, partition, &M) != FCGPU_OK)
        return fail(c, FCGPU_EINVAL, "bad block layout");
    if (in_bytes + kArenaPad > sp.in_cap) {
        HIPCHK(c, hipStreamSynchronize(ss));
        hipFree(sp.d_in);
        sp.d_in = nullptr;
        sp.in_cap = 0;
        const size_t cap = (in_bytes + kArenaPad + (1u << 20) - 1) & ~(size_t)((1u << 20) - 1);
        const int rc = alloc_or_fail(c, "span input block", {dev_buf(sp.d_in, cap, true)});
        if (rc != FCGPU_OK) return rc;
        sp.in_cap = cap;
    }
    if (M.bytes > sp.res_cap) {
        HIPCHK(c, hipStreamSynchronize(ss));
        hipFree(sp.d_res);
        sp.d_res = nullptr;
        sp.res_cap = 0;
        const int rc = alloc_or_fail(c, "span result block", {dev_buf(sp.d_res, M.bytes)});
        if (rc != FCGPU_OK) return rc;
        sp.res_cap = M.bytes;
    }
    return FCGPU_OK;
}

int fcgpu_span_reserve(fcgpu_ctx *c, size_t in_bytes, uint32_t outputs, uint32_t partition) {
    if (!c || partition > FCGPU_PART_TILE) return FCGPU_EINVAL;
    outputs &= ~(FCGPU_SUBMIT_COPY | FCGPU_SUBMIT_DESC32);
    if (in_bytes > 0xffffffffull - kArenaPad) return fail(c, FCGPU_EINVAL, "reservation larger than 4 GiB");
    for (const SpanSlot &sp : c->span)
        if (sp.busy) return fail(c, FCGPU_EINVAL, "fcgpu_span_reserve: a span slot is in flight");
    HIPCHK(c, hipSetDevice(c->device));
    for (uint32_t k = 0; k < FCGPU_SPAN_SLOTS; ++k) {
        hipStream_t ss = nullptr;
        HIPCHK(c, span_stream(c, k, &ss));
        int rc = span_blocks(c, k, ss, in_bytes, outputs, partition);
        if (rc != FCGPU_OK) return rc;
        c->span[k].reserved = true;
    }
    if (c->fl.slots && !c->stream) HIPCHK(c, hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    return FCGPU_OK;
}

int fcgpu_span_submit_block(fcgpu_ctx *c, uint32_t slot, const void *h_in, size_t in_bytes, size_t desc_off,
                            size_t frames_off, uint32_t n, void *h_out, uint32_t outputs, uint32_t partition) {
    if (!c || slot >= FCGPU_SPAN_SLOTS || (n && (!h_in || !h_out))) return FCGPU_EINVAL;
    const bool force_copy = (outputs & FCGPU_SUBMIT_COPY) != 0;
    const bool desc32 = (outputs & FCGPU_SUBMIT_DESC32) != 0;
    outputs &= ~(FCGPU_SUBMIT_COPY | FCGPU_SUBMIT_DESC32);
    if (n > c->max_batch) return fail(c, FCGPU_ENOMEM, "batch larger than max_batch");
    const size_t dsz = desc32 ? 4 : 8;
    if (desc_off + dsz * n > in_bytes || frames_off > in_bytes || (desc_off & (dsz - 1)))
        return fail(c, FCGPU_EINVAL, "block: descriptors (aligned to their size) or frames outside in_bytes");
    // the kernels read the descriptors and store the annotations in the layout
    // these bits name (RxJob::layout), never through tagged pointers
    const uint32_t layout = (desc32 ? kLayDesc32 : 0u) | ((outputs & FCGPU_OUT_ANNO8) ? kLayAnno8 : 0u);
    auto descp = [desc_off](uint8_t *base) { return reinterpret_cast<const uint32_t *>(base + desc_off); };
    if (in_bytes - frames_off > 0xffffffffull - kArenaPad) return fail(c, FCGPU_EINVAL, "frames larger than 4 GiB");
    SpanSlot &sp = c->span[slot];
    if (sp.busy) return fail(c, FCGPU_EINVAL, "span slot busy: fcgpu_span_wait it first");
    if (fault_take(FCGPU_FAULT_SUBMIT)) return fail(c, FCGPU_ERUNTIME, "injected fault: submission failed");
    if (fault_take(FCGPU_FAULT_WAIT)) {
        sp.doomed = sp.busy = true;
        return FCGPU_OK;
    }
    if (outputs & FCGPU_OUT_ANNO8) {
        const bool ip4 = c->cfg.check_mode == FCGPU_CHECK_IP4 || c->cfg.check_mode == FCGPU_MARK_IP4;
        if ((outputs & FCGPU_OUT_ANNO) || !ip4 || c->cfg.offset > 255)
            return fail(c, FCGPU_EINVAL, "FCGPU_OUT_ANNO8: IPv4 check modes with OFFSET < 256, without FCGPU_OUT_ANNO");
    }
    fcgpu_block_layout L;
    if (fcgpu_block_layout_for(c, n, outputs, partition, &L) != FCGPU_OK) return fail(c, FCGPU_EINVAL, "bad block layout");
    HIPCHK(c, hipSetDevice(c->device));
    hipStream_t ss = nullptr;
    HIPCHK(c, span_stream(c, slot, &ss));
    const bool zc = !force_copy && span_zerocopy(c);
    if (zc && n) {
        // the kernels read h_in and write h_out where they lie (page-locked
        // memory mapped into the device's address space): no copy engine
        if (h_in != sp.zc_hin) {
            void *d = nullptr;
            if (hipHostGetDevicePointer(&d, const_cast<void *>(h_in), 0) != hipSuccess || !d) {
                (void)hipGetLastError();
                return fail(c, FCGPU_EINVAL, "zero-copy block: h_in is not page-locked host memory (fcgpu_host_alloc)");
            }
            sp.zc_hin = h_in;
            sp.zc_din = static_cast<uint8_t *>(d);
        }
        if (h_out != sp.zc_hout) {
            void *d = nullptr;
            if (hipHostGetDevicePointer(&d, h_out, 0) != hipSuccess || !d) {
                (void)hipGetLastError();
                return fail(c, FCGPU_EINVAL, "zero-copy block: h_out is not page-locked host memory (fcgpu_host_alloc)");
            }
            sp.zc_hout = h_out;
            sp.zc_dout = static_cast<uint8_t *>(d);
        }
    } else if (in_bytes + kArenaPad > sp.in_cap || L.bytes > sp.res_cap) {
        // a reservation is never grown here: growing means freeing device
        // memory (a device-wide wait) on a submitting thread
        if (sp.reserved)
            return fail(c, FCGPU_ENOMEM, "block larger than the fcgpu_span_reserve reservation");
        int rc = span_blocks(c, slot, ss, in_bytes, outputs, partition);
        if (rc != FCGPU_OK) return rc;
    }
    if (c->fl.slots && !c->stream) HIPCHK(c, hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    sp.s = c->fl.slots ? c->stream : ss;
    hipStream_t s = sp.s;
    if (n == 0) return FCGPU_OK;
    uint8_t *din = zc ? sp.zc_din : sp.d_in, *dres = zc ? sp.zc_dout : sp.d_res;
    if (!zc) HIPCHK(c, hipMemcpyAsync(sp.d_in, h_in, in_bytes, hipMemcpyHostToDevice, s));
    auto at = [&](size_t o) -> void * { return o == FCGPU_OUT_ABSENT ? nullptr : dres + o; };
    fcgpu_out d{};
    d.verdict = (uint16_t *)at(L.verdict);
    d.hash = (uint32_t *)at(L.hash);
    d.anno = (fcgpu_anno *)at(L.anno);     // fcgpu_anno8 entries with kLayAnno8
    d.perm = (uint32_t *)at(L.perm);
    d.port_start = (uint32_t *)at(L.port_start);
    d.tile_count = (uint16_t *)at(L.tile_count);
    d.partition = partition;
    d.tile_perm = (uint8_t *)at(L.tile_perm);
    d.flowid = (uint32_t *)at(L.flowid);
    d.ip_rw = (uint32_t *)at(L.ip_rw);
    if (zc && agg_eligible(c, d)) {   // AUTO chose zero-copy: >= kZeroCopyAuto contexts share the device
        fcgpu_job j{};
        j.arena = din + frames_off;
        j.desc = descp(din);
        j.n = n;
        j.out = d;
        int rc = check_process(c, j.arena, j.desc, n, &j.out);
        if (rc != FCGPU_OK) return rc;
        return agg_submit(c, slot, j, layout);
    }
    int rc = check_process(c, din + frames_off, descp(din), n, &d);
    if (rc == FCGPU_OK) rc = process_one(c, din + frames_off, descp(din), n, &d, s, layout);
    if (rc != FCGPU_OK) return rc;
    if (!zc) HIPCHK(c, hipMemcpyAsync(h_out, sp.d_res, L.bytes, hipMemcpyDeviceToHost, s));
    uint32_t ns = 0;
    if (span_stream_mode(ns) != 0 && !c->fl.slots) {
        // a stream other slots also use: wait for this slot's work alone
        if (!sp.done) HIPCHK(c, hipEventCreateWithFlags(&sp.done, hipEventDisableTiming));
        HIPCHK(c, hipEventRecord(sp.done, s));
        sp.evt = true;
    } else {
        sp.evt = false;
    }
    sp.busy = true;
    return FCGPU_OK;
}

int fcgpu_span_wait(fcgpu_ctx *c, uint32_t slot) {
    if (!c || slot >= FCGPU_SPAN_SLOTS) return FCGPU_EINVAL;
    SpanSlot &sp = c->span[slot];
    if (!sp.busy) return FCGPU_OK;
    if (sp.doomed) {
        sp.doomed = sp.busy = false;
        return fail(c, FCGPU_ERUNTIME, "injected fault: batch failed on the device");
    }
    if (sp.agg) {
        const int r = agg_finish(c, slot, true);
        return r < 0 ? r : FCGPU_OK;
    }
    HIPCHK(c, hipSetDevice(c->device));
    sp.busy = false;
    if (sp.evt) HIPCHK(c, hipEventSynchronize(sp.done));
    else HIPCHK(c, hipStreamSynchronize(sp.s));
    return FCGPU_OK;
}

}  // extern "C"
