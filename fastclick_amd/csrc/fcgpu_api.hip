// fcgpu_api.hip -- C ABI (include/fastclick_gpu.h) over the gfx950 kernels.
//
// A context owns: the uploaded configuration, the partition workspace (per-tile
// histograms + bin totals), the device counter vector, pinned/device staging
// for host-resident batches, and optional per-stage timing events. Launch
// sequence per batch (all on one stream):
//   k_rx   fused check/hash/classify, per-tile histograms, sharded counters,
//          and (FCGPU_PART_TILE) each tile's stable partition  (grid = tiles)
//   FCGPU_PART_GLOBAL only:
//   k_scan per-output exclusive scan over tiles                 (grid = outputs)
//   k_part_multi dense stable partition scatter  (grid = batches' tiles / 8)
//   flow table only: the new-flow pass (fcgpu_flow.hh)
// Queued batches of one stream share one k_rx launch (process_fused).
//
// Sections, in file order:
//   context (struct fcgpu_ctx), error/event helpers
//   k_rx launch dispatch (launch_rx*: template instance per configuration;
//     compiled programs through jit_function)
//   whole-batch host path (process_host_whole)
//   decision programs: jump tables (build_tables), compiled programs (jit_*)
//   flow table: configure / clear / maintain / stats (fcgpu_flow_*)
//   open / configure / close
//   device-resident batches: process_one, fcgpu_process, fused jobs
//     (process_fused, fcgpu_process_jobs)
//   host-resident batches: pipelined chunks (process_host_pipelined), spans
//     and blocks (fcgpu_span_*), mbuf ingress (fcgpu_pool_register,
//     fcgpu_process_mbufs)
//   counters, programs, timing
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>
#include <string.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "fcgpu_device.hh"
#include "fcgpu_flow.hh"
#include "fcgpu_exchange.hh"
#include "capture.hh"
#include "prog_jit.hh"
#include "jit_sources.inc"   // kJitDeviceHh, kJitAbiH (fastclick_amd/build.py)

#pragma clang diagnostic ignored "-Wunused-result"
#pragma clang diagnostic ignored "-Wunused-value"

using namespace fcgpu;

static_assert(kTile == FCGPU_TILE, "tile size is part of the ABI");
static_assert(kCrcTabQ <= kTile, "k_rx copies the CRC tables with one uint4 per thread");
static constexpr size_t kCtrWords = (size_t)FCGPU_CTR_SHARDS * FCGPU_NCOUNTERS;

namespace {
constexpr uint32_t kHostCap = 128;          // bytes gathered per frame in host mode
constexpr uint32_t kArenaPad = 256;

struct EvPair {
    hipEvent_t a, b;
    int stage;
    uint32_t batches = 1;     // batches the bracketed launch processed (fused jobs)
};

constexpr size_t kTimingEvents = 6 * 64;     // pre-created by fcgpu_set_timing
constexpr uint32_t kChunk = 131072;         // packets per host-pipeline chunk (whole tiles)
constexpr int kSlots = 3;                   // chunks in flight: gather / copy+kernel / drain

// Host worker pool for the gather and copy-out loops (fcgpu_set_host_threads).
// The calling thread always takes part; n - 1 workers are started.
class Pool {
  public:
    ~Pool() { resize(1); }
    void resize(uint32_t n) {
        {
            std::unique_lock<std::mutex> lk(m_);
            quit_ = true;
            cv_.notify_all();
        }
        for (auto &t : th_) t.join();
        th_.clear();
        quit_ = false;
        for (uint32_t k = 1; k < n; ++k) th_.emplace_back([this, k] { loop(k); });
    }
    uint32_t size() const { return (uint32_t)th_.size() + 1; }
    // fn(part, nparts) on every member, the caller included; returns when all are done
    void run(const std::function<void(uint32_t, uint32_t)> &fn) {
        const uint32_t np = size();
        if (np == 1) { fn(0, 1); return; }
        {
            std::unique_lock<std::mutex> lk(m_);
            job_ = &fn;
            left_ = np - 1;
            ++gen_;
            cv_.notify_all();
        }
        fn(0, np);
        std::unique_lock<std::mutex> lk(m_);
        done_.wait(lk, [this] { return left_ == 0; });
        job_ = nullptr;
    }

  private:
    void loop(uint32_t k) {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(uint32_t, uint32_t)> *job;
            uint32_t np;
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [&] { return quit_ || gen_ != seen; });
                if (quit_) return;
                seen = gen_;
                job = job_;
                np = (uint32_t)th_.size() + 1;
            }
            (*job)(k, np);
            std::unique_lock<std::mutex> lk(m_);
            if (--left_ == 0) done_.notify_all();
        }
    }
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_, done_;
    const std::function<void(uint32_t, uint32_t)> *job_ = nullptr;
    uint32_t left_ = 0;
    uint64_t gen_ = 0;
    bool quit_ = false;
};

// One in-flight chunk of the host-resident pipeline: pinned staging in, device
// copies, device outputs, pinned outputs (used when the caller's arrays are
// pageable), its own stream and completion event.
struct HostSlot {
    size_t arena_cap = 0;     // bytes of h_arena / d_arena
    hipStream_t s = nullptr;
    hipEvent_t done = nullptr;
    uint8_t *h_arena = nullptr, *d_arena = nullptr;
    uint32_t *h_desc = nullptr, *d_desc = nullptr;
    uint16_t *d_v = nullptr, *h_v = nullptr;
    uint32_t *d_h = nullptr, *h_h = nullptr;
    fcgpu_anno *d_an = nullptr, *h_an = nullptr;
    uint32_t *d_perm = nullptr, *h_perm = nullptr;
    uint8_t *d_tp = nullptr, *h_tp = nullptr;
    uint16_t *d_tc = nullptr, *h_tc = nullptr;
    bool busy = false;
    uint32_t base = 0, n = 0;
};

// One in-flight fcgpu_span_submit: device copy of the span and descriptors,
// device outputs, the stream it runs on.
// one launch of the shared zero-copy queue (FCGPU_SPAN_AUTO, agg_take_locked / agg_issue)
struct AggLaunch {
    hipEvent_t ev = nullptr;
    uint32_t refs = 0;        // submissions it carries that have not been waited for
    // kAggIssuing until the thread that took the group from the queue has
    // issued it (outside the queue's lock), then kAggIssued or kAggFailed
    std::atomic<int> state{0};
};
constexpr int kAggIssuing = 0, kAggIssued = 1, kAggFailed = 2;

struct SpanSlot {
    hipStream_t own = nullptr, s = nullptr;
    uint8_t *d_span = nullptr;
    size_t span_cap = 0;
    uint32_t *d_desc = nullptr;
    uint16_t *d_v = nullptr, *d_tc = nullptr;
    uint32_t *d_h = nullptr, *d_perm = nullptr, *d_start = nullptr, *d_fl = nullptr, *d_rw = nullptr;
    fcgpu_anno *d_an = nullptr;
    uint8_t *d_tp = nullptr;
    uint8_t *d_in = nullptr, *d_res = nullptr;   // block submissions
    size_t in_cap = 0, res_cap = 0;
    // zero-copy block submissions: the device addresses of the last h_in / h_out
    const void *zc_hin = nullptr, *zc_hout = nullptr;
    uint8_t *zc_din = nullptr, *zc_dout = nullptr;
    // zero-copy span submissions: the last host -> device translation of each
    // pointer argument (span, descriptors, the nine output arrays)
    const void *zc_key[11] = {};
    void *zc_val[11] = {};
    // FCGPU_SPAN_AUTO with many contexts: the submission went to the device's
    // shared queue (agg); al = the launch carrying it (nullptr while pending)
    bool agg = false;
    AggLaunch *al = nullptr;
    bool busy = false;
    bool doomed = false;         // fcgpu_inject_fault(FCGPU_FAULT_WAIT): accepted, nothing ran, the wait fails
    hipEvent_t done = nullptr;   // shared streams: the slot's last operation (else the stream is waited)
    bool evt = false;            // the last submission recorded `done`
};

inline uint32_t span(uint32_t n, uint32_t part, uint32_t np) { return (uint32_t)((uint64_t)n * part / np); }

bool host_pinned(const void *p) {
    if (!p) return false;
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return at.type == hipMemoryTypeHost;
}
}  // namespace

struct fcgpu_ctx {
    int device = -1;
    uint32_t max_batch = 0;
    uint32_t max_tiles = 0;
    hipStream_t stream = nullptr;
    fcgpu_cfg cfg{};
    DevCfg dcfg{};
    bool configured = false;
    uint32_t *d_tilecnt = nullptr;
    uint32_t *d_totals = nullptr;
    // fused whole-batch partitions: per-tile counts and totals of each batch
    // of a launch (kMaxFuse x [FCGPU_MAX_PORTS+1][max_tiles], allocated on first use)
    uint32_t *fuse_tilecnt = nullptr, *fuse_totals = nullptr;
    unsigned long long *d_ctr = nullptr;      // active counter vector
    unsigned long long *d_ctr_own = nullptr;  // context-owned vector
    uint4 *d_prog = nullptr;                  // decision program (FCGPU_CLS_PROGRAM)
    uint4 *d_crc = nullptr;                   // LB_CRC slicing tables (crc32c_u32_tab)
    uint8_t *d_lbtab = nullptr;               // LB_TABLE bucket -> output (fcgpu_set_lb_table)
    uint32_t lbtab_n = 0, lbtab_max = 0;      // its buckets and largest output
    uint64_t lbtab_key = 0;                   // hash of its contents (0: none)
    uint32_t prog_n = 0, prog_kind = 0, prog_q = 0, prog_tab = 0;
    int32_t prog_all = -1;
    std::vector<fcgpu_step> prog_host;   // the installed program (capture reach)
    std::vector<uint4> prog_dev;         // ... in the device format (table steps, fallbacks, tables)
    uint64_t prog_key = 0;               // hash of the installed program's contents (0: none)
    // fcgpu_program_jit: the program compiled to code (prog_jit.hh)
    bool jit_on = false;
    std::string jit_src;                 // generated program function ("" = interpreted)
    std::vector<int> jit_keys;           // k_rx instantiations in the module
    JitModule jit;
    uint16_t *d_verdict = nullptr;   // scratch verdicts when the caller wants perm only
    // host-resident staging
    uint8_t *h_arena = nullptr, *d_arena = nullptr;
    size_t h_arena_cap = 0;
    uint32_t *h_desc = nullptr, *d_desc = nullptr;
    uint16_t *d_hv = nullptr;
    uint32_t *d_hh = nullptr, *d_hperm = nullptr, *d_hstart = nullptr;
    uint16_t *d_htc = nullptr;
    uint8_t *d_htp = nullptr;
    fcgpu_anno *d_hanno = nullptr;
    uint32_t *d_hflow = nullptr;
    uint32_t *d_hrw = nullptr;
    // pipelined host path (FCGPU_PART_TILE / no whole-batch partition)
    HostSlot slot[kSlots];
    uint32_t slot_cap = 0;
    Pool pool;
    // fcgpu_span_submit slots
    SpanSlot span[FCGPU_SPAN_SLOTS];
    int span_index = -1;              // FCGPU_SPAN_STREAMS=shared:N: this context's place in the pool
    uint32_t span_mode = FCGPU_SPAN_COPY;   // fcgpu_span_mode: block submissions copied or read in place
    struct AggQueue *aq = nullptr;          // the device's shared queue (FCGPU_SPAN_AUTO), once used
    // flow table (fcgpu_flow_enable)
    uint32_t max_flows = 0, flow_slots = 0, flow_words = 0;
    FlowArgs fl{};            // device pointers; fl.slots == nullptr: disabled
    uint32_t *flow_hint = nullptr;    // mapped: size class of the last finish's misses (kHint*)
    uint32_t flow_epoch = 0;          // batches through the table (FlowArgs::epoch)
    fcgpu_flow_config flow_conf{};    // the manager (fcgpu_flow_configure)
    // fused launches with a flow table: miss records of up to kMaxFuseFlow batches
    uint4 *fuse_key = nullptr;
    uint32_t *fuse_slot = nullptr, *fuse_missed = nullptr;
    uint64_t *fuse_mask = nullptr;
    uint4 *flow_spare = nullptr;      // IMP with timeouts: the slot array a maintainer run rebuilds into
    MaintArgs maint{};                // IMP with timeouts: released list, run numbers, timeout parameters
    uint32_t flow_now = 0;            // fcgpu_flow_set_time
    hipEvent_t flow_order[2] = {nullptr, nullptr};   // orders fcgpu_process against span submissions
    // mbuf ingress (fcgpu_pool_register / fcgpu_process_mbufs)
    uint64_t pool_host = 0, pool_bytes = 0;
    uint8_t *pool_dev = nullptr;
    bool pool_owned = false;          // this context holds a reference on the pool's registration
    uint64_t *d_mptr = nullptr;
    uint2 *d_mdesc = nullptr;
    // timing: every timing_every-th launch is bracketed by events (0 = off)
    uint32_t timing_every = 0;
    uint64_t timing_seq = 0;
    std::vector<EvPair> pending;
    std::vector<hipEvent_t> free_ev;
    // flow re-shard plan (fcgpu_exchange_plan): block sums and segment starts
    unsigned long long *x_bsum = nullptr, *x_base = nullptr, *x_part = nullptr;
    uint32_t *x_src = nullptr;   // arena offset of each leaving frame (plan -> pack)
    uint32_t *x_tcnt = nullptr;               // fcgpu_exchange_build: [64][max_tiles] per tile and owner
    unsigned long long *x_tbyt = nullptr;
    std::string err;
};

// Bytes of each frame the host paths stage (capture.hh): the reach of the
// configured chain, at least 128 B, or whole frames (L4 checksum, PROCESS_EH).
static uint32_t host_capture(const fcgpu_ctx *c) {
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
static hipError_t memset_sync(void *p, int v, size_t bytes) {
    hipError_t e = hipMemsetAsync(p, v, bytes, nullptr);
    if (e != hipSuccess) return e;
    return hipStreamSynchronize(nullptr);
}

static std::string g_open_err;
static bool fault_take(uint32_t where);
static void span_auto_count(fcgpu_ctx *c, uint32_t new_mode);
static bool span_zerocopy(const fcgpu_ctx *c);
int fcgpu_span_wait(fcgpu_ctx *c, uint32_t slot);

// Pools registered by fcgpu_pool_register, with the number of contexts using each.
static std::mutex g_pool_mu;
static std::map<std::pair<uint64_t, uint64_t>, uint32_t> g_pools;

static void pool_release(fcgpu_ctx *c) {
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

static int fail(fcgpu_ctx *c, int code, const std::string &msg) {
    if (c) c->err = msg;
    else g_open_err = msg;
    return code;
}

#define HIPCHK(ctx, expr)                                                                   \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess)                                                               \
            return fail((ctx), FCGPU_ERUNTIME,                                              \
                        std::string(#expr) + ": " + hipGetErrorString(e_));                 \
    } while (0)

static hipEvent_t take_event(fcgpu_ctx *c) {
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

// ev0/ev1 non-null: hipExtLaunchKernelGGL records them around the dispatch
// itself (timestamps of the kernel, not of the stream around it).
// L: one batch (njobs 1, grid = its tiles) or several fused ones (grid =
// their tiles end to end).
static hipFunction_t jit_function(fcgpu_ctx *c, int key);

template <int CM, bool CK, int PART, bool PROG, bool L4, bool FLOW = false>
static void launch_rx(const RxLaunch &L, uint32_t grid, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1,
                      fcgpu_ctx *jc) {
    if (PROG && jc) {   // the program compiled to code, when the context has it
        if (hipFunction_t fn = jit_function(jc, jit_key(CM, CK, PART, L4, FLOW))) {
            void *args[] = {const_cast<RxLaunch *>(&L)};
            if (ev0)
                hipExtModuleLaunchKernel(fn, grid * kTile, 1, 1, kTile, 1, 1, 0, s, args, nullptr, ev0, ev1, 0);
            else
                hipModuleLaunchKernel(fn, grid, 1, 1, kTile, 1, 1, 0, s, args, nullptr);
            return;
        }
    }
    const size_t lds = prog_lds_bytes(L.A.cfg);   // program steps (PROG), CRC tables (LB_CRC), LB table, else 0
    if (ev0)
        hipExtLaunchKernelGGL((k_rx<CM, CK, PART, PROG, L4, FLOW>), dim3(grid), dim3(kTile), lds, s, ev0, ev1,
                              0, L);
    else
        hipLaunchKernelGGL((k_rx<CM, CK, PART, PROG, L4, FLOW>), dim3(grid), dim3(kTile), lds, s, L);
}

// IPv4 check modes: L4 (CheckUDPHeader/CheckTCPHeader) and the flow table
// exist only there (fcgpu_configure / fcgpu_process reject them with CHECK_AUTO).
template <int CM, bool CK, int PART, bool PROG>
static void launch_rx_ip4(const RxLaunch &L, uint32_t grid, hipStream_t s, hipEvent_t e0, hipEvent_t e1, fcgpu_ctx *jc) {
    const bool l4 = L.A.cfg.l4_mode != FCGPU_L4_NONE, flow = L.A.fl.slots != nullptr;
    if (flow) {
        if (l4) launch_rx<CM, CK, PART, PROG, true, true>(L, grid, s, e0, e1, jc);
        else launch_rx<CM, CK, PART, PROG, false, true>(L, grid, s, e0, e1, jc);
    } else {
        if (l4) launch_rx<CM, CK, PART, PROG, true>(L, grid, s, e0, e1, jc);
        else launch_rx<CM, CK, PART, PROG, false>(L, grid, s, e0, e1, jc);
    }
}

template <int PART, bool PROG>
static void launch_rx_part(uint32_t cm, bool ck, const RxLaunch &L, uint32_t grid, hipStream_t s, hipEvent_t e0, hipEvent_t e1, fcgpu_ctx *jc) {
    switch (cm * 2 + (ck ? 1 : 0)) {
    case 0: launch_rx_ip4<FCGPU_CHECK_IP4, false, PART, PROG>(L, grid, s, e0, e1, jc); break;
    case 1: launch_rx_ip4<FCGPU_CHECK_IP4, true, PART, PROG>(L, grid, s, e0, e1, jc); break;
    case 2: case 3: launch_rx_ip4<FCGPU_MARK_IP4, false, PART, PROG>(L, grid, s, e0, e1, jc); break;
    case 4: launch_rx<FCGPU_CHECK_AUTO, false, PART, PROG, false>(L, grid, s, e0, e1, jc); break;
    case 6: case 7: launch_rx<FCGPU_MARK_IP6, false, PART, PROG, false>(L, grid, s, e0, e1, jc); break;
    default: launch_rx<FCGPU_CHECK_AUTO, true, PART, PROG, false>(L, grid, s, e0, e1, jc); break;
    }
}

// PROG: the decision-program classifier is compiled only into the kernels
// launched for FCGPU_CLS_PROGRAM, so the other modes keep their lean code.
template <bool PROG>
static void launch_rx_prog(int part, uint32_t cm, bool ck, const RxLaunch &L, uint32_t grid, hipStream_t s, hipEvent_t e0,
                           hipEvent_t e1, fcgpu_ctx *jc) {
    if (part == kPartTile) launch_rx_part<kPartTile, PROG>(cm, ck, L, grid, s, e0, e1, jc);
    else if (part == kPartGlobal) launch_rx_part<kPartGlobal, PROG>(cm, ck, L, grid, s, e0, e1, jc);
    else launch_rx_part<kPartNone, PROG>(cm, ck, L, grid, s, e0, e1, jc);
}

// The outputs a k_rx launch stores through without a null check, for the
// partition shape it is instantiated with (rx_tile: tile_count for
// kPartTile, tilecnt for kPartGlobal), and the inputs every batch reads: a
// launch missing one is refused on the host instead of faulting the device.
static bool rx_launch_ok(int part, const RxLaunch &L, uint32_t grid) {
    auto batch_ok = [part](const uint8_t *arena, const uint2 *desc, uint32_t n, const uint16_t *tile_count,
                           const uint32_t *tilecnt) {
        if (n && (!arena || !desc)) return false;
        if (part == kPartTile && n && !tile_count) return false;
        if (part == kPartGlobal && n && !tilecnt) return false;
        return true;
    };
    if (L.njobs <= 1)
        return batch_ok(L.A.arena, L.A.desc, L.A.n, L.A.tile_count, L.A.tilecnt) && L.A.ctr &&
               !(L.A.layout & ~kLayKnown) && grid <= (L.A.n + kTile - 1) / kTile;
    if (L.njobs > kMaxFuse) return false;
    uint32_t tiles = 0;
    for (uint32_t k = 0; k < L.njobs; ++k) {
        const RxJob &J = L.job[k];
        if (!batch_ok(J.arena, J.desc, J.n, J.tile_count, J.tilecnt) || !J.ctr || J.tile0 != tiles ||
            (J.layout & ~kLayKnown))
            return false;
        tiles += (J.n + kTile - 1) / kTile;
    }
    return grid <= tiles;
}

static hipError_t launch_rx_any(int part, uint32_t cm, bool ck, const RxLaunch &L, uint32_t grid, hipStream_t s, hipEvent_t e0,
                          hipEvent_t e1, fcgpu_ctx *jc) {
    if (!rx_launch_ok(part, L, grid)) return hipErrorInvalidValue;
    if (L.A.cfg.classify == FCGPU_CLS_PROGRAM) launch_rx_prog<true>(part, cm, ck, L, grid, s, e0, e1, jc);
    else launch_rx_prog<false>(part, cm, ck, L, grid, s, e0, e1, jc);
    return hipSuccess;
}

// One batch: a.ntiles workgroups.
static hipError_t launch_rx_one(int part, uint32_t cm, bool ck, const RxArgs &a, hipStream_t s, hipEvent_t e0,
                          hipEvent_t e1, fcgpu_ctx *jc) {
    RxLaunch L;
    L.A = a;
    L.njobs = 1;
    L.job_tiles = 0;
    return launch_rx_any(part, cm, ck, L, a.ntiles, s, e0, e1, jc);
}

// Whole batch in one shot (FCGPU_PART_GLOBAL: the partition spans the batch).
static int process_host_whole(fcgpu_ctx *c, const uint8_t *const *frames, const uint32_t *lens, uint32_t n,
                              const fcgpu_out *h) {
    const size_t arena_cap = (size_t)c->max_batch * kHostCap + kArenaPad;
    if (!c->h_arena) {
        // the context's own stream exists only for the host-resident path (a
        // stream per context maps onto one of the few hardware queues)
        HIPCHK(c, hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
        HIPCHK(c, hipHostMalloc((void **)&c->h_arena, arena_cap, hipHostMallocDefault));
        HIPCHK(c, hipHostMalloc((void **)&c->h_desc, sizeof(uint32_t) * 2 * c->max_batch, hipHostMallocDefault));
        HIPCHK(c, hipMalloc(&c->d_arena, arena_cap));
        HIPCHK(c, memset_sync(c->d_arena, 0, arena_cap));
        c->h_arena_cap = arena_cap;
        HIPCHK(c, hipMalloc(&c->d_desc, sizeof(uint32_t) * 2 * c->max_batch));
        HIPCHK(c, hipMalloc(&c->d_hv, sizeof(uint16_t) * c->max_batch));
        HIPCHK(c, hipMalloc(&c->d_hh, sizeof(uint32_t) * c->max_batch));
        HIPCHK(c, hipMalloc(&c->d_hperm, sizeof(uint32_t) * c->max_batch));
        HIPCHK(c, hipMalloc(&c->d_hstart, sizeof(uint32_t) * (FCGPU_MAX_PORTS + 2)));
        HIPCHK(c, hipMalloc(&c->d_hanno, sizeof(fcgpu_anno) * c->max_batch));
        HIPCHK(c, hipMalloc(&c->d_htc, sizeof(uint16_t) * (FCGPU_MAX_PORTS + 1) * c->max_tiles));
        HIPCHK(c, hipMalloc(&c->d_htp, (size_t)c->max_batch + kTile));
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
    if (need > c->h_arena_cap) {
        hipHostFree(c->h_arena);
        hipFree(c->d_arena);
        c->h_arena = nullptr;
        c->d_arena = nullptr;
        c->h_arena_cap = 0;
        HIPCHK(c, hipHostMalloc((void **)&c->h_arena, need, hipHostMallocDefault));
        HIPCHK(c, hipMalloc(&c->d_arena, need));
        HIPCHK(c, memset_sync(c->d_arena, 0, need));
        c->h_arena_cap = need;
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
    if (h->flowid && !c->d_hflow) HIPCHK(c, hipMalloc(&c->d_hflow, sizeof(uint32_t) * c->max_batch));
    d.flowid = h->flowid ? c->d_hflow : nullptr;
    if (h->ip_rw && !c->d_hrw) HIPCHK(c, hipMalloc(&c->d_hrw, sizeof(uint32_t) * c->max_batch));
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


// Jump tables for runs of steps that test one word (SURVEY 8(a) A11 programs:
// a rule's fields, and above all a port range the reference's compiler splits
// into a chain of mask tests on the transport word). Lanes of a wave walking
// such a chain for different port values leave it at different steps; a
// table gives every lane the chain's outcome in one step. For each entry step
// e (step 0, and every step reached by a jump from a step at another offset)
// the run R(e) = steps reachable from e through steps at e's offset. If the
// bits R's masks test span at most kTabBits bits of the big-endian word, e
// becomes a table step: tab[(bswap(word) >> lo) & (2^w - 1)] = where a walk
// from e with that word leaves R (an output <= 0 or a step outside R), and
// its original step is appended as the fallback for words that are not
// entirely inside the packet (the length-checked rules decide those). The
// steps keep their indices; dev grows by the fallback copies and the tables.
// Returns the step count (copies included); tab_q = uint4 index of the tables.
static uint32_t build_tables(std::vector<uint4> &dev, uint32_t nsteps, uint32_t &tab_q) {
    constexpr uint32_t kTabBits = 8, kTabBudget = 2048;     // entries per table, in total
    auto off_of = [&](uint32_t k) { return (int16_t)(dev[k].x & 0xffff); };
    auto yes_of = [&](const uint4 &st) { return (int32_t)(int16_t)(st.w & 0xffff); };
    auto no_of = [&](const uint4 &st) { return (int32_t)(int16_t)(st.w >> 16); };
    std::vector<char> entry(nsteps, 0);
    entry[0] = 1;
    for (uint32_t k = 0; k < nsteps; ++k)
        for (int32_t t : {yes_of(dev[k]), no_of(dev[k])})
            if (t > 0 && off_of((uint32_t)t) != off_of(k)) entry[t] = 1;
    std::vector<uint4> copies;
    std::vector<uint16_t> tabs;
    std::vector<int> inr(nsteps, -1);
    for (uint32_t e = 0; e < nsteps; ++e) {
        if (!entry[e]) continue;
        // the run from e
        std::vector<uint32_t> run{e}, todo{e};
        inr[e] = (int)e;
        uint32_t mbe = 0;
        while (!todo.empty()) {
            const uint32_t k = todo.back();
            todo.pop_back();
            mbe |= __builtin_bswap32(dev[k].z);
            for (int32_t t : {yes_of(dev[k]), no_of(dev[k])})
                if (t > 0 && inr[t] != (int)e && off_of((uint32_t)t) == off_of(e)) {
                    inr[t] = (int)e;
                    run.push_back((uint32_t)t);
                    todo.push_back((uint32_t)t);
                }
        }
        if (run.size() < 2 || mbe == 0) continue;
        const uint32_t lo = __builtin_ctz(mbe), w = 32 - __builtin_clz(mbe) - lo;
        if (w > kTabBits || tabs.size() + (1u << w) > kTabBudget) continue;
        const uint32_t base = (uint32_t)tabs.size();
        for (uint32_t idx = 0; idx < (1u << w); ++idx) {
            const uint32_t word = __builtin_bswap32(idx << lo);   // the packet word as the device loads it
            int32_t pos = (int32_t)e, j = -kProgUnmatched;
            for (size_t hops = 0; hops <= run.size(); ++hops) {
                const uint4 &st = dev[pos];
                j = (word & st.z) == st.y ? yes_of(st) : no_of(st);
                if (j <= 0 || inr[j] != (int)e) break;
                pos = j;
                j = -kProgUnmatched;                                // a cycle inside the run
            }
            tabs.push_back((uint16_t)(int16_t)j);
        }
        copies.push_back(dev[e]);
        const uint32_t copy_at = nsteps + (uint32_t)copies.size() - 1;
        dev[e].x = (dev[e].x & 0xffffu) | (kStepTable << 16);
        dev[e].y = base;
        dev[e].z = lo | (w << 8);
        dev[e].w = copy_at;
    }
    dev.resize(nsteps);
    dev.insert(dev.end(), copies.begin(), copies.end());
    tab_q = (uint32_t)dev.size();
    tabs.resize((tabs.size() + 7) & ~(size_t)7, 0);
    for (size_t k = 0; k < tabs.size(); k += 8) {
        uint4 q;
        q.x = tabs[k] | (uint32_t)tabs[k + 1] << 16;
        q.y = tabs[k + 2] | (uint32_t)tabs[k + 3] << 16;
        q.z = tabs[k + 4] | (uint32_t)tabs[k + 5] << 16;
        q.w = tabs[k + 6] | (uint32_t)tabs[k + 7] << 16;
        dev.push_back(q);
    }
    return nsteps + (uint32_t)copies.size();
}

// ---- compiled programs (fcgpu_program_jit, prog_jit.hh) ---------------------
// The k_rx instantiations the context's configuration launches (as the
// launch_rx_part dispatch normalises them), for every partition shape.
static std::vector<int> jit_keys_for(const fcgpu_ctx *c) {
    int cm = (int)c->cfg.check_mode;
    bool ck = c->cfg.checksum != 0;
    if (cm == FCGPU_MARK_IP4 || cm == FCGPU_MARK_IP6) ck = false;
    const bool ip4 = cm == FCGPU_CHECK_IP4 || cm == FCGPU_MARK_IP4;
    const bool l4 = ip4 && c->cfg.l4_mode != FCGPU_L4_NONE, flow = ip4 && c->fl.slots != nullptr;
    std::vector<int> keys;
    for (int part : {kPartTile, kPartNone, kPartGlobal}) keys.push_back(jit_key(cm, ck, part, l4, flow));
    return keys;
}

// (Re)build the module for the installed program and `keys`.
static int jit_build(fcgpu_ctx *c, const std::vector<int> &keys) {
    std::string err;
    HIPCHK(c, hipSetDevice(c->device));
    // launches of the module being replaced may still run
    HIPCHK(c, hipDeviceSynchronize());
    if (!jit_compile(c->jit_src, keys, kJitDeviceHh, kJitAbiH, c->jit, err)) {
        c->jit_src.clear();
        c->jit_keys.clear();
        return fail(c, FCGPU_ERUNTIME, "fcgpu_program_jit: " + err);
    }
    c->jit_keys = keys;
    return FCGPU_OK;
}

// The installed program as code: generated and compiled for the current
// configuration; a program with a cycle stays interpreted (error returned).
static int jit_install(fcgpu_ctx *c) {
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipDeviceSynchronize());      // no launch of the old module still running
    c->jit.unload();
    c->jit_src.clear();
    c->jit_keys.clear();
    if (!c->jit_on || c->prog_all >= 0 || c->prog_dev.empty()) return FCGPU_OK;
    std::string why;
    c->jit_src = jit_program_source(c->prog_dev, c->prog_n, c->prog_tab, c->prog_kind, why);
    if (c->jit_src.empty()) return fail(c, FCGPU_EINVAL, "fcgpu_program_jit: " + why);
    return jit_build(c, jit_keys_for(c));
}

// The compiled kernel for an instantiation; one the module lacks (the
// configuration changed since) is added by recompiling. nullptr: interpret.
static bool agg_queued(const fcgpu_ctx *c);
static hipFunction_t jit_function(fcgpu_ctx *c, int key) {
    auto it = c->jit.fn.find(key);
    if (it != c->jit.fn.end()) return it->second;
    // a rebuild replaces the module, whose functions this context's queued
    // shared-queue submissions hold until they launch: interpret instead
    // (identical results) while one is queued
    if (agg_queued(c)) return nullptr;
    std::vector<int> keys = c->jit_keys;
    keys.push_back(key);
    if (jit_build(c, keys) != FCGPU_OK) return nullptr;
    it = c->jit.fn.find(key);
    return it == c->jit.fn.end() ? nullptr : it->second;
}

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

static void flow_free(fcgpu_ctx *c) {
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
    // at most max_flows IDs plus one batch of FULL markers (the batch that
    // fills the table): keep the load at or under 1/2
    uint32_t slots = 1024;
    while (slots < 2 * (max_flows + c->max_batch)) slots <<= 1;
    const uint32_t words = (c->max_batch + 63) / 64 + 1;
    FlowArgs &F = c->fl;
    HIPCHK(c, hipMalloc(&F.slots, sizeof(uint4) * slots));
    HIPCHK(c, hipMalloc(&F.claim, sizeof(uint32_t) * slots));
    HIPCHK(c, hipMalloc(&F.first, sizeof(uint32_t) * slots));
    HIPCHK(c, hipMalloc(&F.miss_key, sizeof(uint4) * c->max_batch));
    HIPCHK(c, hipMalloc(&F.miss_slot, sizeof(uint32_t) * c->max_batch));
    HIPCHK(c, hipMalloc(&F.miss_first, sizeof(uint32_t) * c->max_batch));
    HIPCHK(c, hipMalloc(&F.missmask, sizeof(uint64_t) * words));
    HIPCHK(c, hipMalloc(&F.firstmask, sizeof(uint64_t) * words));
    HIPCHK(c, hipMalloc(&F.wordpre, sizeof(uint32_t) * words));
    HIPCHK(c, hipMalloc(&F.state, sizeof(uint32_t) * 16));
    F.missed = F.state + kFsMissed;
    if (imp) HIPCHK(c, hipMalloc(&F.stack, sizeof(uint32_t) * max_flows));
    if (te) {
        F.wstride = cap;
        F.wmask = nb - 1;
        F.te = te;
        HIPCHK(c, hipMalloc(&F.lastseen, sizeof(uint32_t) * cap));
        HIPCHK(c, hipMalloc(&F.wheel, sizeof(uint32_t) * (size_t)nb * cap));
        HIPCHK(c, hipMalloc(&F.wheel_len, sizeof(uint32_t) * nb));
        HIPCHK(c, hipMalloc(&c->flow_spare, sizeof(uint4) * slots));
        HIPCHK(c, hipMalloc(&c->maint.qbsr, sizeof(uint32_t) * cap));
        HIPCHK(c, hipMalloc(&c->maint.dead, sizeof(uint32_t) * cap));
        HIPCHK(c, hipMalloc(&c->maint.rbuf, sizeof(uint16_t) * cap));
        HIPCHK(c, hipMalloc(&c->maint.counts, sizeof(uint32_t) * (size_t)((cap + kMaintChunk - 1) / kMaintChunk) *
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

static bool agg_queued(const fcgpu_ctx *c);
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
        HIPCHK(c, hipMalloc(&c->d_crc, sizeof(uint32_t) * 512));
        HIPCHK(c, hipMemcpy(c->d_crc, t.data(), sizeof(uint32_t) * 512, hipMemcpyHostToDevice));
    }
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

// Tiles per k_part_multi workgroup: up to kPartTiles, while the grid keeps
// ~2048 workgroups (8 per CU) to fill the machine.
static uint32_t part_tiles_per_wg(uint32_t tiles) {
    return std::max(1u, std::min(kPartTiles, tiles / 2048u));
}

// Argument checks shared by fcgpu_process and fcgpu_process_jobs.
static int check_process(fcgpu_ctx *c, const uint8_t *d_arena, const uint32_t *d_desc, uint32_t n,
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

// The new-flow pass of one batch of n packets (fcgpu_flow.hh), its shape
// predicted by the last pass's class of misses (no sync: maybe older).
static hipError_t flow_pass(fcgpu_ctx *c, const FlowArgs &F, uint32_t n, hipStream_t s) {
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

// One batch's launches on stream s (arguments checked, device current).
// layout: kLay* bits of the batch's descriptors and annotations (0 through
// the public entry points: {off, len} descriptors, fcgpu_anno).
static int process_one(fcgpu_ctx *c, const uint8_t *d_arena, const uint32_t *d_desc, uint32_t n,
                       const fcgpu_out *o, hipStream_t s, uint32_t layout = 0) {
    if (n == 0) return FCGPU_OK;
    const uint32_t ntiles = (n + kTile - 1) / kTile;
    const uint32_t nports = c->cfg.nports;
    uint16_t *verdict = o->verdict;
    if (!verdict && o->partition == FCGPU_PART_GLOBAL && o->perm) {
        if (!c->d_verdict) HIPCHK(c, hipMalloc(&c->d_verdict, sizeof(uint16_t) * c->max_batch));
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

int fcgpu_process(fcgpu_ctx *c, const uint8_t *d_arena, const uint32_t *d_desc, uint32_t n,
                  const fcgpu_out *o, void *stream) {
    if (!c || !o) return FCGPU_EINVAL;
    int rc = check_process(c, d_arena, d_desc, n, o);
    if (rc != FCGPU_OK || n == 0) return rc;
    HIPCHK(c, hipSetDevice(c->device));
    return process_one(c, d_arena, d_desc, n, o, (hipStream_t)stream);   // NULL = the null stream
}

// The partition shape process_one launches k_rx with for these outputs.
static int out_part(const fcgpu_out *o) {
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
            HIPCHK(c, hipMalloc(&c->fuse_key, sizeof(uint4) * (size_t)kMaxFuseFlow * c->max_batch));
            HIPCHK(c, hipMalloc(&c->fuse_slot, sizeof(uint32_t) * (size_t)kMaxFuseFlow * c->max_batch));
            HIPCHK(c, hipMalloc(&c->fuse_mask, sizeof(uint64_t) * kMaxFuseFlow * words));
            HIPCHK(c, hipMalloc(&c->fuse_missed, sizeof(uint32_t) * kMaxFuseFlow));
            HIPCHK(c, memset_sync(c->fuse_mask, 0, sizeof(uint64_t) * kMaxFuseFlow * words));
            HIPCHK(c, memset_sync(c->fuse_missed, 0, sizeof(uint32_t) * kMaxFuseFlow));
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
        HIPCHK(c, hipMalloc(&c->fuse_tilecnt, sizeof(uint32_t) * (size_t)kMaxFuse * kFuseCntStride * c->max_tiles));
        HIPCHK(c, hipMalloc(&c->fuse_totals, sizeof(uint32_t) * (size_t)kMaxFuse * kFuseCntStride));
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
    if (flow && *(volatile uint32_t *)c->flow_hint != kHintBig) {
        // the batches' new-flow passes, in batch order, in one block
        static_assert(kMaxFuseFlow <= kMaxFusePass, "k_flow_finish_multi");
        FinishMulti M{};
        M.g = g;
        M.stride = L.flow_stride;
        M.words = L.flow_words;
        for (uint32_t k = 0; k < g; ++k) {
            M.n[k] = grp[k]->n;
            M.flowid[k] = grp[k]->out.flowid;
        }
        hipLaunchKernelGGL(k_flow_finish_multi, dim3(1), dim3(kFinishBlock), 0, s, a.fl, M);
        HIPCHK(c, hipGetLastError());
    } else if (flow) {
        // many new flows: each batch's grid-wide pass, in batch order
        for (uint32_t k = 0; k < g; ++k) {
            FlowArgs F = a.fl;
            F.miss_key += (size_t)k * L.flow_stride;
            F.miss_slot += (size_t)k * L.flow_stride;
            F.missmask += (size_t)k * L.flow_words;
            F.missed += k;
            F.epoch = epoch0 + k;
            F.flowid = grp[k]->out.flowid;
            HIPCHK(c, flow_pass(c, F, grp[k]->n, s));
        }
    }
    if (flow) {
        if (cross) {
            HIPCHK(c, hipEventRecord(c->flow_order[1], s));
            HIPCHK(c, hipStreamWaitEvent(c->stream, c->flow_order[1], 0));
        }
    }
    return FCGPU_OK;
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

static int slot_alloc(fcgpu_ctx *c, HostSlot &sl, uint32_t cap) {
    const size_t tiles = (cap + kTile - 1) / kTile;
    HIPCHK(c, hipStreamCreateWithFlags(&sl.s, hipStreamNonBlocking));
    HIPCHK(c, hipEventCreateWithFlags(&sl.done, hipEventDisableTiming));
    const size_t arena = (size_t)cap * kHostCap + kArenaPad;
    sl.arena_cap = arena;
    HIPCHK(c, hipHostMalloc((void **)&sl.h_arena, arena, hipHostMallocDefault));
    HIPCHK(c, hipHostMalloc((void **)&sl.h_desc, sizeof(uint32_t) * 2 * cap, hipHostMallocDefault));
    HIPCHK(c, hipMalloc(&sl.d_arena, arena));
    HIPCHK(c, memset_sync(sl.d_arena, 0, arena));
    HIPCHK(c, hipMalloc(&sl.d_desc, sizeof(uint32_t) * 2 * cap));
    HIPCHK(c, hipMalloc(&sl.d_v, sizeof(uint16_t) * cap));
    HIPCHK(c, hipMalloc(&sl.d_h, sizeof(uint32_t) * cap));
    HIPCHK(c, hipMalloc(&sl.d_an, sizeof(fcgpu_anno) * cap));
    HIPCHK(c, hipMalloc(&sl.d_perm, sizeof(uint32_t) * cap));
    HIPCHK(c, hipMalloc(&sl.d_tp, (size_t)cap + kTile));
    HIPCHK(c, hipMalloc(&sl.d_tc, sizeof(uint16_t) * (FCGPU_MAX_PORTS + 1) * tiles));
    HIPCHK(c, hipHostMalloc((void **)&sl.h_v, sizeof(uint16_t) * cap, hipHostMallocDefault));
    HIPCHK(c, hipHostMalloc((void **)&sl.h_h, sizeof(uint32_t) * cap, hipHostMallocDefault));
    HIPCHK(c, hipHostMalloc((void **)&sl.h_an, sizeof(fcgpu_anno) * cap, hipHostMallocDefault));
    HIPCHK(c, hipHostMalloc((void **)&sl.h_perm, sizeof(uint32_t) * cap, hipHostMallocDefault));
    HIPCHK(c, hipHostMalloc((void **)&sl.h_tp, (size_t)cap + kTile, hipHostMallocDefault));
    HIPCHK(c, hipHostMalloc((void **)&sl.h_tc, sizeof(uint16_t) * (FCGPU_MAX_PORTS + 1) * tiles,
                            hipHostMallocDefault));
    return FCGPU_OK;
}

namespace {
struct PinnedOut {           // which caller arrays the DMA engine can write directly
    bool v, h, an, perm, tp, tc;
};
}

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
            HIPCHK(c, hipHostMalloc((void **)&sl.h_arena, want, hipHostMallocDefault));
            HIPCHK(c, hipMalloc(&sl.d_arena, want));
            HIPCHK(c, memset_sync(sl.d_arena, 0, want));
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
    if (!sp.own) {
        const size_t m = c->max_batch, tiles = (m + kTile - 1) / kTile;
        HIPCHK(c, hipStreamCreateWithFlags(&sp.own, hipStreamNonBlocking));
        HIPCHK(c, hipMalloc(&sp.d_desc, sizeof(uint32_t) * 2 * m));
        HIPCHK(c, hipMalloc(&sp.d_v, sizeof(uint16_t) * m));
        HIPCHK(c, hipMalloc(&sp.d_h, sizeof(uint32_t) * m));
        HIPCHK(c, hipMalloc(&sp.d_an, sizeof(fcgpu_anno) * m));
        HIPCHK(c, hipMalloc(&sp.d_perm, sizeof(uint32_t) * m));
        HIPCHK(c, hipMalloc(&sp.d_start, sizeof(uint32_t) * (FCGPU_MAX_PORTS + 2)));
        HIPCHK(c, hipMalloc(&sp.d_tp, m + kTile));
        HIPCHK(c, hipMalloc(&sp.d_tc, sizeof(uint16_t) * (FCGPU_MAX_PORTS + 1) * tiles));
        HIPCHK(c, hipMalloc(&sp.d_fl, sizeof(uint32_t) * m));
        HIPCHK(c, hipMalloc(&sp.d_rw, sizeof(uint32_t) * m));
    }
    const bool zc = span_zerocopy(c);
    if (!zc && bytes + kArenaPad > sp.span_cap) {
        HIPCHK(c, hipStreamSynchronize(sp.own));
        hipFree(sp.d_span);
        sp.d_span = nullptr;
        sp.span_cap = 0;
        const size_t cap = (bytes + kArenaPad + (1u << 20) - 1) & ~(size_t)((1u << 20) - 1);
        HIPCHK(c, hipMalloc(&sp.d_span, cap));
        HIPCHK(c, memset_sync(sp.d_span, 0, cap));
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

// FCGPU_SPAN_AUTO: contexts per device in that mode; block submissions go
// zero-copy while at least kZeroCopyAuto of them exist (one or two threads
// submit few enough copies for the copy engine, and copies are faster there:
// profiles/r03_s8/el_zc.log)
constexpr uint32_t kZeroCopyAuto = 4;
constexpr int kMaxDevices = 64;
static std::atomic<uint32_t> g_auto_n[kMaxDevices];   // AUTO contexts per device (read on every submission)
static void agg_release(int device);
static void span_auto_count(fcgpu_ctx *c, uint32_t new_mode) {
    const bool was = c->span_mode == FCGPU_SPAN_AUTO, now = new_mode == FCGPU_SPAN_AUTO;
    if (was == now || c->device < 0 || c->device >= kMaxDevices) return;
    if (now) {
        g_auto_n[c->device].fetch_add(1, std::memory_order_relaxed);
    } else if (g_auto_n[c->device].fetch_sub(1, std::memory_order_acq_rel) == 1) {
        agg_release(c->device);
    }
}
static bool span_zerocopy(const fcgpu_ctx *c) {
    if (c->span_mode != FCGPU_SPAN_AUTO) return c->span_mode == FCGPU_SPAN_ZEROCOPY;
    return c->device >= 0 && c->device < kMaxDevices &&
           g_auto_n[c->device].load(std::memory_order_relaxed) >= kZeroCopyAuto;
}

// ---- fault injection (fcgpu_inject_fault) ------------------------------------
static std::atomic<uint32_t> g_fault_armed{0};     // bit k: kind k has events to skip or fail
static std::mutex g_fault_mu;
static uint32_t g_fault_skip[3], g_fault_count[3];
static bool fault_take(uint32_t where) {
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
struct AggQueue {
    std::mutex mu;
    int device = -1;
    std::vector<AggItem> pending;
    hipStream_t st[4] = {};
    uint32_t rr = 0;
    std::vector<AggLaunch *> spare;
};
constexpr uint32_t kAggLaunch = 4;
static std::mutex g_agg_mu;
static std::map<int, AggQueue *> g_agg;
static AggQueue &agg_queue(fcgpu_ctx *c) {
    if (c->aq) return *c->aq;
    std::lock_guard<std::mutex> g(g_agg_mu);
    AggQueue *&q = g_agg[c->device];
    if (!q) {
        q = new AggQueue();
        q->device = c->device;
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
static bool agg_queued(const fcgpu_ctx *c) {
    for (const SpanSlot &sp : c->span)
        if (sp.busy && sp.agg) return true;
    return false;
}
static hipError_t launch_rx_fn(hipFunction_t fn, int part, const RxLaunch &L, uint32_t grid, hipStream_t s) {
    if (!rx_launch_ok(part, L, grid)) return hipErrorInvalidValue;
    void *args[] = {const_cast<RxLaunch *>(&L)};
    return hipModuleLaunchKernel(fn, grid, 1, 1, kTile, 1, 1, 0, s, args, nullptr);
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
    hipStream_t st;
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
        const uint32_t si = q.rr++ % 4;
        if (!q.st[si] && hipStreamCreateWithFlags(&q.st[si], hipStreamNonBlocking) != hipSuccess) {
            (void)hipGetLastError();
            q.st[si] = nullptr;
        }
        is.st = q.st[si];
        AggLaunch *al = nullptr;
        if (!q.spare.empty()) {
            al = q.spare.back();
            q.spare.pop_back();
        } else {
            al = new AggLaunch();
            if (hipEventCreateWithFlags(&al->ev, hipEventDisableTiming) != hipSuccess) {
                (void)hipGetLastError();
                al->ev = nullptr;
            }
        }
        al->state.store(kAggIssuing, std::memory_order_relaxed);
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
static void agg_issue(int device, std::vector<AggIssue> &iss) {
    if (iss.empty()) return;
    const bool dev_ok = hipSetDevice(device) == hipSuccess;
    for (AggIssue &is : iss) {
        hipError_t e = dev_ok && is.st && is.al->ev ? hipSuccess : hipErrorInvalidValue;
        if (e == hipSuccess && fault_take(FCGPU_FAULT_LAUNCH)) e = hipErrorLaunchFailure;
        if (e == hipSuccess) {
            if (is.fn) {
                e = launch_rx_fn(is.fn, is.part, is.L, is.tiles, is.st);
            } else {
                e = launch_rx_any(is.part, is.cm, is.ck, is.L, is.tiles, is.st, nullptr, nullptr, nullptr);
                if (e == hipSuccess) e = hipGetLastError();
            }
        }
        if (e == hipSuccess) e = hipEventRecord(is.al->ev, is.st);
        if (e != hipSuccess) (void)hipGetLastError();
        is.al->state.store(e == hipSuccess ? kAggIssued : kAggFailed, std::memory_order_release);
    }
    iss.clear();
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
        if (q.pending.size() >= kAggLaunch) agg_take_locked(q, iss);
    }
    agg_issue(q.device, iss);
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
    agg_issue(q.device, iss);
    // the thread that took its group issues it outside the lock
    int st;
    while ((st = al->state.load(std::memory_order_acquire)) == kAggIssuing) {
        if (!block) return 0;
        std::this_thread::yield();
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
    } else if (in_bytes + kArenaPad > sp.in_cap) {
        HIPCHK(c, hipStreamSynchronize(ss));
        hipFree(sp.d_in);
        sp.d_in = nullptr;
        sp.in_cap = 0;
        const size_t cap = (in_bytes + kArenaPad + (1u << 20) - 1) & ~(size_t)((1u << 20) - 1);
        HIPCHK(c, hipMalloc(&sp.d_in, cap));
        HIPCHK(c, memset_sync(sp.d_in, 0, cap));
        sp.in_cap = cap;
    }
    if (!zc && L.bytes > sp.res_cap) {
        HIPCHK(c, hipStreamSynchronize(ss));
        hipFree(sp.d_res);
        sp.d_res = nullptr;
        sp.res_cap = 0;
        fcgpu_block_layout M;    // room for a full batch with these outputs
        fcgpu_block_layout_for(c, c->max_batch, outputs, partition, &M);
        const size_t cap = std::max(M.bytes, L.bytes);
        HIPCHK(c, hipMalloc(&sp.d_res, cap));
        sp.res_cap = cap;
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

int fcgpu_launch_guard_selftest(void) {
    // host-only: rx_launch_ok decides before any HIP call
    static uint8_t arena[64];
    static uint2 desc[1];
    static uint16_t tc[FCGPU_MAX_PORTS + 1];
    static uint32_t tcnt[FCGPU_MAX_PORTS + 1];
    static unsigned long long ctr[1];
    auto one = [](uint32_t n) {
        RxLaunch L;
        L.A = RxArgs{};
        L.A.arena = arena;
        L.A.desc = desc;
        L.A.n = n;
        L.A.ctr = ctr;
        L.A.tile_count = tc;
        L.A.tilecnt = tcnt;
        L.njobs = 1;
        L.job_tiles = 0;
        return L;
    };
    auto fused = [](uint32_t njobs, uint32_t n) {
        RxLaunch L;
        L.A = RxArgs{};
        L.njobs = njobs;
        L.job_tiles = 0;
        for (uint32_t k = 0; k < njobs && k < kMaxFuse; ++k) {
            RxJob &J = L.job[k];
            J = RxJob{};
            J.arena = arena;
            J.desc = desc;
            J.n = n;
            J.ctr = ctr;
            J.tile_count = tc;
            J.tilecnt = tcnt;
            J.tile0 = k * ((n + kTile - 1) / kTile);
        }
        return L;
    };
    const uint32_t n = 1000, t = (n + kTile - 1) / kTile;
    // well-formed launches must pass, or the checks below prove nothing
    if (!rx_launch_ok(kPartTile, one(n), t) || !rx_launch_ok(kPartGlobal, one(n), t) ||
        !rx_launch_ok(kPartTile, fused(3, n), 3 * t))
        return -1;
    {   // every known layout passes, alone and mixed within a launch
        RxLaunch K = one(n);
        K.A.layout = kLayKnown;
        RxLaunch F = fused(3, n);
        F.job[0].layout = kLayDesc32;
        F.job[1].layout = kLayAnno8;
        F.job[2].layout = kLayKnown;
        if (!rx_launch_ok(kPartTile, K, t) || !rx_launch_ok(kPartTile, F, 3 * t)) return -1;
    }
    int accepted = 0;
    RxLaunch L = one(n);
    L.A.tile_count = nullptr;                           // the r03_s17 fault: TILE stores through tile_count
    accepted += rx_launch_ok(kPartTile, L, t);
    L = one(n);
    L.A.tilecnt = nullptr;                              // GLOBAL stores per-tile counts
    accepted += rx_launch_ok(kPartGlobal, L, t);
    L = one(n);
    L.A.arena = nullptr;
    accepted += rx_launch_ok(kPartNone, L, t);
    L = one(n);
    L.A.desc = nullptr;
    accepted += rx_launch_ok(kPartNone, L, t);
    L = one(n);
    L.A.ctr = nullptr;
    accepted += rx_launch_ok(kPartNone, L, t);
    accepted += rx_launch_ok(kPartNone, one(n), t + 1);       // more workgroups than tiles
    L = fused(3, n);
    L.job[1].tile_count = nullptr;
    accepted += rx_launch_ok(kPartTile, L, 3 * t);
    L = fused(3, n);
    L.job[2].tile0 += 1;                                // tiles not end to end
    accepted += rx_launch_ok(kPartTile, L, 3 * t);
    L = fused(3, n);
    accepted += rx_launch_ok(kPartTile, L, 3 * t + 1);
    L = fused(kMaxFuse, n);
    L.njobs = kMaxFuse + 1;
    accepted += rx_launch_ok(kPartTile, L, kMaxFuse * t);
    L = one(n);
    L.A.layout = kLayKnown + 1;                         // a layout bit no kernel knows
    accepted += rx_launch_ok(kPartTile, L, t);
    L = one(n);
    L.A.layout = 0x80000000u;
    accepted += rx_launch_ok(kPartTile, L, t);
    L = fused(3, n);
    L.job[2].layout = 4u;
    accepted += rx_launch_ok(kPartTile, L, 3 * t);
    return accepted;
}

int fcgpu_inject_fault(uint32_t where, uint32_t skip, uint32_t count) {
    if (where > FCGPU_FAULT_LAUNCH) return FCGPU_EINVAL;
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
    void *dev = nullptr;
    HIPCHK(c, hipHostGetDevicePointer(&dev, base, 0));
    c->pool_host = (uint64_t)base;
    c->pool_bytes = bytes;
    c->pool_dev = static_cast<uint8_t *>(dev);
    if (!c->d_mptr) {
        HIPCHK(c, hipMalloc(&c->d_mptr, sizeof(uint64_t) * c->max_batch));
        HIPCHK(c, hipMalloc(&c->d_mdesc, sizeof(uint2) * c->max_batch));
    }
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

int fcgpu_set_program(fcgpu_ctx *c, uint32_t kind, const fcgpu_step *steps, uint32_t nsteps,
                      int32_t output_everything) {
    if (!c) return FCGPU_EINVAL;
    if (kind > FCGPU_PROG_CLASSIFIER) return fail(c, FCGPU_EINVAL, "bad program kind");
    if (nsteps > FCGPU_MAX_STEPS || (nsteps && !steps)) return fail(c, FCGPU_EINVAL, "bad program size");
    if (nsteps == 0 && output_everything < 0) return fail(c, FCGPU_EINVAL, "empty program without output");
    if (agg_queued(c)) return fail(c, FCGPU_EINVAL, "fcgpu_set_program: a queued span submission is not waited for");
    std::vector<uint4> dev(nsteps ? nsteps : 1);
    auto jump = [](int32_t j) -> int32_t {       // [X] (drop) and out-of-range -> unmatched
        if (j <= -32767 || j > 32767) return -kProgUnmatched;
        return j;
    };
    for (uint32_t k = 0; k < nsteps; ++k) {
        const fcgpu_step &st = steps[k];
        if (st.offset < -32768 || st.offset > 32767) return fail(c, FCGPU_EINVAL, "step offset out of range");
        const int32_t y = jump(st.yes), n = jump(st.no);
        if (y > (int32_t)nsteps - 1 || n > (int32_t)nsteps - 1) return fail(c, FCGPU_EINVAL, "jump past the program");
        dev[k].x = (uint32_t)(uint16_t)st.offset | ((st.flags & FCGPU_STEP_SHORT_YES) << 16);
        dev[k].y = st.value & st.mask;
        dev[k].z = st.mask;
        dev[k].w = (uint32_t)(uint16_t)y | ((uint32_t)(uint16_t)n << 16);
    }
    uint32_t tab_q = 0;
    const uint32_t total_n = nsteps ? build_tables(dev, nsteps, tab_q) : 0;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipDeviceSynchronize());
    hipFree(c->d_prog);
    c->d_prog = nullptr;
    HIPCHK(c, hipMalloc(&c->d_prog, sizeof(uint4) * dev.size()));
    HIPCHK(c, hipMemcpy(c->d_prog, dev.data(), sizeof(uint4) * dev.size(), hipMemcpyHostToDevice));
    c->prog_host.assign(steps, steps + nsteps);
    c->prog_n = total_n;
    c->prog_q = (uint32_t)dev.size();
    c->prog_tab = tab_q;
    c->dcfg.prog_q = c->prog_q;
    c->dcfg.prog_tab = c->prog_tab;
    c->prog_kind = kind;
    c->prog_all = nsteps == 0 ? output_everything : -1;
    c->dcfg.prog = c->d_prog;
    c->dcfg.prog_n = c->prog_n;
    c->dcfg.prog_kind = c->prog_kind;
    c->dcfg.prog_all = c->prog_all;
    c->prog_dev = dev;
    // contents, not the device copy: contexts with one program share launches
    uint64_t key = 1469598103934665603ull;
    auto mix = [&key](uint32_t v) {
        for (int b = 0; b < 4; ++b) key = (key ^ ((v >> (8 * b)) & 0xff)) * 1099511628211ull;
    };
    for (const uint4 &q : dev) {
        mix(q.x);
        mix(q.y);
        mix(q.z);
        mix(q.w);
    }
    for (uint32_t v : {c->prog_n, c->prog_q, c->prog_tab, c->prog_kind, (uint32_t)c->prog_all}) mix(v);
    c->prog_key = key | 1;
    if (c->jit_on && jit_install(c) != FCGPU_OK) c->err.clear();   // a cycle: interpreted
    return FCGPU_OK;
}

// Server i at cantor(i, j) % size (include/click/algorithm.hh:136-138,
// unsigned) for j < ((size - 1) / nsel) + 1, later placements winning; an
// empty bucket takes the last server placed before it (server 0 before the
// first).
int fcgpu_lb_hash_ring(uint32_t nsel, uint32_t size, uint8_t *out) {
    if (nsel < 1 || nsel > FCGPU_MAX_PORTS || size < 1 || size > FCGPU_LB_TABLE_MAX || !out) return FCGPU_EINVAL;
    std::vector<uint32_t> ring(size, 0xffffffffu);
    const uint32_t fac = (size - 1) / nsel + 1;
    for (uint32_t j = 0; j < fac; ++j)
        for (uint32_t i = 0; i < nsel; ++i) ring[(((i + j) * (i + j + 1)) / 2 + j) % size] = i;
    uint32_t cur = 0;
    for (uint32_t i = 0; i < size; ++i) {
        if (ring[i] != 0xffffffffu) cur = ring[i];
        out[i] = (uint8_t)cur;
    }
    return FCGPU_OK;
}

int fcgpu_set_lb_table(fcgpu_ctx *c, const uint8_t *table, uint32_t nbuckets) {
    if (!c) return FCGPU_EINVAL;
    if (!table || nbuckets == 0 || nbuckets > FCGPU_LB_TABLE_MAX) return fail(c, FCGPU_EINVAL, "bad LB table size");
    if (agg_queued(c)) return fail(c, FCGPU_EINVAL, "fcgpu_set_lb_table: a queued span submission is not waited for");
    // ((h >> 16) ^ (h & 0xffff)) < 65536: entries past 65535 are never read
    const uint32_t n = std::min(nbuckets, 65536u);
    uint32_t mx = 0;
    for (uint32_t k = 0; k < n; ++k) mx = std::max(mx, (uint32_t)table[k]);
    if (c->configured && mx >= c->cfg.nports) return fail(c, FCGPU_EINVAL, "LB table output >= nports");
    // k_rx copies whole uint4s of it into LDS: zero-padded to 16 B
    std::vector<uint8_t> dev((n + 15u) & ~15u, 0);
    memcpy(dev.data(), table, n);
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipDeviceSynchronize());
    hipFree(c->d_lbtab);
    c->d_lbtab = nullptr;
    HIPCHK(c, hipMalloc(&c->d_lbtab, dev.size()));
    HIPCHK(c, hipMemcpy(c->d_lbtab, dev.data(), dev.size(), hipMemcpyHostToDevice));
    c->lbtab_n = n;
    c->lbtab_max = mx;
    uint64_t key = 1469598103934665603ull;
    for (uint32_t k = 0; k < n; ++k) key = (key ^ table[k]) * 1099511628211ull;
    c->lbtab_key = (key ^ n) | 1;
    DevCfg &d = c->dcfg;
    d.lb_tab = c->cfg.classify == FCGPU_CLS_LB_TABLE ? c->d_lbtab : nullptr;
    d.lb_tab_n = n;
    d.lb_tab_magic = n > 1 ? (uint32_t)((((uint64_t)1 << 32) + n - 1) / n) : 0u;
    return FCGPU_OK;
}

int fcgpu_program_jit(fcgpu_ctx *c, int enable) {
    if (!c) return FCGPU_EINVAL;
    if (agg_queued(c)) return fail(c, FCGPU_EINVAL, "fcgpu_program_jit: a queued span submission is not waited for");
    c->jit_on = enable != 0;
    return jit_install(c);
}

int fcgpu_program_jit_active(fcgpu_ctx *c) { return c && !c->jit_src.empty() ? 1 : 0; }

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

// ---- flow re-shard across GPUs (fcgpu_exchange.hh) ---------------------------
int fcgpu_exchange_plan(fcgpu_ctx *c, const uint32_t *d_desc, const uint32_t *d_perm, const uint32_t *d_port_start,
                        uint32_t n, uint32_t world, uint32_t rank, fcgpu_xmeta *d_meta, uint64_t *d_seg_bytes,
                        void *stream) {
    if (!c) return FCGPU_EINVAL;
    if (world == 0 || world > FCGPU_MAX_PORTS) return fail(c, FCGPU_EINVAL, "fcgpu_exchange_plan: world must be 1..64");
    if (n > c->max_batch) return fail(c, FCGPU_ENOMEM, "fcgpu_exchange_plan: batch larger than the context's max_batch");
    if (!d_port_start || !d_seg_bytes || (n && (!d_desc || !d_perm || !d_meta)))
        return fail(c, FCGPU_EINVAL, "fcgpu_exchange_plan: null buffer");
    HIPCHK(c, hipSetDevice(c->device));
    const uint32_t nblk_max = (c->max_batch + kXItems - 1) / kXItems;
    if (!c->x_bsum) {
        HIPCHK(c, hipMalloc(&c->x_bsum, sizeof(unsigned long long) * (nblk_max + 1)));
        HIPCHK(c, hipMalloc(&c->x_base, sizeof(unsigned long long) * (FCGPU_MAX_PORTS + 1)));
        HIPCHK(c, hipMalloc(&c->x_part, sizeof(unsigned long long) * (FCGPU_MAX_PORTS + 1)));
        HIPCHK(c, hipMalloc(&c->x_src, sizeof(uint32_t) * ((size_t)c->max_batch + 1)));
    }
    hipStream_t s = static_cast<hipStream_t>(stream);
    XPlan P{};
    P.desc = d_desc;
    P.perm = d_perm;
    P.port_start = d_port_start;
    P.n = n;
    P.world = world;
    P.rank = rank;
    P.nblk = (n + kXItems - 1) / kXItems;
    P.meta = reinterpret_cast<uint4 *>(d_meta);
    P.bsum = c->x_bsum;
    P.base = c->x_base;
    P.part = c->x_part;
    P.src = c->x_src;
    P.seg_bytes = reinterpret_cast<unsigned long long *>(d_seg_bytes);
    if (P.nblk) hipLaunchKernelGGL(k_xsum, dim3(P.nblk), dim3(kXThreads), 0, s, P);
    hipLaunchKernelGGL(k_xscan, dim3(1), dim3(1024), 0, s, P);
    if (P.nblk) hipLaunchKernelGGL(k_xmeta, dim3(P.nblk), dim3(kXThreads), 0, s, P);
    HIPCHK(c, hipGetLastError());
    return FCGPU_OK;
}

int fcgpu_exchange_pack(fcgpu_ctx *c, const uint8_t *d_arena, const uint32_t *d_port_start,
                        const fcgpu_xmeta *d_meta, const uint64_t *d_seg_bytes, uint32_t n, uint32_t world,
                        uint8_t *d_send, uint64_t send_cap, void *stream) {
    if (!c) return FCGPU_EINVAL;
    if (world == 0 || world > FCGPU_MAX_PORTS) return fail(c, FCGPU_EINVAL, "fcgpu_exchange_pack: world must be 1..64");
    if (!d_port_start || !d_seg_bytes || (n && (!d_arena || !d_meta || (send_cap && !d_send))))
        return fail(c, FCGPU_EINVAL, "fcgpu_exchange_pack: null buffer");
    if (n > c->max_batch) return fail(c, FCGPU_ENOMEM, "fcgpu_exchange_pack: batch larger than the context's max_batch");
    if (n == 0) return FCGPU_OK;
    if (!c->x_src) return fail(c, FCGPU_EINVAL, "fcgpu_exchange_pack: no fcgpu_exchange_plan on this context");
    HIPCHK(c, hipSetDevice(c->device));
    XPack X{};
    X.arena = d_arena;
    X.src = c->x_src;
    X.port_start = d_port_start;
    X.meta = reinterpret_cast<const uint4 *>(d_meta);
    X.seg_bytes = reinterpret_cast<const unsigned long long *>(d_seg_bytes);
    X.send = d_send;
    X.send_cap = send_cap;
    X.n = n;
    X.world = world;
    // lanes per frame by the mean slot (send_cap / n): 16 B per lane per step
    hipStream_t s = static_cast<hipStream_t>(stream);
    const uint64_t mean = send_cap / n;
    if (mean <= 96)
        hipLaunchKernelGGL(k_xpack<4>, dim3((n + kXThreads / 4 - 1) / (kXThreads / 4)), dim3(kXThreads), 0, s, X);
    else if (mean <= 512)
        hipLaunchKernelGGL(k_xpack<16>, dim3((n + kXThreads / 16 - 1) / (kXThreads / 16)), dim3(kXThreads), 0, s, X);
    else
        hipLaunchKernelGGL(k_xpack<64>, dim3((n + kXThreads / 64 - 1) / (kXThreads / 64)), dim3(kXThreads), 0, s, X);
    HIPCHK(c, hipGetLastError());
    return FCGPU_OK;
}

int fcgpu_exchange_build(fcgpu_ctx *c, const uint8_t *d_arena, const uint32_t *d_desc, const uint16_t *d_verdict,
                         uint32_t n, uint32_t world, uint32_t rank, fcgpu_xmeta *d_meta, uint32_t *d_seg_n,
                         uint64_t *d_seg_bytes, uint8_t *d_send, uint64_t send_cap, void *stream) {
    if (!c) return FCGPU_EINVAL;
    if (world == 0 || world > FCGPU_MAX_PORTS) return fail(c, FCGPU_EINVAL, "fcgpu_exchange_build: world must be 1..64");
    if (n > c->max_batch) return fail(c, FCGPU_ENOMEM, "fcgpu_exchange_build: batch larger than the context's max_batch");
    if (!d_seg_n || !d_seg_bytes || (n && (!d_arena || !d_desc || !d_verdict || !d_meta || (send_cap && !d_send))))
        return fail(c, FCGPU_EINVAL, "fcgpu_exchange_build: null buffer");
    HIPCHK(c, hipSetDevice(c->device));
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (!c->x_tcnt) {
        HIPCHK(c, hipMalloc(&c->x_tcnt, sizeof(uint32_t) * (size_t)FCGPU_MAX_PORTS * c->max_tiles));
        HIPCHK(c, hipMalloc(&c->x_tbyt, sizeof(unsigned long long) * (size_t)FCGPU_MAX_PORTS * c->max_tiles));
    }
    XBuild B{};
    B.arena = d_arena;
    B.desc = d_desc;
    B.verdict = d_verdict;
    B.n = n;
    B.ntiles = (n + kXTile - 1) / kXTile;
    B.world = world;
    B.rank = rank;
    B.tcnt = c->x_tcnt;
    B.tbyt = c->x_tbyt;
    B.seg_n = d_seg_n;
    B.seg_bytes = reinterpret_cast<unsigned long long *>(d_seg_bytes);
    B.meta = reinterpret_cast<uint4 *>(d_meta);
    B.send = d_send;
    B.send_cap = send_cap;
    if (B.ntiles) hipLaunchKernelGGL(k_xbtile, dim3(B.ntiles), dim3(kXTile), 0, s, B);
    hipLaunchKernelGGL(k_xbscan, dim3(world), dim3(1024), 0, s, B);    // n = 0: zero counts
    if (B.ntiles) hipLaunchKernelGGL(k_xbuild, dim3(B.ntiles), dim3(kXTile), 0, s, B);   // lanes per frame: per tile
    HIPCHK(c, hipGetLastError());
    return FCGPU_OK;
}

int fcgpu_exchange_unpack(fcgpu_ctx *c, const fcgpu_xmeta *d_meta, uint32_t n, const uint64_t *src_displ,
                          uint32_t world, uint32_t *d_desc, void *stream) {
    if (!c) return FCGPU_EINVAL;
    if (world == 0 || world > FCGPU_MAX_PORTS) return fail(c, FCGPU_EINVAL, "fcgpu_exchange_unpack: world must be 1..64");
    if (!src_displ || (n && (!d_meta || !d_desc))) return fail(c, FCGPU_EINVAL, "fcgpu_exchange_unpack: null buffer");
    if (n == 0) return FCGPU_OK;
    HIPCHK(c, hipSetDevice(c->device));
    XUnpack U{};
    U.meta = reinterpret_cast<const uint4 *>(d_meta);
    U.desc = d_desc;
    U.n = n;
    U.world = world;
    for (uint32_t r = 0; r < world; ++r) U.displ[r] = src_displ[r];
    hipLaunchKernelGGL(k_xunpack, dim3((n + kXThreads - 1) / kXThreads), dim3(kXThreads), 0,
                       static_cast<hipStream_t>(stream), U);
    HIPCHK(c, hipGetLastError());
    return FCGPU_OK;
}

}  // extern "C"
