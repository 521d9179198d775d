// fcgpu_internal.hh -- what the translation units of libfcgpu.so share: the
// context (struct fcgpu_ctx, the opaque handle of include/fastclick_gpu.h),
// its slot and queue records, and the host helpers one unit defines and
// others call (namespace fcgpu_rt). Host code only; the kernels each unit
// launches come from the device header it alone includes:
//   fcgpu_launch.hip        k_rx instantiations (fcgpu_device.hh)
//   fcgpu_process.hip       whole-batch partition scan/scatter, mbuf
//                           descriptors (fcgpu_part.hh)
//   fcgpu_flow_api.hip      new-flow passes, maintainer (fcgpu_flow.hh)
//   fcgpu_exchange_api.hip  flow re-shard (fcgpu_exchange.hh)
// and the units without kernels:
//   fcgpu_context.hip       open / configure / close, counters, timing,
//                           errors, fault injection, host memory
//   fcgpu_program.hip       decision programs, LB tables, compiled programs
//   fcgpu_span.hip          span and block submissions, the shared
//                           zero-copy queue of FCGPU_SPAN_AUTO
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>
#include <string.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <map>
#include <mutex>
#include <initializer_list>
#include <string>
#include <thread>
#include <vector>

#include "fcgpu_device.hh"
#include "capture.hh"
#include "prog_jit.hh"

#pragma clang diagnostic ignored "-Wunused-result"
#pragma clang diagnostic ignored "-Wunused-value"

namespace fcgpu_rt {
using namespace fcgpu;

static_assert(kTile == FCGPU_TILE, "tile size is part of the ABI");
constexpr size_t kCtrWords = (size_t)FCGPU_CTR_SHARDS * FCGPU_NCOUNTERS;
struct AggQueue;              // fcgpu_span.hip
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
    // issued it (outside the queue's lock), then kAggIssued or kAggFailed;
    // owners waiting for that sleep on the queue's condition variable
    std::atomic<int> state{0};
    // where the issuing thread is (kAggPhase*), for the wait's watchdog report
    std::atomic<int> phase{0};
};
constexpr int kAggPhaseTaken = 0, kAggPhaseLaunch = 1, kAggPhaseRecord = 2;
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
    bool reserved = false;       // fcgpu_span_reserve sized d_in / d_res: never regrown on submission
    bool doomed = false;         // fcgpu_inject_fault(FCGPU_FAULT_WAIT): accepted, nothing ran, the wait fails
    hipEvent_t done = nullptr;   // shared streams: the slot's last operation (else the stream is waited)
    bool evt = false;            // the last submission recorded `done`
};

inline uint32_t span(uint32_t n, uint32_t part, uint32_t np) { return (uint32_t)((uint64_t)n * part / np); }

inline bool host_pinned(const void *p) {
    if (!p) return false;
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return at.type == hipMemoryTypeHost;
}
}  // namespace fcgpu_rt

using namespace fcgpu;

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
    fcgpu_rt::HostSlot slot[fcgpu_rt::kSlots];
    uint32_t slot_cap = 0;
    fcgpu_rt::Pool pool;
    // fcgpu_span_submit slots
    fcgpu_rt::SpanSlot span[FCGPU_SPAN_SLOTS];
    int span_index = -1;              // FCGPU_SPAN_STREAMS=shared:N: this context's place in the pool
    uint32_t span_mode = FCGPU_SPAN_COPY;   // fcgpu_span_mode: block submissions copied or read in place
    fcgpu_rt::AggQueue *aq = nullptr;          // the device's shared queue (FCGPU_SPAN_AUTO), once used
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
    std::vector<fcgpu_rt::EvPair> pending;
    std::vector<hipEvent_t> free_ev;
    // flow re-shard plan (fcgpu_exchange_plan): block sums and segment starts
    unsigned long long *x_bsum = nullptr, *x_base = nullptr, *x_part = nullptr;
    uint32_t *x_src = nullptr;   // arena offset of each leaving frame (plan -> pack)
    uint32_t *x_tcnt = nullptr;               // fcgpu_exchange_build: [64][max_tiles] per tile and owner
    unsigned long long *x_tbyt = nullptr;
    uint32_t *x_segn = nullptr;               // fcgpu_exchange_build_fixed: per-owner totals (scratch)
    unsigned long long *x_segb = nullptr;
    std::string err;
};

namespace fcgpu_rt {

// ---- fcgpu_context.hip ------------------------------------------------------
extern std::string g_open_err;     // fcgpu_last_error(NULL): errors without a context
int fail(fcgpu_ctx *c, int code, const std::string &msg);
hipError_t memset_sync(void *p, int v, size_t bytes);
hipEvent_t take_event(fcgpu_ctx *c);
uint32_t host_capture(const fcgpu_ctx *c);
bool fault_take(uint32_t where);

// Device and pinned scratch made after fcgpu_open (lazily, or at a
// reconfiguration), all or nothing: a group's buffers are allocated in order
// and, at the first failure, the ones made are freed and every pointer of the
// group is null again -- the guard that skips a group next time never sees a
// partial set, so a failed call returns its error and the next one retries
// instead of launching on a null or stale pointer. Every allocation is one
// FCGPU_FAULT_ALLOC event. The group's pointers must be null on entry.
struct Scratch {
    void **p;
    size_t bytes;
    uint8_t kind;        // 0 device, 1 device zero-filled, 2 pinned host
};
template <class T> inline Scratch dev_buf(T *&p, size_t bytes, bool zero = false) {
    return Scratch{reinterpret_cast<void **>(&p), bytes, static_cast<uint8_t>(zero ? 1 : 0)};
}
template <class T> inline Scratch pinned_buf(T *&p, size_t bytes) {
    return Scratch{reinterpret_cast<void **>(&p), bytes, 2};
}
hipError_t alloc_group(std::initializer_list<Scratch> g);
// alloc_group, and on failure fail(c, FCGPU_ENOMEM / FCGPU_ERUNTIME, what: ...)
int alloc_or_fail(fcgpu_ctx *c, const char *what, std::initializer_list<Scratch> g);
// one device allocation that counts as a FCGPU_FAULT_ALLOC event
hipError_t dev_malloc(void **p, size_t bytes);
template <class T> inline hipError_t dev_malloc(T **p, size_t bytes) {
    return dev_malloc(reinterpret_cast<void **>(p), bytes);
}

#define HIPCHK(ctx, expr)                                                                   \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess)                                                               \
            return ::fcgpu_rt::fail((ctx), FCGPU_ERUNTIME,                                  \
                                    std::string(#expr) + ": " + hipGetErrorString(e_));     \
    } while (0)

// ---- fcgpu_program.hip ------------------------------------------------------
hipFunction_t jit_function(fcgpu_ctx *c, int key);

// ---- fcgpu_launch.hip -------------------------------------------------------
bool rx_launch_ok(int part, const RxLaunch &L, uint32_t grid);
hipError_t launch_rx_any(int part, uint32_t cm, bool ck, const RxLaunch &L, uint32_t grid, hipStream_t s,
                         hipEvent_t e0, hipEvent_t e1, fcgpu_ctx *jc);
hipError_t launch_rx_one(int part, uint32_t cm, bool ck, const RxArgs &a, hipStream_t s, hipEvent_t e0,
                         hipEvent_t e1, fcgpu_ctx *jc);
hipError_t launch_rx_fn(hipFunction_t fn, int part, const RxLaunch &L, uint32_t grid, hipStream_t s);

// ---- fcgpu_process.hip ------------------------------------------------------
int check_process(fcgpu_ctx *c, const uint8_t *d_arena, const uint32_t *d_desc, uint32_t n, const fcgpu_out *o);
// n_dev: a counted batch (fcgpu_process_counted): n is the bound, the packets
// processed the first *n_dev - n_base
int process_one(fcgpu_ctx *c, const uint8_t *d_arena, const uint32_t *d_desc, uint32_t n, const fcgpu_out *o,
                hipStream_t s, uint32_t layout = 0, const uint32_t *n_dev = nullptr, uint32_t n_base = 0);
int out_part(const fcgpu_out *o);
void pool_release(fcgpu_ctx *c);

// ---- fcgpu_span.hip ---------------------------------------------------------
void span_auto_count(fcgpu_ctx *c, uint32_t new_mode);
bool span_zerocopy(const fcgpu_ctx *c);
bool agg_queued(const fcgpu_ctx *c);

// ---- fcgpu_flow_api.hip -----------------------------------------------------
void flow_free(fcgpu_ctx *c);
hipError_t flow_pass(fcgpu_ctx *c, const FlowArgs &F, uint32_t n, hipStream_t s);
// the new-flow passes of the g batches of one fused k_rx launch, in batch
// order (F: the launch's flow arguments; batch k's miss records at k * stride
// / k * words, its epoch epoch0 + k)
hipError_t flow_pass_fused(fcgpu_ctx *c, const FlowArgs &F, uint32_t g, const uint32_t *n,
                           uint32_t *const *flowid, uint32_t stride, uint32_t words, uint32_t epoch0, hipStream_t s);

}  // namespace fcgpu_rt
