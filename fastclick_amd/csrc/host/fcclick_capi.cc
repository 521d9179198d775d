// fcclick_capi.cc -- C ABI of the host harness (include/fcclick.h).
#include <algorithm>
#include <chrono>
#include <thread>
#include <condition_variable>
#include <mutex>
#include <memory>
#include <string>
#include <vector>

#include "../../../include/fcclick.h"
#include "click_model.hh"
#include "gpu_element.hh"

using namespace fcx;

namespace {

// Records every packet that leaves the element on one output, then frees it.
class Sink : public Element {
  public:
    Sink(int port, fcclick_result *r, uint32_t *seq, uint32_t *nbatch, uint64_t *count = nullptr)
        : _port(port), _r(r), _seq(seq), _nbatch(nbatch), _count(count) {}
    const char *class_name() const override { return "Sink"; }
    int configure(const std::vector<std::string> &, std::string &) override { return 0; }
    void push_batch(int, PacketBatch *b) override {
        const uint32_t bi = (*_nbatch)++;
        unsigned cnt = 0;
        for (Packet *p = b->first(); p;) {
            Packet *nx = p->next();
            const uint32_t i = p->id;
            if (_r) {
                if (_r->out_port) _r->out_port[i] = (uint32_t)_port;
                if (_r->out_seq) _r->out_seq[i] = (*_seq);
                if (_r->out_batch) _r->out_batch[i] = bi;
                if (_r->out_agg) _r->out_agg[i] = p->anno_u32(AGGREGATE_ANNO_OFFSET);
                if (_r->out_dst) _r->out_dst[i] = p->anno_u32(DST_IP_ANNO_OFFSET);
                if (_r->out_len) _r->out_len[i] = p->length();
                if (_r->out_nh) _r->out_nh[i] = p->network_header_offset();
                if (_r->out_paint) _r->out_paint[i] = p->anno_u8(PAINT_ANNO_OFFSET);
                if (_r->out_flow) _r->out_flow[i] = p->anno_u32(28);
                if (_r->out_ip8 && p->network_header_offset() >= 0 &&
                    p->network_header_offset() + 12 <= (int)p->length()) {
                    uint32_t w;
                    memcpy(&w, p->data() + p->network_header_offset() + 8, 4);
                    _r->out_ip8[i] = w;
                }
            }
            ++*_seq;
            ++cnt;
            p->kill();
            p = nx;
        }
        if (cnt != b->count()) fprintf(stderr, "Sink: batch count %u != linked %u\n", b->count(), cnt);
        if (_count) *_count += cnt;
    }

  private:
    int _port;
    fcclick_result *_r;
    uint32_t *_seq, *_nbatch;
    uint64_t *_count;
};

// The harness floor: a BatchElement that forwards every PacketBatch to output
// 0 unchanged (what the source and sinks cost without the GPU element).
class Pass : public Element {
  public:
    const char *class_name() const override { return "Pass"; }
    int configure(const std::vector<std::string> &, std::string &) override { return 0; }
    void push_batch(int, PacketBatch *b) override { output_push_batch(0, b); }
    uint32_t max_held() const override { return 0; }
};

bool parse_element(const char *conf, std::string &cls, std::vector<std::string> &args, std::string &err) {
    std::string s = trim(conf ? conf : "");
    size_t lp = s.find('(');
    if (lp == std::string::npos) {
        cls = s;
        return !cls.empty();
    }
    if (s.back() != ')') {
        err = "syntax error: expected ')'";
        return false;
    }
    cls = trim(s.substr(0, lp));
    args = split_conf(s.substr(lp + 1, s.size() - lp - 2));
    return true;
}

std::unique_ptr<Element> make_element(const char *conf, std::string &err) {
    std::string cls;
    std::vector<std::string> args;
    if (!parse_element(conf, cls, args, err)) {
        if (err.empty()) err = "empty configuration";
        return nullptr;
    }
    std::unique_ptr<Element> e;
    if (cls == "GPUIPCheckClassify") e.reset(new GPUIPCheckClassify());
    else if (cls == "Pass") e.reset(new Pass());
    else {
        err = "unknown element class '" + cls + "'";
        return nullptr;
    }
    if (e->configure(args, err) < 0) return nullptr;
    return e;
}

void copy_err(const std::string &m, char *err, size_t cap) {
    if (err && cap) {
        snprintf(err, cap, "%s", m.c_str());
    }
}

uint32_t max_len(const uint32_t *desc, uint32_t n) {
    uint32_t m = 64;
    for (uint32_t i = 0; i < n; ++i) m = desc[2 * i + 1] > m ? desc[2 * i + 1] : m;
    return m;
}

}  // namespace

extern "C" int fcclick_check_config(const char *conf, char *err, size_t errcap) {
    std::string e;
    auto el = make_element(conf, e);
    if (!el) {
        copy_err(e, err, errcap);
        return -1;
    }
    return 0;
}

extern "C" int fcclick_element_cfg(const char *conf, fcgpu_cfg *cfg, char *err, size_t errcap) {
    if (!conf || !cfg) {
        copy_err("null argument", err, errcap);
        return -1;
    }
    std::string e;
    auto el = make_element(conf, e);
    if (!el) {
        copy_err(e, err, errcap);
        return -1;
    }
    auto *g = dynamic_cast<GPUIPCheckClassify *>(el.get());
    if (!g) {
        copy_err("not a GPUIPCheckClassify", err, errcap);
        return -1;
    }
    *cfg = g->device_cfg();
    return 0;
}

extern "C" int fcclick_parse_program(const char *text, fcgpu_step *steps, uint32_t cap, uint32_t *nsteps,
                                     int32_t *output_everything, char *err, size_t errcap) {
    if (!text || !nsteps || !output_everything) {
        copy_err("null argument", err, errcap);
        return -1;
    }
    fcx::ParsedProgram pr;
    std::string e = fcx::parse_program(text, pr);
    if (e.empty() && pr.steps.size() > cap) e = "program longer than cap";
    if (!e.empty()) {
        copy_err(e, err, errcap);
        return -1;
    }
    for (size_t i = 0; i < pr.steps.size(); ++i) steps[i] = pr.steps[i];
    *nsteps = (uint32_t)pr.steps.size();
    *output_everything = pr.output_everything;
    return 0;
}

static int run_graph(const char *conf, const uint8_t *arena, const uint32_t *desc, uint32_t n, uint32_t burst,
                     uint32_t nsinks, uint32_t flags, const uint64_t *burst_ns, fcclick_result *res, char *err,
                     size_t errcap, const fcclick_event *ev = nullptr, uint32_t nev = 0, char *reads = nullptr,
                     size_t reads_cap = 0);

static const char *const kHandlerNames[] = {"count",      "drops",           "drop_details", "port_counts",
                                            "flow_count", "flow_count_fids", "flow_drops",   "gpu_errors",
                                            "gpu_retries", "error"};
static std::string read_all(Element *el) {
    std::string h;
    for (const char *name : kHandlerNames) h += std::string(name) + "=" + el->read_handler(name) + "\n";
    return h;
}

extern "C" int fcclick_run_ex(const char *conf, const uint8_t *arena, const uint32_t *desc, uint32_t n,
                              uint32_t burst, uint32_t nsinks, uint32_t flags, fcclick_result *res, char *err,
                              size_t errcap) {
    return run_graph(conf, arena, desc, n, burst, nsinks, flags, nullptr, res, err, errcap);
}

extern "C" int fcclick_run_clocked(const char *conf, const uint8_t *arena, const uint32_t *desc, uint32_t n,
                                   uint32_t burst, uint32_t nsinks, const uint64_t *burst_ns, fcclick_result *res,
                                   char *err, size_t errcap) {
    if (!burst_ns) return -1;
    const int rc = run_graph(conf, arena, desc, n, burst, nsinks, 0, burst_ns, res, err, errcap);
    ModelPolicy::virtual_ns.store(0);
    return rc;
}

extern "C" int fcclick_run_events(const char *conf, const uint8_t *arena, const uint32_t *desc, uint32_t n,
                                  uint32_t nsinks, const fcclick_event *ev, uint32_t nev, fcclick_result *res,
                                  char *reads, size_t reads_cap, char *err, size_t errcap) {
    if (!ev || !nev) {
        copy_err("no events", err, errcap);
        return -1;
    }
    uint64_t total = 0;
    for (uint32_t k = 0; k < nev; ++k) {
        if (ev[k].kind != FCCLICK_EV_BURST && ev[k].kind != FCCLICK_EV_READ) {
            copy_err("unknown event kind", err, errcap);
            return -1;
        }
        if (ev[k].kind == FCCLICK_EV_BURST) {
            if (!ev[k].count) {
                copy_err("an empty burst", err, errcap);
                return -1;
            }
            total += ev[k].count;
        }
    }
    if (total != n) {
        copy_err("the bursts do not cover the n packets exactly", err, errcap);
        return -1;
    }
    const int rc = run_graph(conf, arena, desc, n, 0, nsinks, 0, nullptr, res, err, errcap, ev, nev, reads, reads_cap);
    ModelPolicy::virtual_ns.store(0);
    return rc;
}

static int run_graph(const char *conf, const uint8_t *arena, const uint32_t *desc, uint32_t n, uint32_t burst,
                     uint32_t nsinks, uint32_t flags, const uint64_t *burst_ns, fcclick_result *res, char *err,
                     size_t errcap, const fcclick_event *ev, uint32_t nev, char *reads, size_t reads_cap) {
    std::string e;
    auto el = make_element(conf, e);
    if (!el || el->initialize(e) < 0) {
        copy_err(e, err, errcap);
        return -1;
    }
    const bool per_packet = burst == FCCLICK_PER_PACKET;
    if (burst == 0) burst = 32;
    if (per_packet) burst = 32;
    uint32_t seq = 0, nbatch = 0;
    if (res) {
        for (uint32_t i = 0; i < n; ++i) {
            if (res->out_port) res->out_port[i] = 0xffffffffu;
            if (res->out_seq) res->out_seq[i] = 0xffffffffu;
            if (res->out_batch) res->out_batch[i] = 0xffffffffu;
        }
    }
    std::vector<std::unique_ptr<Sink>> sinks;
    for (uint32_t k = 0; k < nsinks; ++k) {
        sinks.emplace_back(new Sink((int)k, res, &seq, &nbatch));
        el->connect_output((int)k, sinks.back().get(), 0);
    }
    const uint32_t headroom = 128;
    PacketPool pool(n ? n : 1, headroom + max_len(desc, n) + 64, headroom);
    // FromDPDKDevice-style source: BURST packets per PacketBatch -- or the
    // events' bursts, with handler reads between them
    std::vector<fcclick_event> evs;
    if (ev) {
        evs.assign(ev, ev + nev);
    } else {
        for (uint32_t i = 0; i < n; i += burst)
            evs.push_back(fcclick_event{burst_ns ? burst_ns[i / burst] : 0, FCCLICK_EV_BURST,
                                        n - i < burst ? n - i : burst});
    }
    std::string rd;
    uint32_t i = 0;
    for (const fcclick_event &e : evs) {
        if (ev && e.t_ns) ModelPolicy::virtual_ns.store(e.t_ns);
        else if (burst_ns) ModelPolicy::virtual_ns.store(e.t_ns ? e.t_ns : 1);
        if (e.kind == FCCLICK_EV_READ) {
            // the element's Timer fires at this time (the maintainer runs due,
            // a partial batch due), then every handler is read
            el->run_timer(ModelPolicy::now_ns());
            rd += read_all(el.get()) + "--\n";
            continue;
        }
        const uint32_t m = e.count;
        Packet *head = nullptr, *prev = nullptr;
        for (uint32_t j = 0; j < m; ++j) {
            Packet *p = pool.make(arena + desc[2 * (i + j)], desc[2 * (i + j) + 1]);
            p->id = i + j;
            if (prev) prev->set_next(p);
            else head = p;
            prev = p;
        }
        if (per_packet)
            for (Packet *p = head, *nx; p; p = nx) {
                nx = p->next();
                p->set_next(nullptr);
                el->push(0, p);
            }
        else
            el->push_batch(0, PacketBatch::make_from_list(head, prev, m));
        i += m;
    }
    if (reads && reads_cap) snprintf(reads, reads_cap, "%s", rd.c_str());
    if (flags & FCCLICK_TIMER_FLUSH) {
        // the source has stopped: only the element's Timer can release what it
        // still holds (MinBatch's timer, minbatch.cc:35,57-76)
        auto now = []() {
            return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                       std::chrono::steady_clock::now().time_since_epoch()).count();
        };
        if (res && res->out_parked) *res->out_parked = el->held();
        for (int k = 0; k < 100000 && el->run_timer(now()); ++k)
            std::this_thread::sleep_for(std::chrono::microseconds(20));
    } else {
        el->flush();
    }
    if (res) {
        if (res->out_batches) *res->out_batches = nbatch;
        if (res->handlers && res->handlers_cap)
            snprintf(res->handlers, res->handlers_cap, "%s", read_all(el.get()).c_str());
    }
    std::string er = el->read_handler("error");
    // what the element still holds (TIMER -1 and no flush) is killed back into
    // the pool: the element goes before the pool does
    el.reset();
    if (!er.empty()) {
        copy_err(er, err, errcap);
        return -2;
    }
    return 0;
}

// The element's compact staging of a batch (capture.hh), for tests: records
// of the bytes the configured chain reads, as RxCore stages them.
extern "C" int fcclick_stage_compact(const char *conf, const uint8_t *arena, const uint32_t *desc, uint32_t n,
                                     uint8_t *out_arena, size_t out_cap, uint32_t *out_desc, size_t *out_bytes,
                                     char *err, size_t errcap) {
    std::string e;
    std::string cls;
    std::vector<std::string> args;
    if (!parse_element(conf, cls, args, e) || cls != "GPUIPCheckClassify") {
        copy_err(e.empty() ? "not a GPUIPCheckClassify configuration" : e, err, errcap);
        return -1;
    }
    RxCore<ModelPolicy> core;
    if (core.configure(args, e) < 0) {
        copy_err(e, err, errcap);
        return -1;
    }
    const fcgpu_cfg &cfg = core.device_cfg();
    const fcgpu::StagePlan plan = fcgpu::stage_plan(cfg);
    if (!plan.compact) {
        copy_err("this chain stages whole captures (no compact records)", err, errcap);
        return -2;
    }
    size_t used = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const uint8_t *f = arena + desc[2 * i];
        const uint32_t len = desc[2 * i + 1];
        uint32_t so, cp;
        const uint32_t rec = fcgpu::stage_record_size(plan, (uint32_t)cfg.offset, f, len, so, cp);
        if (fcgpu::kStageLead + used + rec > out_cap) {
            copy_err("out_arena too small", err, errcap);
            return -1;
        }
        memcpy(out_arena + fcgpu::kStageLead + used, f + so, cp);
        out_desc[2 * i] = (uint32_t)(fcgpu::kStageLead + used) - plan.start;
        out_desc[2 * i + 1] = len;
        used += rec;
    }
    if (out_bytes) *out_bytes = fcgpu::kStageLead + used;
    return 0;
}

extern "C" int fcclick_run(const char *conf, const uint8_t *arena, const uint32_t *desc, uint32_t n,
                           uint32_t burst, uint32_t nsinks, fcclick_result *res, char *err, size_t errcap) {
    return fcclick_run_ex(conf, arena, desc, n, burst, nsinks, 0, res, err, errcap);
}

namespace {
// Every thread's timed loop starts together: after each has set up its
// element (GPU context, pinned staging, possibly hiprtc) and run its warm-up.
struct StartLine {
    std::mutex mu;
    std::condition_variable cv;
    uint32_t waiting = 0, parties = 1;
    void arrive() {
        std::unique_lock<std::mutex> g(mu);
        if (++waiting >= parties) cv.notify_all();
        else cv.wait(g, [this] { return waiting >= parties; });
    }
};
using Clock = std::chrono::steady_clock;

// One element instance (its own GPU context, like one Click thread) pushed
// `reps` times through the trace; returns packets per second, or < 0. With a
// start line, the timed loop begins once every thread has reached it (a
// thread that fails still arrives), and [t_beg, t_end] is its timed window.
// With `stop`, the timed loop runs whole passes over the trace until *stop is
// set (reps ignored) and *done gets the packets pushed -- a source that keeps
// pushing for a fixed time, as the CPU baseline's threads do.
double bench_one(const char *conf, const uint8_t *arena, const uint32_t *desc, uint32_t n, uint32_t burst,
                 uint32_t reps, std::string &e, StartLine *line = nullptr, Clock::time_point *t_beg = nullptr,
                 Clock::time_point *t_end = nullptr, const std::atomic<bool> *stop = nullptr,
                 uint64_t *done = nullptr) {
    auto el = make_element(conf, e);
    if (!el || el->initialize(e) < 0) {
        if (line) line->arrive();
        return -1.0;
    }
    const bool per_packet = burst == FCCLICK_PER_PACKET;
    if (burst == 0) burst = 32;
    if (per_packet) burst = 32;
    uint32_t seq = 0, nbatch = 0;
    std::vector<std::unique_ptr<Sink>> sinks;
    for (uint32_t k = 0; k < 65; ++k) {
        sinks.emplace_back(new Sink((int)k, nullptr, &seq, &nbatch));
        el->connect_output((int)k, sinks.back().get(), 0);
    }
    // a DPDK-style mempool: as many packets as the element can hold plus the
    // bursts in flight, recycled LIFO (packets freed by the sinks are reused
    // first, as a mempool's per-core cache does) -- not one packet per frame
    const uint32_t headroom = 128;
    const uint32_t pool_n = std::max<uint32_t>(4096, el->max_held() + 4 * burst + 4096);
    PacketPool pool(pool_n, headroom + max_len(desc, n) + 64, headroom);
    // one pass of the source over the trace; the element drains only at the
    // end of the timed loop (a source that keeps pushing never flushes it)
    auto one = [&]() {
        for (uint32_t i = 0; i < n; i += burst) {
            uint32_t m = n - i < burst ? n - i : burst;
            if (pool.available() < m) el->flush();      // never expected: the pool covers max_held
            Packet *head = nullptr, *prev = nullptr;
            for (uint32_t j = 0; j < m; ++j) {
                Packet *p = pool.make(arena + desc[2 * (i + j)], desc[2 * (i + j) + 1]);
                if (prev) prev->set_next(p);
                else head = p;
                prev = p;
            }
            if (per_packet)
                for (Packet *p = head, *nx; p; p = nx) {
                    nx = p->next();
                    p->set_next(nullptr);
                    el->push(0, p);
                }
            else
                el->push_batch(0, PacketBatch::make_from_list(head, prev, m));
        }
    };
    one();   // warm-up (allocations, first launch)
    el->flush();
    if (line) line->arrive();
    auto t0 = Clock::now();
    uint64_t passes = 0;
    if (stop) {
        while (!stop->load(std::memory_order_relaxed)) {
            one();
            ++passes;
        }
    } else {
        for (uint32_t r = 0; r < reps; ++r) one();
        passes = reps;
    }
    el->flush();
    auto t1 = Clock::now();
    if (t_beg) *t_beg = t0;
    if (t_end) *t_end = t1;
    if (done) *done = passes * n;
    const double s = std::chrono::duration<double>(t1 - t0).count();
    e = el->read_handler("error");
    el.reset();                      // before the pool its packets belong to
    if (!e.empty()) return -2.0;
    return (double)n * passes / s;
}
}  // namespace

extern "C" int fcclick_bench(const char *conf, const uint8_t *arena, const uint32_t *desc, uint32_t n,
                             uint32_t burst, uint32_t reps, double *pps, char *err, size_t errcap) {
    std::string e;
    const double r = bench_one(conf, arena, desc, n, burst, reps, e);
    if (r < 0) {
        copy_err(e, err, errcap);
        return r == -1.0 ? -1 : -2;
    }
    if (pps) *pps = r;
    return 0;
}

// T element threads pushing for `seconds` (every thread set up and warmed up
// first): packets of all threads over the union of their windows, each window
// ending at the first pass boundary after the stop plus the final flush.
extern "C" int fcclick_bench_timed(const char *conf, const uint8_t *arena, const uint32_t *desc, uint32_t n,
                                   uint32_t burst, double seconds, uint32_t threads, double *pps, char *err,
                                   size_t errcap) {
    if (threads == 0) threads = 1;
    if (!(seconds > 0)) {
        copy_err("seconds must be > 0", err, errcap);
        return -1;
    }
    std::vector<double> r(threads, 0.0);
    std::vector<std::string> es(threads);
    std::vector<Clock::time_point> beg(threads), end(threads);
    std::vector<uint64_t> cnt(threads, 0);
    std::atomic<bool> stop{false};
    std::vector<std::thread> th;
    StartLine line;
    line.parties = threads + 1;                   // the threads and this timer
    for (uint32_t t = 0; t < threads; ++t)
        th.emplace_back([&, t]() {
            r[t] = bench_one(conf, arena, desc, n, burst, 0, es[t], &line, &beg[t], &end[t], &stop, &cnt[t]);
        });
    line.arrive();
    std::this_thread::sleep_for(std::chrono::duration<double>(seconds));
    stop.store(true, std::memory_order_relaxed);
    for (auto &x : th) x.join();
    for (uint32_t t = 0; t < threads; ++t)
        if (r[t] < 0) {
            copy_err(es[t], err, errcap);
            return r[t] == -1.0 ? -1 : -2;
        }
    Clock::time_point b = beg[0], e = end[0];
    uint64_t total = 0;
    for (uint32_t t = 0; t < threads; ++t) {
        b = std::min(b, beg[t]);
        e = std::max(e, end[t]);
        total += cnt[t];
    }
    const double s = std::chrono::duration<double>(e - b).count();
    if (pps) *pps = s > 0 ? (double)total / s : 0.0;
    return 0;
}

extern "C" int fcclick_bench_threads(const char *conf, const uint8_t *arena, const uint32_t *desc, uint32_t n,
                                     uint32_t burst, uint32_t reps, uint32_t threads, double *pps, char *err,
                                     size_t errcap) {
    if (threads == 0) threads = 1;
    std::vector<double> r(threads, 0.0);
    std::vector<std::string> es(threads);
    std::vector<Clock::time_point> beg(threads), end(threads);
    std::vector<std::thread> th;
    StartLine line;
    line.parties = threads;
    for (uint32_t t = 0; t < threads; ++t)
        th.emplace_back([&, t]() { r[t] = bench_one(conf, arena, desc, n, burst, reps, es[t], &line, &beg[t], &end[t]); });
    for (auto &x : th) x.join();
    for (uint32_t t = 0; t < threads; ++t)
        if (r[t] < 0) {
            copy_err(es[t], err, errcap);
            return r[t] == -1.0 ? -1 : -2;
        }
    // aggregate: every thread's packets over the union of the timed windows
    // (earliest start to latest end), not the sum of per-thread rates
    Clock::time_point b = beg[0], e = end[0];
    for (uint32_t t = 1; t < threads; ++t) {
        b = std::min(b, beg[t]);
        e = std::max(e, end[t]);
    }
    const double s = std::chrono::duration<double>(e - b).count();
    if (pps) *pps = s > 0 ? (double)n * reps * threads / s : 0.0;
    return 0;
}

extern "C" int fcclick_run_threads(const char *conf, const uint8_t *arena, const uint32_t *desc, uint32_t n,
                                   uint32_t burst, uint32_t reps, uint32_t threads, uint32_t nsinks,
                                   uint64_t *port_pkts, char *handlers, size_t handlers_cap, char *err,
                                   size_t errcap) {
    if (threads == 0 || !port_pkts || nsinks == 0) {
        copy_err("threads, nsinks and port_pkts are required", err, errcap);
        return -1;
    }
    if (burst == 0) burst = 32;
    std::vector<std::string> es(threads), hs(threads);
    std::vector<int> rc(threads, 0);
    std::vector<std::thread> th;
    StartLine line;
    line.parties = threads;
    for (uint32_t t = 0; t < threads; ++t)
        th.emplace_back([&, t]() {
            auto el = make_element(conf, es[t]);
            if (!el || el->initialize(es[t]) < 0) {
                rc[t] = -1;
                line.arrive();
                return;
            }
            uint32_t seq = 0, nbatch = 0;
            uint64_t *cnt = port_pkts + (size_t)t * nsinks;
            std::vector<std::unique_ptr<Sink>> sinks;
            for (uint32_t k = 0; k < nsinks; ++k) {
                cnt[k] = 0;
                sinks.emplace_back(new Sink((int)k, nullptr, &seq, &nbatch, cnt + k));
                el->connect_output((int)k, sinks.back().get(), 0);
            }
            const uint32_t headroom = 128;
            PacketPool pool(std::max<uint32_t>(4096, el->max_held() + 4 * burst + 4096),
                            headroom + max_len(desc, n) + 64, headroom);
            line.arrive();                    // every thread's context exists: the run starts together
            for (uint32_t r = 0; r < reps; ++r)
                for (uint32_t i = 0; i < n; i += burst) {
                    const uint32_t m = n - i < burst ? n - i : burst;
                    if (pool.available() < m) el->flush();
                    Packet *head = nullptr, *prev = nullptr;
                    for (uint32_t j = 0; j < m; ++j) {
                        Packet *p = pool.make(arena + desc[2 * (i + j)], desc[2 * (i + j) + 1]);
                        if (prev) prev->set_next(p);
                        else head = p;
                        prev = p;
                    }
                    el->push_batch(0, PacketBatch::make_from_list(head, prev, m));
                }
            el->flush();
            hs[t] = read_all(el.get());
            el.reset();                       // before the pool its packets belong to
        });
    for (auto &x : th) x.join();
    for (uint32_t t = 0; t < threads; ++t)
        if (rc[t] < 0) {
            copy_err(es[t], err, errcap);
            return -1;
        }
    std::string all;
    for (uint32_t t = 0; t < threads; ++t) all += hs[t] + "--\n";
    if (handlers && handlers_cap) snprintf(handlers, handlers_cap, "%s", all.c_str());
    return 0;
}
