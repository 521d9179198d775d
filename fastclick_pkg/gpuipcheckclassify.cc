/*
 * gpuipcheckclassify.{cc,hh} -- the MI355X receive-path element for FastClick.
 * The element logic lives in fcx::RxCore (fastclick_amd/csrc/host/gpu_core.hh);
 * this file is the FastClick glue: configuration, per-thread state, the
 * Timer, handlers.
 */
#include <click/config.h>
#include "gpuipcheckclassify.hh"
#include <click/error.hh>
#include <click/glue.hh>
#include <click/bitvector.hh>
CLICK_DECLS

enum { h_count, h_drops, h_drop_details, h_port_counts, h_flow_count, h_flow_count_fids, h_flow_drops,
       h_gpu_errors, h_gpu_retries, h_error };

GPUIPCheckClassify::GPUIPCheckClassify() : _timer_us(100), _error_output(-1)
{
    in_batch_mode = BATCH_MODE_NEEDED;
}

GPUIPCheckClassify::~GPUIPCheckClassify()
{
}

int
GPUIPCheckClassify::configure(Vector<String> &conf, ErrorHandler *errh)
{
    // keyword arguments are parsed by the shared core (gpu_core.hh); a
    // throw-away core validates them here, each thread's core re-reads them
    _conf.clear();
    for (int i = 0; i < conf.size(); i++)
        _conf.push_back(std::string(conf[i].c_str()));
    Core probe;
    probe.name = std::string(name().c_str());
    std::string err;
    if (probe.configure(_conf, err) < 0)
        return errh->error("%s", err.c_str());
    _timer_us = probe.timer_us();
    _error_output = probe.error_output();
    return 0;
}

// Thread `thread`'s core: GPU context, staging slots, its Timer.
int
GPUIPCheckClassify::make_state(int thread, ErrorHandler *errh)
{
    State &s = _state.get_value_for_thread(thread);
    if (s.core)
        return 0;
    Core *c = new Core();
    c->name = std::string(name().c_str());
    std::string err;
    if (c->configure(_conf, err) < 0 || c->initialize(err) < 0) {
        delete c;
        if (errh)
            return errh->error("%s", err.c_str());
        click_chatter("%s", err.c_str());
        return -1;
    }
    s.core = c;
    if (_timer_us >= 0 || c->flow_timeouts()) {
        s.timer = new Timer(this);
        s.timer->initialize(this);
        s.timer->move_thread(thread);
    }
    return 0;
}

int
GPUIPCheckClassify::initialize(ErrorHandler *errh)
{
    // the failed batches' packets need an output that exists
    // (checked_output_push_batch would kill them uncounted)
    if (_error_output >= noutputs())
        return errh->error("ERROR_OUTPUT %d: the element has %d outputs", _error_output, noutputs());
    // a core for every thread that can push into this element
    Bitvector b = get_passing_threads();
    bool any = false;
    for (int i = 0; i < b.size(); i++)
        if (b[i]) {
            if (make_state(i, errh) < 0)
                return -1;
            any = true;
        }
    if (!any && make_state(home_thread_id(), errh) < 0)
        return -1;
    return 0;
}

void
GPUIPCheckClassify::cleanup(CleanupStage)
{
    for (unsigned i = 0; i < _state.weight(); i++) {
        State &s = _state.get_value_for_thread(i);
        if (s.timer) {
            s.timer->clear();
            delete s.timer;
            s.timer = 0;
        }
        delete s.core;          // kills what is still staged or in flight
        s.core = 0;
    }
}

// The timer covers what is staged (due TIMER us after its first packet),
// what is on the device, and (IMP timeouts) the next maintainer run.
inline void
GPUIPCheckClassify::arm(State &s)
{
    if (!s.timer)
        return;
    const uint64_t now = ClickPolicy::now_ns();
    uint64_t due = ~(uint64_t)0, m;
    if (_timer_us >= 0 && !s.core->idle())
        due = s.core->staged() ? s.core->due_ns() : now + (uint64_t)_timer_us * 1000;
    if (s.core->maint_due_ns(&m) && m < due)
        due = m;
    if (due == ~(uint64_t)0)
        return;
    if (due < now)
        due = now;
    // an earlier deadline than the one scheduled (a batch staged while the
    // timer waits for the next maintainer run) moves the timer up
    if (s.timer->scheduled() && (uint64_t)s.timer->expiry_steady().nsecval() <= due)
        return;
    s.timer->schedule_after(Timestamp::make_nsec((Timestamp::value_type)(due - now)));
}

void
GPUIPCheckClassify::push_batch(int, PacketBatch *batch)
{
    State &s = *_state;
    if (!s.core && make_state(click_current_cpu_id(), 0) < 0) {
        batch->kill();
        return;
    }
    s.core->push_list(batch->first(), Emit{this});
    arm(s);
}

void
GPUIPCheckClassify::push(int, Packet *p)
{
    State &s = *_state;
    if (!s.core && make_state(click_current_cpu_id(), 0) < 0) {
        p->kill();
        return;
    }
    p->set_next(0);
    s.core->push_one(p, Emit{this});
    arm(s);
}

void
GPUIPCheckClassify::run_timer(Timer *)
{
    State &s = *_state;
    if (!s.core)
        return;
    s.core->run_timer(ClickPolicy::now_ns(), Emit{this});
    arm(s);
}

String
GPUIPCheckClassify::read_handler(Element *e, void *thunk)
{
    GPUIPCheckClassify *g = static_cast<GPUIPCheckClassify *>(e);
    static const char *const names[] = {"count", "drops", "drop_details", "port_counts", "flow_count",
                                        "flow_count_fids", "flow_drops", "gpu_errors", "gpu_retries", "error"};
    // PER_THREAD_SUM (include/click/sync.hh:384): the per-thread cores'
    // counters are summed on read. Each core's counters and error are read
    // under that core's own lock (RxCore::counters), never racing the thread
    // that owns its GPU context.
    uint64_t sum[FCGPU_NCOUNTERS] = {0};
    Core::HostStats hsum;
    std::string error;
    uint32_t nports = 1;
    bool details = false;
    for (unsigned i = 0; i < g->_state.weight(); i++) {
        State &s = g->_state.get_value_for_thread(i);
        if (!s.core)
            continue;
        uint64_t c[FCGPU_NCOUNTERS];
        Core::HostStats hs;
        std::string e;
        s.core->counters(c, hs, &e);
        for (int k = 0; k < FCGPU_NCOUNTERS; k++)
            sum[k] += c[k];
        hsum += hs;
        nports = s.core->nports();
        details = s.core->details();
        if (error.empty())
            error = e;
    }
    const int h = (int)(uintptr_t)thunk;
    std::string out = Core::format_handler(names[h], sum, nports, details, hsum, error);
    return String(out.c_str());
}

void
GPUIPCheckClassify::add_handlers()
{
    add_read_handler("count", read_handler, h_count);
    add_read_handler("drops", read_handler, h_drops);
    add_read_handler("drop_details", read_handler, h_drop_details);
    add_read_handler("port_counts", read_handler, h_port_counts);
    add_read_handler("flow_count", read_handler, h_flow_count);
    add_read_handler("flow_count_fids", read_handler, h_flow_count_fids);
    add_read_handler("flow_drops", read_handler, h_flow_drops);
    add_read_handler("gpu_errors", read_handler, h_gpu_errors);
    add_read_handler("gpu_retries", read_handler, h_gpu_retries);
    add_read_handler("error", read_handler, h_error);
}

CLICK_ENDDECLS
ELEMENT_REQUIRES(batch)
ELEMENT_LIBS(-lfcgpu)
EXPORT_ELEMENT(GPUIPCheckClassify)
ELEMENT_MT_SAFE(GPUIPCheckClassify)
