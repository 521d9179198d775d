// fcgpu_launch.hip -- k_rx launches: one template instance of the kernel
// (fcgpu_device.hh) per configuration a context can take, chosen at run time
// (launch_rx_any), compiled programs through their hiprtc module
// (jit_function), and the host-side launch guard every launch passes
// (rx_launch_ok, fcgpu_launch_guard_selftest). The only unit that
// instantiates k_rx.
#include "fcgpu_internal.hh"

using namespace fcgpu;
using namespace fcgpu_rt;

namespace fcgpu_rt {

static_assert(kCrcTabQ <= kTile, "k_rx copies the CRC tables with one uint4 per thread");

// ev0/ev1 non-null: hipExtLaunchKernelGGL records them around the dispatch
// itself (timestamps of the kernel, not of the stream around it).
// L: one batch (njobs 1, grid = its tiles) or several fused ones (grid =
// their tiles end to end).

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
bool rx_launch_ok(int part, const RxLaunch &L, uint32_t grid) {
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

hipError_t launch_rx_any(int part, uint32_t cm, bool ck, const RxLaunch &L, uint32_t grid, hipStream_t s, hipEvent_t e0,
                          hipEvent_t e1, fcgpu_ctx *jc) {
    if (!rx_launch_ok(part, L, grid)) return hipErrorInvalidValue;
    if (L.A.cfg.classify == FCGPU_CLS_PROGRAM) launch_rx_prog<true>(part, cm, ck, L, grid, s, e0, e1, jc);
    else launch_rx_prog<false>(part, cm, ck, L, grid, s, e0, e1, jc);
    return hipSuccess;
}

// One batch: a.ntiles workgroups.
hipError_t launch_rx_one(int part, uint32_t cm, bool ck, const RxArgs &a, hipStream_t s, hipEvent_t e0,
                          hipEvent_t e1, fcgpu_ctx *jc) {
    RxLaunch L;
    L.A = a;
    L.njobs = 1;
    L.job_tiles = 0;
    return launch_rx_any(part, cm, ck, L, a.ntiles, s, e0, e1, jc);
}

hipError_t launch_rx_fn(hipFunction_t fn, int part, const RxLaunch &L, uint32_t grid, hipStream_t s) {
    if (!rx_launch_ok(part, L, grid)) return hipErrorInvalidValue;
    void *args[] = {const_cast<RxLaunch *>(&L)};
    return hipModuleLaunchKernel(fn, grid, 1, 1, kTile, 1, 1, 0, s, args, nullptr);
}

}  // namespace fcgpu_rt

extern "C" {

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

}  // extern "C"
