// fcgpu_exchange_api.hip -- the flow re-shard across GPUs (SURVEY 8(f) #1 x
// (e), fcgpu_exchange.hh): plan / pack (the counted exchange of a
// partitioned batch), build (owner pass + send records in one sequence of
// launches) and unpack (descriptors over the received arena).
#include "fcgpu_internal.hh"
#include "fcgpu_exchange.hh"

using namespace fcgpu;
using namespace fcgpu_rt;

extern "C" {

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
        const int rc = alloc_or_fail(c, "fcgpu_exchange_plan scratch",
                                     {dev_buf(c->x_bsum, sizeof(unsigned long long) * (nblk_max + 1)),
                                      dev_buf(c->x_base, sizeof(unsigned long long) * (FCGPU_MAX_PORTS + 1)),
                                      dev_buf(c->x_part, sizeof(unsigned long long) * (FCGPU_MAX_PORTS + 1)),
                                      dev_buf(c->x_src, sizeof(uint32_t) * ((size_t)c->max_batch + 1))});
        if (rc != FCGPU_OK) return rc;
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

// The build's per-tile scratch ([64][max_tiles] counts and bytes) and the
// per-owner totals: allocated together on first use, or not at all (a failed
// allocation leaves none, so the next call allocates again instead of
// launching with a null one).
static int xbuild_scratch(fcgpu_ctx *c) {
    if (c->x_tcnt) return FCGPU_OK;         // the group is all or nothing
    return alloc_or_fail(c, "fcgpu_exchange_build scratch",
                         {dev_buf(c->x_tcnt, sizeof(uint32_t) * (size_t)FCGPU_MAX_PORTS * c->max_tiles),
                          dev_buf(c->x_tbyt, sizeof(unsigned long long) * (size_t)FCGPU_MAX_PORTS * c->max_tiles),
                          dev_buf(c->x_segn, sizeof(uint32_t) * FCGPU_MAX_PORTS),
                          dev_buf(c->x_segb, sizeof(unsigned long long) * FCGPU_MAX_PORTS)});
}

// k_xbtile -> k_xbscan -> k_xbuild over B (counted or fixed layout).
static int xbuild_launch(fcgpu_ctx *c, XBuild &B, hipStream_t s) {
    B.ntiles = (B.n + kXTile - 1) / kXTile;
    B.tcnt = c->x_tcnt;
    B.tbyt = c->x_tbyt;
    if (B.ntiles) hipLaunchKernelGGL(k_xbtile, dim3((B.ntiles + kXbTiles - 1) / kXbTiles), dim3(kXTile), 0, s, B);
    hipLaunchKernelGGL(k_xbscan, dim3(B.world), dim3(1024), 0, s, B);    // n = 0: zero counts
    if (B.ntiles) hipLaunchKernelGGL(k_xbuild, dim3(B.ntiles), dim3(kXTile), 0, s, B);   // lanes per frame: per tile
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
    int rc = xbuild_scratch(c);
    if (rc != FCGPU_OK) return rc;
    XBuild B{};
    B.arena = d_arena;
    B.desc = d_desc;
    B.verdict = d_verdict;
    B.n = n;
    B.world = world;
    B.rank = rank;
    B.seg_n = d_seg_n;
    B.seg_bytes = reinterpret_cast<unsigned long long *>(d_seg_bytes);
    B.meta = reinterpret_cast<uint4 *>(d_meta);
    B.send = d_send;
    B.send_cap = send_cap;
    return xbuild_launch(c, B, static_cast<hipStream_t>(stream));
}

int fcgpu_exchange_build_fixed(fcgpu_ctx *c, const uint8_t *d_arena, const uint32_t *d_desc,
                               const uint16_t *d_verdict, uint32_t n, uint32_t world, uint32_t rank,
                               uint32_t seg_recs, uint64_t seg_bytes, fcgpu_xmeta *d_meta, uint8_t *d_send,
                               void *stream) {
    if (!c) return FCGPU_EINVAL;
    if (world == 0 || world > FCGPU_MAX_PORTS)
        return fail(c, FCGPU_EINVAL, "fcgpu_exchange_build_fixed: world must be 1..64");
    if (n > c->max_batch)
        return fail(c, FCGPU_ENOMEM, "fcgpu_exchange_build_fixed: batch larger than the context's max_batch");
    if (seg_recs == 0 || seg_recs > 0x7fffffffu / world || seg_bytes == 0 || (seg_bytes & 15) ||
        (uint64_t)world * seg_bytes > 0xffffffffull - 256)
        return fail(c, FCGPU_EINVAL, "fcgpu_exchange_build_fixed: capacities (seg_bytes a multiple of 16, "
                                     "world x seg_bytes below 4 GiB)");
    if (!d_meta || !d_send || (n && (!d_arena || !d_desc || !d_verdict)))
        return fail(c, FCGPU_EINVAL, "fcgpu_exchange_build_fixed: null buffer");
    HIPCHK(c, hipSetDevice(c->device));
    int rc = xbuild_scratch(c);
    if (rc != FCGPU_OK) return rc;
    XBuild B{};
    B.arena = d_arena;
    B.desc = d_desc;
    B.verdict = d_verdict;
    B.n = n;
    B.world = world;
    B.rank = rank;
    B.seg_n = c->x_segn;
    B.seg_bytes = c->x_segb;
    B.meta = reinterpret_cast<uint4 *>(d_meta);
    B.send = d_send;
    B.send_cap = (uint64_t)world * seg_bytes;
    B.fix_recs = seg_recs;
    B.fix_bytes = seg_bytes;
    return xbuild_launch(c, B, static_cast<hipStream_t>(stream));
}

int fcgpu_exchange_unpack_fixed(fcgpu_ctx *c, const fcgpu_xmeta *d_rmeta, uint32_t world, uint32_t seg_recs,
                                uint64_t seg_bytes, uint32_t *d_desc, uint32_t *d_count, uint32_t *d_stall,
                                uint64_t *d_total, uint32_t step, void *stream) {
    if (!c) return FCGPU_EINVAL;
    if (world == 0 || world > FCGPU_MAX_PORTS)
        return fail(c, FCGPU_EINVAL, "fcgpu_exchange_unpack_fixed: world must be 1..64");
    if (seg_recs == 0 || seg_recs > 0x7fffffffu / world || (uint64_t)world * seg_bytes > 0xffffffffull - 256)
        return fail(c, FCGPU_EINVAL, "fcgpu_exchange_unpack_fixed: capacities");
    if (!d_rmeta || !d_desc || !d_count || !d_stall || step == 0)
        return fail(c, FCGPU_EINVAL, "fcgpu_exchange_unpack_fixed: null buffer or step 0");
    HIPCHK(c, hipSetDevice(c->device));
    XUnpackFixed U{};
    U.meta = reinterpret_cast<const uint4 *>(d_rmeta);
    U.desc = d_desc;
    U.world = world;
    U.recs = seg_recs;
    U.bytes = seg_bytes;
    U.count = d_count;
    U.stall = d_stall;
    U.total = reinterpret_cast<unsigned long long *>(d_total);
    U.step = step;
    hipLaunchKernelGGL(k_xunpack_fixed, dim3((seg_recs + kXThreads - 1) / kXThreads, world), dim3(kXThreads), 0,
                       static_cast<hipStream_t>(stream), U);
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
