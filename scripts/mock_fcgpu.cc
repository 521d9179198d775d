// mock_fcgpu.cc -- profiling aid, not product code and never loaded by the
// product path, the tests or bench.py: a host-only stand-in for the handful
// of libfcgpu.so entry points the element harness (libfcclick) calls, so the
// element's HOST work per packet (staging, annotation write-back, relinking)
// can be timed and A/B'd on a machine without a GPU. Every block submission
// "completes" at once with a fixed C2-like result (every packet valid, one
// output, the identity tile partition); no packet is checked. With the mock
// the element's rate is its host-side ceiling.
//
// scripts/mock_element.sh builds it (libfcgpu_mock.so), the element harness
// linked against it (libfcclick_mock.so) and scripts/mock_element_bench.cc.
#include <stdlib.h>
#include <string.h>

#include <string>

#include "fastclick_gpu.h"

struct fcgpu_ctx {
    fcgpu_cfg cfg;
    uint32_t max_batch;
    uint64_t count = 0;
    const void *filled[4] = {};   // result blocks already holding the fixed result for filled_n[k] packets
    uint32_t filled_n[4] = {};
};

namespace {
std::string g_err = "mock";
constexpr uint32_t kTile = 256;
}

extern "C" {

void fcgpu_default_cfg(fcgpu_cfg *c) {
    memset(c, 0, sizeof(*c));
    c->size = sizeof(fcgpu_cfg);
    c->check_mode = FCGPU_CHECK_IP4;
    c->hash_mode = FCGPU_HASH_FLOWID;
    c->nports = 1;
    c->hs_length = 1;
    c->nbad6 = 1;
    c->l4_checksum = 1;
    c->ttl_multicast = 1;
    memset(c->bad6[0], 0xff, 16);
}
const char *fcgpu_last_error(fcgpu_ctx *) { return g_err.c_str(); }
int fcgpu_open(int, uint32_t max_batch, fcgpu_ctx **out) {
    *out = new fcgpu_ctx();
    (*out)->max_batch = max_batch;
    fcgpu_default_cfg(&(*out)->cfg);
    return FCGPU_OK;
}
void fcgpu_close(fcgpu_ctx *c) { delete c; }
int fcgpu_configure(fcgpu_ctx *c, const fcgpu_cfg *cfg) {
    c->cfg = *cfg;
    return FCGPU_OK;
}
int fcgpu_span_mode(fcgpu_ctx *, uint32_t) { return FCGPU_OK; }
// MOCK_ZEROCOPY=1: report zero-copy (the element's BATCH auto then stages
// 4096-packet batches, as with >= 4 threads on a real GPU)
int fcgpu_span_zerocopy_active(const fcgpu_ctx *) {
    const char *e = getenv("MOCK_ZEROCOPY");
    return e && *e == '1';
}
void *fcgpu_host_alloc(size_t bytes) { return aligned_alloc(4096, (bytes + 4095) & ~(size_t)4095); }
void fcgpu_host_free(void *p) { free(p); }
int fcgpu_block_layout_for(const fcgpu_ctx *c, uint32_t n, uint32_t outputs, uint32_t, fcgpu_block_layout *L) {
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
int fcgpu_span_reserve(fcgpu_ctx *, size_t, uint32_t, uint32_t) { return FCGPU_OK; }
// every packet valid, on output 0, the tile partition the identity
int fcgpu_span_submit_block(fcgpu_ctx *c, uint32_t, const void *h_in, size_t, size_t desc_off, size_t,
                            uint32_t n, void *h_out, uint32_t outputs, uint32_t partition) {
    c->count += n;
    // the element never writes its result blocks: a block that already holds
    // the fixed result for n packets is left as is, so the mock costs the
    // calling thread nothing per packet in steady state
    // one entry per block: a block refilled for another n is re-keyed (a
    // stale entry for the old n would skip a later refill)
    int slot = -1;
    for (int k = 0; k < 4 && slot < 0; ++k)
        if (c->filled[k] == h_out) slot = k;
    if (slot >= 0 && c->filled_n[slot] == n) return FCGPU_OK;
    for (int k = 0; k < 4 && slot < 0; ++k)
        if (!c->filled[k]) slot = k;
    if (slot < 0) slot = 3;
    c->filled[slot] = h_out;
    c->filled_n[slot] = n;
    fcgpu_block_layout L;
    fcgpu_block_layout_for(c, n, outputs, partition, &L);
    uint8_t *o = static_cast<uint8_t *>(h_out);
    const uint32_t *desc = reinterpret_cast<const uint32_t *>(static_cast<const uint8_t *>(h_in) + desc_off);
    const uint32_t nb = c->cfg.nports + 1;
    for (uint32_t i = 0; i < n; ++i) {
        if (L.verdict != FCGPU_OUT_ABSENT) ((uint16_t *)(o + L.verdict))[i] = FCGPU_R_OK;
        if (L.hash != FCGPU_OUT_ABSENT) ((uint32_t *)(o + L.hash))[i] = 0x9e3779b1u * (i + 1);
        const uint32_t len = (outputs & FCGPU_SUBMIT_DESC32) ? desc[i] >> 16 : desc[2 * i + 1];
        if (L.anno != FCGPU_OUT_ABSENT && (outputs & FCGPU_OUT_ANNO8)) {
            fcgpu_anno8 &a = ((fcgpu_anno8 *)(o + L.anno))[i];
            a.dst_ip = 0x0200000au;
            a.length = (uint16_t)len;
            a.nh = (uint8_t)c->cfg.offset;
            a.thl = 20;
        } else if (L.anno != FCGPU_OUT_ABSENT) {
            fcgpu_anno &a = ((fcgpu_anno *)(o + L.anno))[i];
            memset(&a, 0, sizeof a);
            a.dst_ip = 0x0200000au;
            a.length = (uint16_t)len;
            a.nh = (uint16_t)c->cfg.offset;
            a.th = (uint16_t)(c->cfg.offset + 20);
            a.ipver = 4;
        }
        if (L.tile_perm != FCGPU_OUT_ABSENT) ((uint8_t *)(o + L.tile_perm))[i] = (uint8_t)(i % kTile);
        if (L.perm != FCGPU_OUT_ABSENT) ((uint32_t *)(o + L.perm))[i] = i;
    }
    if (L.tile_count != FCGPU_OUT_ABSENT) {
        const uint32_t tiles = (n + kTile - 1) / kTile;
        uint16_t *tc = (uint16_t *)(o + L.tile_count);
        memset(tc, 0, 2ull * nb * tiles);
        for (uint32_t t = 0; t < tiles; ++t) tc[(size_t)t * nb] = (uint16_t)(t + 1 < tiles ? kTile : n - t * kTile);
    }
    if (L.port_start != FCGPU_OUT_ABSENT) {
        uint32_t *ps = (uint32_t *)(o + L.port_start);
        ps[0] = 0;
        for (uint32_t p = 1; p <= nb; ++p) ps[p] = n;
    }
    return FCGPU_OK;
}
int fcgpu_span_wait(fcgpu_ctx *, uint32_t) { return FCGPU_OK; }
int fcgpu_read_counters(fcgpu_ctx *c, uint64_t *out, int n) {
    memset(out, 0, sizeof(uint64_t) * (size_t)n);
    if (n > FCGPU_CTR_COUNT) out[FCGPU_CTR_COUNT] = c->count;
    return FCGPU_OK;
}
int fcgpu_set_program(fcgpu_ctx *, uint32_t, const fcgpu_step *, uint32_t, int32_t) { return FCGPU_OK; }
int fcgpu_program_jit(fcgpu_ctx *, int) { return FCGPU_OK; }
int fcgpu_flow_configure(fcgpu_ctx *, const fcgpu_flow_config *) { return FCGPU_OK; }
int fcgpu_flow_count(fcgpu_ctx *, uint32_t *n) { *n = 0; return FCGPU_OK; }
int fcgpu_flow_maintain(fcgpu_ctx *, uint32_t, void *) { return FCGPU_OK; }
int fcgpu_flow_set_time(fcgpu_ctx *, uint32_t) { return FCGPU_OK; }
int fcgpu_flow_stats(fcgpu_ctx *, fcgpu_flow_stat *st) { memset(st, 0, sizeof *st); return FCGPU_OK; }
int fcgpu_set_lb_table(fcgpu_ctx *, const uint8_t *, uint32_t) { return FCGPU_OK; }
int fcgpu_lb_hash_ring(uint32_t nsel, uint32_t size, uint8_t *out) {
    for (uint32_t i = 0; i < size; ++i) out[i] = (uint8_t)(nsel ? i % nsel : 0);
    return FCGPU_OK;
}

}  // extern "C"
